"""World / team: one PE per GPU, one process per PE.

Mirrors LamellarWorldBuilder / LamellarWorld (src/lamellar_world.rs:572-675)
only as far as the batched op path needs: PE count and id, a barrier, and the
exchange step that replaces the shmem lamellae's per-destination command
buffers (src/lamellae/command_queues.rs:725-807, 1395-1531) with all-to-all(v)
collectives — RCCL over xGMI on GPUs (torch.distributed backend "nccl" is RCCL
on ROCm), gloo for CPU-only rehearsal tests.

PE id / count come from the torchrun environment (RANK, WORLD_SIZE,
LOCAL_RANK) or from the reference's launcher variables (LAMELLAR_PE_ID,
LAMELLAR_NUM_PES, lamellar_run.sh:31-40).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return int(v)
    return default


_WIDE = {8: torch.int64, 4: torch.int32, 2: torch.int16, 1: torch.uint8}
_MAX_SPLIT = (1 << 31) - 1


def _widen(send, recv, send_splits, recv_splits, unit):
    """View 1-D uint8 buffers as `unit`-byte integers (unit 4 or 8: the record
    field width, the same on every PE, so all ranks agree on the element type)
    so per-peer element counts stay below 2^31 (RCCL/NCCL all-to-all-v counts
    are signed 32-bit); split sizes converted to elements."""
    ss = [int(x) for x in send_splits]
    rs = [int(x) for x in recv_splits]
    if unit in (4, 8) and send.dtype == torch.uint8 and recv.dtype == torch.uint8:
        if send.storage_offset() % unit:
            send = send.clone()
        send, recv = send.view(_WIDE[unit]), recv.view(_WIDE[unit])
        ss, rs = [x // unit for x in ss], [x // unit for x in rs]
    if max(ss + rs + [0]) > _MAX_SPLIT:
        raise ValueError("exchange split of %d elements exceeds 2^31 - 1; lower LAMELLAR_EXCHANGE_CHUNK"
                         % max(ss + rs))
    return send, recv, ss, rs


class _Done:
    """Work handle of an exchange that has already completed."""

    def wait(self):
        return True


class LamellarTeam:
    def __init__(self, num_pes, my_pe, device, kernels, group=None):
        self._num_pes = num_pes
        self._my_pe = my_pe
        self.device = device
        self.kernels = kernels
        self.group = group
        self.comm_device = device if (dist.is_initialized() and dist.get_backend(group) == "nccl") \
            else torch.device("cpu")

    def num_pes(self):
        return self._num_pes

    def my_pe(self):
        return self._my_pe

    def barrier(self):
        if self._num_pes > 1:
            if dist.get_backend(self.group) == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    # ---- exchange step (collective) ----
    def alltoall_header(self, send: torch.Tensor) -> torch.Tensor:
        """send: int64 [num_pes, k] (row p goes to PE p) -> recv int64 [num_pes, k]."""
        if not self._collective():
            return send.clone()
        s = send.to(self.comm_device).contiguous()
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s, group=self.group)
        return r.cpu()

    def alltoallv(self, send: torch.Tensor, send_splits, recv_splits, unit=1) -> torch.Tensor:
        """Byte / element all-to-all-v of a 1-D tensor with per-PE split sizes."""
        total = int(sum(recv_splits))
        if not self._collective():
            return send[:total].clone()
        dev = send.device
        s = send.to(self.comm_device).contiguous()
        r = torch.empty(total, dtype=send.dtype, device=self.comm_device)
        sw, rw, ss, rs = _widen(s, r, send_splits, recv_splits, unit)
        dist.all_to_all_single(rw, sw, output_split_sizes=rs, input_split_sizes=ss, group=self.group)
        return r.to(dev)

    def alltoallv_async(self, send: torch.Tensor, send_splits, recv_splits, unit=1):
        """Asynchronous alltoallv -> (recv tensor, work). work.wait() orders the
        caller's current stream after the transfer (RCCL) or blocks until it is
        done (gloo). The recv tensor lives on the comm device."""
        total = int(sum(recv_splits))
        if not self._collective():
            return send[:total].clone(), _Done()
        if send.device != self.comm_device:
            # host-side backend (gloo) with device tensors: synchronous round trip
            return self.alltoallv(send, send_splits, recv_splits, unit), _Done()
        r = torch.empty(total, dtype=send.dtype, device=self.comm_device)
        sw, rw, ss, rs = _widen(send.contiguous(), r, send_splits, recv_splits, unit)
        w = dist.all_to_all_single(rw, sw, output_split_sizes=rs, input_split_sizes=ss, group=self.group,
                                   async_op=True)
        return r, w

    def _collective(self):
        # a 1-PE world still goes through the collective when a process group
        # exists (LAMELLAR_FORCE_EXCHANGE rehearsal of the RCCL calls)
        return self._num_pes > 1 or (dist.is_available() and dist.is_initialized())

    def all_gather_object(self, obj):
        if self._num_pes == 1:
            return [obj]
        out = [None] * self._num_pes
        dist.all_gather_object(out, obj, group=self.group)
        return out


class LamellarWorld:
    def __init__(self, team: LamellarTeam):
        self._team = team

    def team(self):
        return self._team

    def num_pes(self):
        return self._team.num_pes()

    def my_pe(self):
        return self._team.my_pe()

    def barrier(self):
        self._team.barrier()

    def wait_all(self):
        self._team.kernels.synchronize()
        self._team.kernels.check_errors()

    def block_on(self, handle):
        return handle.block()


class LamellarWorldBuilder:
    """LamellarWorldBuilder::new().build() for the device op path."""

    def __init__(self):
        self._kernels_factory = None
        self._device = None
        self._strategy = None

    def with_kernels(self, factory):
        """Test hook: build with another kernels implementation (CPU rehearsal of
        the exchange logic). The product path always uses DeviceKernels."""
        self._kernels_factory = factory
        return self

    def with_device(self, device):
        self._device = torch.device(device)
        return self

    def with_strategy(self, strategy):
        self._strategy = strategy
        return self

    def build(self) -> LamellarWorld:
        from .kernels import DeviceKernels
        from .types import Strategy
        world_size = _env_int("WORLD_SIZE", "LAMELLAR_NUM_PES", default=1)
        rank = _env_int("RANK", "LAMELLAR_PE_ID", default=0)
        local_rank = _env_int("LOCAL_RANK", default=rank)
        if self._device is not None:
            device = self._device
        elif self._kernels_factory is None:
            if not torch.cuda.is_available():
                from .kernels import LamellarError
                from .types import LmrStatus
                raise LamellarError(LmrStatus.INVALID, "no HIP device visible; the op path is GPU-only")
            device = torch.device("cuda", local_rank % torch.cuda.device_count())
        else:
            device = torch.device("cpu")
        if device.type == "cuda":
            torch.cuda.set_device(device)
        group = None
        force = os.environ.get("LAMELLAR_FORCE_EXCHANGE", "0") == "1"
        if world_size > 1 or force:
            if not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", "29511")
                backend = os.environ.get("LAMELLAR_COMM_BACKEND") or \
                    ("nccl" if device.type == "cuda" else "gloo")
                kw = {"device_id": device} if backend == "nccl" else {}
                dist.init_process_group(backend, rank=rank, world_size=world_size, **kw)
            group = dist.group.WORLD
        if self._kernels_factory is not None:
            kernels = self._kernels_factory(device)
        else:
            strategy = self._strategy
            if strategy is None:
                strategy = {"auto": Strategy.Auto, "direct": Strategy.Direct,
                            "tiled": Strategy.Tiled}[os.environ.get("LAMELLAR_OP_STRATEGY", "auto")]
            kernels = DeviceKernels(device, strategy=strategy)
        team = LamellarTeam(world_size, rank, device, kernels, group)
        return LamellarWorld(team)
