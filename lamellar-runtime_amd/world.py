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

import ctypes
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
_LMR_E_HIP = 6


def _host_view(addr, nbytes):
    """uint8 tensor over nbytes of host memory at addr (no copy)."""
    if nbytes == 0:
        return torch.empty(0, dtype=torch.uint8)
    return torch.frombuffer((ctypes.c_uint8 * nbytes).from_address(addr), dtype=torch.uint8)


class HostTransport:
    """lmr_transport_t whose collectives run on a host (gloo) process group.

    host_buffers = 1: lmr_batch_exchange stages device data through pinned host
    memory around each callback, so the callbacks see host pointers. Used where
    the process group cannot carry device memory (LAMELLAR_COMM_BACKEND=gloo,
    CPU rehearsals). A callback that raises returns LMR_E_HIP to the library and
    the exception is re-raised by `raise_pending` after the C call returns."""

    def __init__(self, num_pes, my_pe, group):
        from . import _capi
        self.num_pes, self.my_pe, self.group = num_pes, my_pe, group
        self.error = None
        self.self_bytes = 0                                  # bytes this PE sent itself (tests)
        self._a2a = _capi.ALLTOALL_FN(self._alltoall)       # keep the thunks alive
        self._a2av = _capi.ALLTOALLV_FN(self._alltoallv)
        self.t = _capi.lmr_transport_t(num_pes, my_pe, 1, 0, None, self._a2a, self._a2av)

    @property
    def ptr(self):
        return ctypes.c_void_p(ctypes.addressof(self.t))

    def raise_pending(self):
        if self.error is not None:
            e, self.error = self.error, None
            raise e

    def _alltoall(self, _self, send, recv, nbytes, _stream):
        try:
            tot = int(nbytes) * self.num_pes
            s, r = _host_view(send, tot), _host_view(recv, tot)
            if tot:
                dist.all_to_all_single(r, s, group=self.group)
            return 0
        except Exception as e:  # noqa: BLE001 - handed back to the caller of the C entry point
            self.error = e
            return _LMR_E_HIP

    def _alltoallv(self, _self, send, sb, so, recv, rb, ro, unit, _stream):
        try:
            n = self.num_pes
            sb, so, rb, ro = ([int(a[p]) for p in range(n)] for a in (sb, so, rb, ro))
            # the library's splits are back to back (offsets are prefix sums)
            if any(so[p] != sum(sb[:p]) for p in range(n)) or any(ro[p] != sum(rb[:p]) for p in range(n)):
                raise ValueError("alltoallv splits are not contiguous")
            self.self_bytes += sb[self.my_pe]
            s, r = _host_view(send, sum(sb)), _host_view(recv, sum(rb))
            sw, rw, ss, rs = _widen(s, r, sb, rb, int(unit))
            dist.all_to_all_single(rw, sw, output_split_sizes=rs, input_split_sizes=ss, group=self.group)
            return 0
        except Exception as e:  # noqa: BLE001
            self.error = e
            return _LMR_E_HIP


class RcclTransport:
    """lmr_transport_rccl_create: RCCL grouped send/recv over xGMI on the library's
    streams. PE 0 makes the unique id and the process group broadcasts it."""

    def __init__(self, num_pes, my_pe, device, group):
        from . import _capi
        from .kernels import check
        lib = _capi.lib()
        uid = (ctypes.c_uint8 * 128)()
        if my_pe == 0:
            check(lib.lmr_rccl_unique_id(uid), "lmr_rccl_unique_id")
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0, group=group)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
        self.ptr = ctypes.c_void_p()
        check(lib.lmr_transport_rccl_create(uid, num_pes, my_pe, device.index or 0, ctypes.byref(self.ptr)),
              "lmr_transport_rccl_create")

    def raise_pending(self):
        pass

    def close(self):
        from . import _capi
        if self.ptr:
            _capi.lib().lmr_transport_rccl_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()


class PeerTransport:
    """lmr_transport_peer_create over a base transport (RCCL or host callbacks): the exchange
    pushes count-free records straight into the owners' IPC-mapped receive regions, with a
    /dev/shm mailbox for counts and flags (the reference's shmem heap, shmem_comm.rs:47-80);
    every other batch uses the base transport's collectives. PE 0 names the job's mailbox."""

    def __init__(self, base, num_pes, my_pe, device, group):
        import uuid
        from . import _capi
        from .kernels import check
        self.base = base
        obj = [uuid.uuid4().hex[:16] if my_pe == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        recs = int(os.environ.get("LAMELLAR_PEER_REGION_RECORDS", "0"))
        self.ptr = ctypes.c_void_p()
        check(_capi.lib().lmr_transport_peer_create(base.ptr, obj[0].encode(), recs, device.index or 0,
                                                     ctypes.byref(self.ptr)), "lmr_transport_peer_create")

    @property
    def self_bytes(self):
        return getattr(self.base, "self_bytes", -1)

    def stats(self):
        """(batches handshaken, chunks pushed) -- lmr_transport_peer_stats."""
        from . import _capi
        b, c = ctypes.c_uint64(), ctypes.c_uint64()
        _capi.lib().lmr_transport_peer_stats(self.ptr, ctypes.byref(b), ctypes.byref(c))
        return b.value, c.value

    def raise_pending(self):
        self.base.raise_pending()

    def close(self):
        from . import _capi
        if self.ptr:
            _capi.lib().lmr_transport_peer_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()
        if hasattr(self.base, "close"):
            self.base.close()


def _widen(send, recv, send_splits, recv_splits, unit):
    """View 1-D uint8 buffers as `unit`-byte integers (the record field width,
    the same on every PE, so all ranks agree on the element type) so per-peer
    element counts stay below 2^31 (all-to-all-v counts are signed 32-bit);
    split sizes converted to elements."""
    ss = [int(x) for x in send_splits]
    rs = [int(x) for x in recv_splits]
    if unit in (4, 8):                 # gloo has no 16-bit integer type; 2-byte splits stay bytes
        send, recv = send.view(_WIDE[unit]), recv.view(_WIDE[unit])
        ss, rs = [x // unit for x in ss], [x // unit for x in rs]
    if max(ss + rs + [0]) > _MAX_SPLIT:
        raise ValueError("exchange split of %d elements exceeds 2^31 - 1; lower LAMELLAR_EXCHANGE_CHUNK"
                         % max(ss + rs))
    return send, recv, ss, rs


class LamellarTeam:
    def __init__(self, num_pes, my_pe, device, kernels, group=None):
        self._num_pes = num_pes
        self._my_pe = my_pe
        self.device = device
        self.kernels = kernels
        self.group = group
        self._transport = None

    def num_pes(self):
        return self._num_pes

    def my_pe(self):
        return self._my_pe

    def barrier(self):
        flush = getattr(self.kernels, "flush", None)
        if flush is not None:
            flush()                           # batches deferred on this PE are applied first
        if self._num_pes > 1:
            if dist.get_backend(self.group) == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    # ---- exchange step (collective) ----
    def transport(self):
        """The lmr_transport_t of lmr_batch_exchange (made on first use, collective):
        RCCL when the process group is "nccl", host callbacks over the group otherwise;
        LAMELLAR_TRANSPORT=peer puts the peer-memory push transport over it."""
        if self._transport is None:
            if self.group is None:
                raise RuntimeError("the exchange needs a process group (num_pes > 1 or LAMELLAR_FORCE_EXCHANGE=1)")
            if dist.get_backend(self.group) == "nccl":
                t = RcclTransport(self._num_pes, self._my_pe, self.device, self.group)
            else:
                t = HostTransport(self._num_pes, self._my_pe, self.group)
            if os.environ.get("LAMELLAR_TRANSPORT", "") == "peer":
                t = PeerTransport(t, self._num_pes, self._my_pe, self.device, self.group)
            self._transport = t
        return self._transport

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
                            "tiled": Strategy.Tiled, "ordered": Strategy.Ordered}[os.environ.get("LAMELLAR_OP_STRATEGY", "auto")]
            kernels = DeviceKernels(device, strategy=strategy)
        team = LamellarTeam(world_size, rank, device, kernels, group)
        return LamellarWorld(team)
