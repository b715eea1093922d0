"""Host orchestration of one batched element op (the body of the reference's
UnsafeArray::initiate_batch_op / initiate_batch_fetch_op_2 /
initiate_batch_result_op_2, src/array/unsafe/operations.rs:290-477).

1 PE (local lamellae): the reference never serialises (every AM takes the
`dst == src` shortcut, active_messaging/registered_active_message.rs:150-154),
so the records go straight to the apply kernel: at one PE a global index *is*
the local offset (Block, Cyclic and sub-arrays alike), bounds-checked on the
device.

N PEs (one per GPU): a collective step replaces the shmem lamellae:
  lmr_pack (device, stable by destination PE, IndexSize-narrowed offsets)
  -> header all-to-all (per destination: count, MVSI index, scalar value)
  -> all-to-all-v of indices and values (RCCL over xGMI)
  -> apply of every received segment (device)
  -> [fetch / result ops] reverse all-to-all-v of results + lmr_scatter_results
     back into input order (operations/handle.rs:315-317).
Every PE must issue the same sequence of batch calls (a PE with nothing to
send passes an empty batch): the exchange is collective where the reference's
AMs are one-sided.
"""
from __future__ import annotations

import numbers
import os

import numpy as np
import torch

from .kernels import LamellarError
from .types import RET_KIND, BatchReturnType, DType, LmrStatus, op_supported


# Route 1-PE batches through the exchange step too (rehearses the RCCL calls of
# the multi-GPU path on a one-GPU box); off by default.
_FORCE_EXCHANGE = os.environ.get("LAMELLAR_FORCE_EXCHANGE", "0") == "1"


class BatchResult:
    """Results of a fetch / result batch: values (and Ok flags) in input order."""

    def __init__(self, vals, ok, dt: DType, ret):
        self.vals = vals     # torch tensor (storage dtype) or None
        self.ok = ok         # torch uint8 tensor (Result ops) or None
        self.dt = dt
        self.ret = ret

    def numpy(self):
        v = self.vals.cpu().numpy().view(self.dt.np) if self.vals is not None else None
        if self.ret == BatchReturnType.Result:
            return v, self.ok.cpu().numpy().astype(bool)
        return v

    def __len__(self):
        return 0 if self.vals is None else int(self.vals.numel())


def _is_scalar(x):
    return isinstance(x, (numbers.Number, np.generic)) or (isinstance(x, np.ndarray) and x.ndim == 0)


def index_input(k, x):
    """OpInput<usize>: scalar -> (True, int, 1); sequence -> (False, int64 tensor, len)."""
    if _is_scalar(x):
        return True, int(x), 1
    if isinstance(x, torch.Tensor):
        t = x.reshape(-1)
        if t.dtype != torch.int64:
            t = t.to(torch.int64)
        t = t.to(k.device) if t.device != k.device else t
        return False, t.contiguous(), int(t.numel())
    a = np.asarray(x)
    if a.size == 0:
        return False, k.empty(0, torch.int64), 0
    a = a.reshape(-1)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    else:
        a = a.astype(np.int64)
    return False, torch.from_numpy(np.ascontiguousarray(a)).to(k.device), int(a.size)


def value_input(k, dt: DType, x):
    """OpInput<T>: scalar -> (True, bits, 1); sequence -> (False, storage tensor, len)."""
    if _is_scalar(x):
        return True, dt.to_bits(x), 1
    if isinstance(x, torch.Tensor):
        t = x.reshape(-1)
        if t.dtype != dt.torch:
            if t.element_size() == dt.bytes and not t.is_floating_point() and not dt.is_float:
                t = t.view(dt.torch)          # same-width integer: reinterpret the bits
            else:
                t = _np_to_storage(t.cpu().numpy(), dt)
        t = t.to(k.device) if t.device != k.device else t
        return False, t.contiguous(), int(t.numel())
    a = np.asarray(x).reshape(-1)
    if a.size == 0:
        return False, k.empty(0, dt.torch), 0
    return False, _np_to_storage(a, dt).to(k.device), int(a.size)


_STORAGE_NP = {1: np.int8, 2: np.int16, 4: np.int32, 8: np.int64}


def _np_to_storage(a: np.ndarray, dt: DType) -> torch.Tensor:
    v = np.ascontiguousarray(a.astype(dt.np))
    if dt.is_float:
        return torch.from_numpy(v)
    if dt.torch_name == "uint8":
        return torch.from_numpy(v.view(np.uint8))
    return torch.from_numpy(v.view(_STORAGE_NP[dt.bytes]))


def run_batch(arr, op, index, val, current=None, eps=None) -> BatchResult:
    """Apply `op` for every (index, value) pair; returns results in input order."""
    team = arr.team
    k = team.kernels
    dt = arr.dtype
    if not op_supported(arr.kind, dt, op):
        raise LamellarError(LmrStatus.UNSUPPORTED, f"{op!r} on {type(arr).__name__}<{dt.name}>")
    ret = RET_KIND[op]
    cmp_bits = dt.to_bits(current) if current is not None else 0
    eps_bits = dt.to_bits(eps) if eps is not None else 0
    i_scalar, idx, i_len = index_input(k, index)
    v_scalar, vals, v_len = value_input(k, dt, val)
    if i_len == 0 or v_len == 0:                        # "no vals no indices" :345-347
        return BatchResult(k.empty(0, dt.torch) if ret else None,
                           k.empty(0, torch.uint8) if ret == BatchReturnType.Result else None, dt, ret)
    if i_len > 1 and v_len > 1 and i_len != v_len:
        raise LamellarError(LmrStatus.LENGTH, f"{i_len} indices vs {v_len} values")
    n = max(i_len, v_len)
    results = k.empty(n, dt.torch) if ret != BatchReturnType.None_ else None
    ok = k.empty(n, torch.uint8) if ret == BatchReturnType.Result else None
    mvsi = (i_len == 1 and v_len > 1)
    if team.num_pes() == 1 and not _FORCE_EXCHANGE:
        _local(arr, k, dt, op, i_scalar, idx, v_scalar, vals, n, mvsi, results, ok, cmp_bits, eps_bits)
    else:
        _distributed(arr, k, dt, op, ret, i_scalar, idx, v_scalar, vals, n, mvsi, results, ok,
                     cmp_bits, eps_bits)
    return BatchResult(results, ok, dt, ret)


def _host_map(arr, g):
    from . import _capi
    import ctypes
    pe, off = ctypes.c_uint64(0), ctypes.c_uint64(0)
    okm = _capi.lib().lmr_pe_and_offset(ctypes.byref(arr.layout), int(g) & 0xFFFFFFFFFFFFFFFF,
                                        ctypes.byref(pe), ctypes.byref(off))
    if not okm:
        raise LamellarError(LmrStatus.OOB, f"Index: {g} out of bounds for array of len: {arr.len()}")
    return pe.value, off.value


def _local(arr, k, dt, op, i_scalar, idx, v_scalar, vals, n, mvsi, results, ok, cmp_bits, eps_bits):
    shard, slen = arr.local_shard(), arr.num_elems_local()
    if mvsi:
        _, off = _host_map(arr, idx)
        k.apply_mvsi(shard, slen, arr.kind, dt, op, vals, n, off, results, ok, cmp_bits, eps_bits)
        return
    if i_scalar:
        idx = torch.tensor([idx], dtype=torch.int64, device=k.device)
    k.apply_soa(shard, slen, arr.kind, dt, op, idx, 8, None if v_scalar else vals,
                vals if v_scalar else 0, n, results, ok, cmp_bits, eps_bits)


def _distributed(arr, k, dt, op, ret, i_scalar, idx, v_scalar, vals, n, mvsi, results, ok,
                 cmp_bits, eps_bits):
    team = arr.team
    npes = team.num_pes()
    iw = arr.index_size()
    eb = dt.bytes
    header = torch.zeros(npes, 4, dtype=torch.int64)
    # ---- pack (sender side) ----
    if mvsi:
        pe, off = _host_map(arr, idx)
        header[pe, 0] = n
        header[:, 1] = -1
        header[pe, 1] = off
        send_idx = k.empty(0, torch.uint8)
        send_vals = vals.view(torch.uint8) if vals.dtype != torch.uint8 else vals
        pos = None
    else:
        if i_scalar:
            idx = torch.tensor([idx], dtype=torch.int64, device=k.device)
        m = int(idx.numel())
        send_idx, send_vals, pos, counts_t = k.pack(arr.layout, idx, m, None if v_scalar else vals, dt, iw)
        header[:, 0] = counts_t.cpu()
        header[:, 1] = -1
        if v_scalar:
            header[:, 2] = 1
            header[:, 3] = torch.tensor(np.array([vals & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64).view(np.int64))
        if send_vals is None:
            send_vals = k.empty(0, torch.uint8)
    send_counts = header[:, 0].tolist()
    # ---- exchange (collective) ----
    rh = team.alltoall_header(header)
    recv_counts = rh[:, 0].tolist()
    idx_send_splits = [c * iw if header[p, 1] < 0 else 0 for p, c in enumerate(send_counts)]
    idx_recv_splits = [c * iw if rh[p, 1] < 0 else 0 for p, c in enumerate(recv_counts)]
    val_send_splits = [0 if header[p, 2] else c * eb for p, c in enumerate(send_counts)]
    val_recv_splits = [0 if rh[p, 2] else c * eb for p, c in enumerate(recv_counts)]
    r_idx = team.alltoallv(send_idx, idx_send_splits, idx_recv_splits)
    r_vals = team.alltoallv(send_vals, val_send_splits, val_recv_splits)
    # ---- apply every received segment ----
    total_recv = int(sum(recv_counts))
    r_res = k.empty(total_recv * eb, torch.uint8) if ret != BatchReturnType.None_ else None
    r_ok = k.empty(total_recv, torch.uint8) if ret == BatchReturnType.Result else None
    shard, slen = arr.local_shard(), arr.num_elems_local()
    io = vo = ro = 0
    for s in range(npes):
        c = int(recv_counts[s])
        if c == 0:
            continue
        seg_res = r_res[ro * eb:(ro + c) * eb] if r_res is not None else None
        seg_ok = r_ok[ro:ro + c] if r_ok is not None else None
        if rh[s, 1] >= 0:
            k.apply_mvsi(shard, slen, arr.kind, dt, op, r_vals[vo:vo + c * eb], c, int(rh[s, 1]),
                         seg_res, seg_ok, cmp_bits, eps_bits)
            vo += c * eb
        else:
            seg_idx = r_idx[io:io + c * iw]
            io += c * iw
            if rh[s, 2]:
                bits = int(np.array([int(rh[s, 3])], dtype=np.int64).view(np.uint64)[0])
                k.apply_soa(shard, slen, arr.kind, dt, op, seg_idx, iw, None, bits, c, seg_res, seg_ok,
                            cmp_bits, eps_bits)
            else:
                k.apply_soa(shard, slen, arr.kind, dt, op, seg_idx, iw, r_vals[vo:vo + c * eb], 0, c,
                            seg_res, seg_ok, cmp_bits, eps_bits)
                vo += c * eb
        ro += c
    if ret == BatchReturnType.None_:
        return
    # ---- results back to the sender, into input order ----
    back = team.alltoallv(r_res, [c * eb for c in recv_counts], [c * eb for c in send_counts])
    back_ok = team.alltoallv(r_ok, recv_counts, send_counts) if r_ok is not None else None
    nsent = int(sum(send_counts))
    if mvsi:
        results.view(torch.uint8)[:nsent * eb].copy_(back[:nsent * eb])
        if ok is not None:
            ok[:nsent].copy_(back_ok[:nsent])
    else:
        k.scatter_results(back, pos, nsent, eb, results, back_ok, ok)
