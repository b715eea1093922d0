"""Host orchestration of one batched element op (the body of the reference's
UnsafeArray::initiate_batch_op / initiate_batch_fetch_op_2 /
initiate_batch_result_op_2, src/array/unsafe/operations.rs:290-477).

1 PE (local lamellae): the reference never serialises (every AM takes the
`dst == src` shortcut, active_messaging/registered_active_message.rs:150-154),
so the records go straight to the apply kernel: at one PE a global index *is*
the local offset (Block, Cyclic and sub-arrays alike), bounds-checked on the
device.

N PEs (one per GPU): one collective C-ABI call, lmr_batch_exchange, replaces
the shmem lamellae (pack by owner PE -> header all-to-all -> all-to-all-v of
indices and values over RCCL/xGMI -> staged apply at the owner -> reverse
all-to-all-v of results -> scatter into input order,
operations/handle.rs:315-317), chunked and pipelined inside the library.
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

# Large 1-PE batches are deferred: staged into the context's open session and applied with the
# batches issued after them in one shard sweep, at the next flush point (a handle's block(),
# wait_all, reading the array, any other device call). LAMELLAR_DEFER=0 applies each at once.
# The reference consumes a batch's input when the batch is built (the pack copies it into op
# buffers before batch_* returns, unsafe/operations.rs:663-811; a Vec input is moved in), so a
# caller may change its own buffers right after spawn(). A deferred batch whose input is the
# caller's device tensor (borrowed) is therefore partitioned at spawn, in stream order
# (lmr_stage_flush): its records are in the library's workspace before any later work on the
# stream, and only the shard sweep is shared. Inputs the library made itself (host sequences,
# converted dtypes) or that the caller hands over with Owned(...) -- Rust's by-value Vec input --
# stay with the session until it is applied, so consecutive batches also share the partition.
_DEFER = os.environ.get("LAMELLAR_DEFER", "1") != "0"
_DEFER_MIN = 65536


class Owned:
    """An op input handed over to the library (the reference's by-value `Vec<T>` OpInput,
    src/array/operations.rs:435-585): the caller does not modify the tensor until the batch has
    been applied (its handle's block(), wait_all(), or any read of the array)."""

    __slots__ = ("value",)

    def __init__(self, value):
        self.value = value


def _unwrap(x):
    return (x.value, True) if isinstance(x, Owned) else (x, False)


def _same_storage(a, b):
    return isinstance(b, torch.Tensor) and a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()


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
    """OpInput<usize>: scalar -> (True, int, 1, False); sequence -> (False, int64 tensor, len,
    borrowed). `borrowed`: the tensor is the caller's own device storage (not Owned)."""
    x, owned = _unwrap(x)
    if _is_scalar(x):
        return True, int(x), 1, False
    if isinstance(x, torch.Tensor):
        t = x.reshape(-1)
        if t.dtype != torch.int64:
            t = t.to(torch.int64)
        t = t.to(k.device) if t.device != k.device else t
        t = t.contiguous()
        return False, t, int(t.numel()), (not owned) and _same_storage(t, x)
    a = np.asarray(x)
    if a.size == 0:
        return False, k.empty(0, torch.int64), 0, False
    a = a.reshape(-1)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    else:
        a = a.astype(np.int64)
    return False, torch.from_numpy(np.ascontiguousarray(a)).to(k.device), int(a.size), False


def value_input(k, dt: DType, x):
    """OpInput<T>: scalar -> (True, bits, 1, False); sequence -> (False, storage tensor, len,
    borrowed)."""
    x, owned = _unwrap(x)
    if _is_scalar(x):
        return True, dt.to_bits(x), 1, False
    if isinstance(x, torch.Tensor):
        t = x.reshape(-1)
        if t.dtype != dt.torch:
            if t.element_size() == dt.bytes and not t.is_floating_point() and not dt.is_float:
                t = t.view(dt.torch)          # same-width integer: reinterpret the bits
            else:
                t = _np_to_storage(t.cpu().numpy(), dt)
        t = t.to(k.device) if t.device != k.device else t
        t = t.contiguous()
        return False, t, int(t.numel()), (not owned) and _same_storage(t, x)
    a = np.asarray(x).reshape(-1)
    if a.size == 0:
        return False, k.empty(0, dt.torch), 0, False
    return False, _np_to_storage(a, dt).to(k.device), int(a.size), False


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
    i_scalar, idx, i_len, i_borrowed = index_input(k, index)
    v_scalar, vals, v_len, v_borrowed = value_input(k, dt, val)
    if i_len > 1 and v_len > 1 and i_len != v_len:
        raise LamellarError(LmrStatus.LENGTH, f"{i_len} indices vs {v_len} values")
    n = 0 if (i_len == 0 or v_len == 0) else max(i_len, v_len)   # "no vals no indices" :345-347
    results = k.empty(n, dt.torch) if ret != BatchReturnType.None_ else None
    ok = k.empty(n, torch.uint8) if ret == BatchReturnType.Result else None
    if team.num_pes() > 1 or _FORCE_EXCHANGE:
        _distributed(arr, k, dt, op, i_scalar, idx, i_len, v_scalar, vals, v_len, results, ok, cmp_bits, eps_bits)
    elif n:
        _local(arr, k, dt, op, i_scalar, idx, v_scalar, vals, n, i_len == 1 and v_len > 1, results, ok,
               cmp_bits, eps_bits, i_borrowed or v_borrowed)
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


def _local(arr, k, dt, op, i_scalar, idx, v_scalar, vals, n, mvsi, results, ok, cmp_bits, eps_bits,
           borrowed=False):
    shard, slen = arr._shard_view(), arr.num_elems_local()
    if mvsi:
        _, off = _host_map(arr, idx)
        k.apply_mvsi(shard, slen, arr.kind, dt, op, vals, n, off, results, ok, cmp_bits, eps_bits)
        return
    if i_scalar:
        idx = torch.tensor([idx], dtype=torch.int64, device=k.device)
    if _DEFER and n >= _DEFER_MIN and getattr(k, "defer_soa", None) is not None:
        k.defer_soa(shard, slen, arr.kind, dt, op, idx, 8, None if v_scalar else vals,
                    vals if v_scalar else 0, n, results, ok, cmp_bits, eps_bits, borrowed=borrowed)
        return
    k.apply_soa(shard, slen, arr.kind, dt, op, idx, 8, None if v_scalar else vals,
                vals if v_scalar else 0, n, results, ok, cmp_bits, eps_bits)


def _distributed(arr, k, dt, op, i_scalar, idx, i_len, v_scalar, vals, v_len, results, ok, cmp_bits, eps_bits):
    """One collective lmr_batch_exchange: pack by owner PE ->
    header all-to-all -> all-to-all-v of indices and values -> the owner stages
    every arriving stream and applies them in one shard sweep -> reverse
    all-to-all-v of results -> scatter into input order, chunked and pipelined
    inside the library (include/lamellar_gpu_ops.h, exchange section).

    Collective: every PE issues the same sequence of batch calls; a PE with an
    empty batch still takes part (others may send it records)."""
    team = arr.team
    m = 0 if (i_len == 0 or v_len == 0) else max(i_len, v_len)
    expect = 0 if (i_scalar and v_len > 1) else m + m // 8 + (1 << 16)   # about what this PE sends
    # (the shard view without a flush: batch_exchange applies or continues a deferred session itself)
    k.batch_exchange(team.transport(), arr.layout, arr._shard_view(), arr.num_elems_local(), arr.kind, dt, op,
                     None if i_scalar else idx, idx if i_scalar else 0, i_len,
                     None if v_scalar else vals, vals if v_scalar else 0, v_len,
                     results, ok, cmp_bits, eps_bits, expect=expect)
