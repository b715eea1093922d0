"""LamellarArray types and their op-builder API, over the device op path.

Mirrors the reference's user-facing surface for this path:
  - array kinds: UnsafeArray, AtomicArray (Native for integers, Generic for
    f32/f64, src/array/atomic.rs:28-41), LocalLockArray, GlobalLockArray,
    ReadOnlyArray; construction zero-fills every shard (src/array/unsafe.rs:178-274);
  - op builders with the reference's names and argument order
    (src/array/operations/{arithmetic,bitwise,access,compare_exchange,
    read_only,shift}.rs): add / batch_add / fetch_add / batch_fetch_add, ...;
  - lazy handles: nothing runs until spawn() / block(); a handle dropped
    without either never runs and warns (src/array/operations/handle.rs:19-46).

Values cross the API as Python / numpy scalars, numpy arrays, lists or torch
tensors; indices are global (usize). Batch results come back as device
tensors in input order (`.numpy()` on BatchResult for host copies).
"""
from __future__ import annotations

import ctypes
import warnings

import numpy as np
import torch

from . import _capi
from .engine import BatchResult, run_batch
from .kernels import LamellarError
from .types import (ArrayKind, ArrayOpCmd as Op, BatchReturnType, Distribution, LmrStatus,
                    dtype_of)


class Ok:
    __slots__ = ("value",)

    def __init__(self, v):
        self.value = v

    def is_ok(self):
        return True

    def is_err(self):
        return False

    def __eq__(self, o):
        return isinstance(o, Ok) and o.value == self.value

    def __repr__(self):
        return f"Ok({self.value!r})"


class Err(Ok):
    def is_ok(self):
        return False

    def is_err(self):
        return True

    def __eq__(self, o):
        return isinstance(o, Err) and o.value == self.value

    def __repr__(self):
        return f"Err({self.value!r})"


# ------------------------------------------------------------------ handles
class _Handle:
    def __init__(self, array, op, index, val, current=None, eps=None):
        self._array = array
        self._args = (op, index, val, current, eps)
        self._res = None
        self._launched = False

    def spawn(self):
        """Launch the op (enqueue on the device stream); returns self."""
        if not self._launched:
            self._launched = True
            op, index, val, cur, eps = self._args
            self._res = run_batch(self._array, op, index, val, cur, eps)
        return self

    def block(self):
        self.spawn()
        k = self._array.team.kernels
        k.synchronize()
        k.check_errors()
        return self._value()

    def _value(self):
        return None

    def __del__(self):
        if not getattr(self, "_launched", True):
            warnings.warn("a LamellarArray op handle was dropped without spawn()/block(): its ops "
                          "never run (reference: src/array/operations/handle.rs:39-46)",
                          RuntimeWarning, stacklevel=2)


class ArrayBatchOpHandle(_Handle):
    pass


class ArrayOpHandle(_Handle):
    pass


class ArrayFetchBatchOpHandle(_Handle):
    def _value(self):
        return self._res.vals


class ArrayResultBatchOpHandle(_Handle):
    def _value(self):
        return self._res


class ArrayFetchOpHandle(_Handle):
    def _value(self):
        return self._res.numpy()[0]


class ArrayResultOpHandle(_Handle):
    def _value(self):
        v, ok = self._res.numpy()
        return Ok(v[0]) if ok[0] else Err(v[0])


REDUCE_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3}    # lmr_reduce_op_t


def _reduce_combine(op, dt, a, b):
    """One step of the reference's reduction closures (impl/src/array_reduce.rs:283-319)
    in the element type: integers wrap, floats round as T."""
    x, y = np.array([a], dtype=dt.np), np.array([b], dtype=dt.np)
    with np.errstate(over="ignore", invalid="ignore"):
        if op == "sum":
            return (x + y)[0]
        if op == "prod":
            return (x * y)[0]
    if op == "max":
        return a if a > b else b
    return a if a < b else b


def _reduce_tree(op, dt, parts, lo, hi):
    """The cross-PE tree of the reduction AM (impl/src/array_reduce.rs:90-107):
    [lo, hi] splits at mid; None (an empty PE) is the identity."""
    if lo == hi:
        return parts[lo]
    mid = (lo + hi) // 2
    left = _reduce_tree(op, dt, parts, lo, mid)
    right = _reduce_tree(op, dt, parts, mid + 1, hi)
    if left is None:
        return right
    if right is None:
        return left
    return _reduce_combine(op, dt, left, right)


class ReduceHandle:
    """AmHandle<Option<T>> of UnsafeArray::reduce (src/array/unsafe.rs:1414-1557).
    Collective here (every PE calls it; every PE gets the value) where the
    reference's is one-sided."""

    def __init__(self, array, op):
        if op not in REDUCE_OPS:
            raise LamellarError(LmrStatus.UNSUPPORTED, f"unknown reduction {op!r} (sum, prod, max, min)")
        self._array, self._op = array, op

    def block(self):
        a = self._array
        k = a.team.kernels
        has, bits = k.reduce(a.local_data(), a.num_elems_local(), a.dtype, REDUCE_OPS[self._op])
        mine = a.dtype.from_bits(bits) if has else None
        parts = a.team.all_gather_object(mine)
        return _reduce_tree(self._op, a.dtype, parts, 0, len(parts) - 1)

    spawn = block


# ------------------------------------------------------------------ arrays
class LamellarArray:
    KIND = ArrayKind.Unsafe

    def __init__(self, team, array_size, distribution=Distribution.Block, dtype="usize",
                 _parent=None, _layout=None):
        self.team = team
        self.dtype = dtype_of(dtype)
        lib = _capi.lib()
        if _layout is None:
            L = _capi.lmr_layout_t()
            st = lib.lmr_layout_new(ctypes.byref(L), int(array_size), team.num_pes(), team.my_pe(),
                                    int(distribution))
            if st:
                raise LamellarError(st, "lmr_layout_new")
            self.layout = L
        else:
            self.layout = _layout
        self.kind = self._kind()
        if _parent is not None:
            self._data = _parent._data
            self._root_layout = _parent._root_layout
        else:
            full = self.layout
            if full.sub:   # array_size < num_pes: storage is the full array's
                root = _capi.lmr_layout_t()
                lib.lmr_layout_new(ctypes.byref(root), max(int(array_size), team.num_pes()),
                                   team.num_pes(), team.my_pe(), int(distribution))
            else:
                root = full
            self._root_layout = root
            n = int(lib.lmr_num_elems_pe(ctypes.byref(root), team.my_pe()))
            # +4 elements: 8/16-bit device RMWs CAS the containing 32-bit word
            self._data = torch.zeros(n + 4, dtype=self.dtype.torch, device=team.kernels.device)
        team.barrier()

    def _kind(self):
        return self.KIND

    @classmethod
    def new(cls, team, array_size, distribution=Distribution.Block, dtype="usize"):
        """`Array::<T>::new(team, len, dist)` — returns a handle; `.block()` gives the array."""
        class _New:
            def block(_self):
                return cls(team, array_size, distribution, dtype)
        return _New()

    # ---- layout ----
    def len(self):
        return int(self.layout.size)

    def __len__(self):
        return self.len()

    def num_pes(self):
        return self.team.num_pes()

    def my_pe(self):
        return self.team.my_pe()

    def num_elems_local(self):
        return int(_capi.lib().lmr_num_elems_pe(ctypes.byref(self.layout), self.team.my_pe()))

    def index_size(self):
        """IndexSize byte width (src/array/unsafe/operations.rs:56-75)."""
        return int(_capi.lib().lmr_index_size(ctypes.byref(self.layout)))

    def local_shard(self):
        """Device tensor of this PE's local slice (UnsafeArray::local_as_mut_slice), with every
        batch issued so far applied (stream-ordered)."""
        flush = getattr(self.team.kernels, "flush", None)
        if flush is not None:
            flush()
        return self._shard_view()

    def _shard_view(self):
        start = int(_capi.lib().lmr_local_slice_start(ctypes.byref(self.layout), self.team.my_pe()))
        n = self.num_elems_local()
        if n == 0:
            return self._data[:1]
        return self._data[start:start + n]

    def local_data(self):
        return self.local_shard()[: self.num_elems_local()]

    def sub_array(self, start, end=None):
        end = self.len() if end is None else end
        L = _capi.lmr_layout_t()
        st = _capi.lib().lmr_layout_sub(ctypes.byref(self.layout), int(start), int(end), ctypes.byref(L))
        if st:
            raise LamellarError(st, f"subregion range ({start}-{end}) exceeds size of array {self.len()}")
        a = object.__new__(type(self))
        a.team, a.dtype, a.layout, a.kind = self.team, self.dtype, L, self.kind
        a._data, a._root_layout = self._data, self._root_layout
        return a

    def _convert(self, cls):
        a = object.__new__(cls)
        a.team, a.dtype, a.layout = self.team, self.dtype, self.layout
        a._data, a._root_layout = self._data, self._root_layout
        a.kind = a._kind()
        return a

    def into_unsafe(self):
        return self._convert(UnsafeArray)

    def into_atomic(self):
        return self._convert(AtomicArray)

    def into_local_lock(self):
        return self._convert(LocalLockArray)

    def into_global_lock(self):
        return self._convert(GlobalLockArray)

    def into_read_only(self):
        return self._convert(ReadOnlyArray)

    # ---- collective helpers ----
    def barrier(self):
        self.team.barrier()

    def wait_all(self):
        self.team.kernels.synchronize()
        self.team.kernels.check_errors()

    def fill(self, value):
        """dist_iter_mut().for_each(|x| *x = value) on this PE's slice (no barrier)."""
        self.local_data().fill_(self.dtype.as_storage_scalar(value))
        return self

    def local_numpy(self):
        return self.local_data().cpu().numpy().view(self.dtype.np)

    def to_numpy(self):
        """Whole (sub)array in global order on every PE (collective; onesided_iter())."""
        self.team.kernels.synchronize()
        parts = self.team.all_gather_object(self.local_numpy())
        L = self.layout
        npes = self.team.num_pes()
        n = self.len()
        if L.distribution == Distribution.Block:
            return np.concatenate(parts)[:n] if parts else np.zeros(0, self.dtype.np)
        out = np.empty(n, dtype=self.dtype.np)
        i = np.arange(n, dtype=np.uint64)
        pe = ((i + np.uint64(L.offset)) % np.uint64(npes)).astype(np.int64)
        off = (i // np.uint64(npes)).astype(np.int64)
        for p in range(npes):
            m = pe == p
            out[m] = parts[p][off[m]]
        return out

    def print(self):
        print(f"{type(self).__name__}<{self.dtype.name}> pe {self.my_pe()}: {self.local_numpy()}")

    # ---- reductions (src/array/unsafe.rs:1414-1557) ----
    def reduce(self, op: str) -> ReduceHandle:
        """array.reduce("sum"|"prod"|"max"|"min").block() -> value, or None for an empty array."""
        return ReduceHandle(self, op)

    def sum(self) -> ReduceHandle:
        return self.reduce("sum")

    def prod(self) -> ReduceHandle:
        return self.reduce("prod")

    def max(self) -> ReduceHandle:
        return self.reduce("max")

    def min(self) -> ReduceHandle:
        return self.reduce("min")

    # ---- op plumbing ----
    def _batch(self, op, index, val, current=None, eps=None):
        rk = {BatchReturnType.None_: ArrayBatchOpHandle, BatchReturnType.Vals: ArrayFetchBatchOpHandle,
              BatchReturnType.Result: ArrayResultBatchOpHandle}
        from .types import RET_KIND
        return rk[RET_KIND[op]](self, op, index, val, current, eps)

    def _single(self, op, index, val, current=None, eps=None):
        rk = {BatchReturnType.None_: ArrayOpHandle, BatchReturnType.Vals: ArrayFetchOpHandle,
              BatchReturnType.Result: ArrayResultOpHandle}
        from .types import RET_KIND
        return rk[RET_KIND[op]](self, op, int(index), val, current, eps)

    def _dummy_val(self):
        # UnsafeArray::dummy_val (unsafe/operations.rs:274-287): loads carry an unused value
        return 0


class _ArithmeticOps:
    """ArithmeticOps (src/array/operations/arithmetic.rs:100-845)."""
    def add(self, index, val): return self._single(Op.Add, index, val)
    def batch_add(self, index, val): return self._batch(Op.Add, index, val)
    def fetch_add(self, index, val): return self._single(Op.FetchAdd, index, val)
    def batch_fetch_add(self, index, val): return self._batch(Op.FetchAdd, index, val)
    def sub(self, index, val): return self._single(Op.Sub, index, val)
    def batch_sub(self, index, val): return self._batch(Op.Sub, index, val)
    def fetch_sub(self, index, val): return self._single(Op.FetchSub, index, val)
    def batch_fetch_sub(self, index, val): return self._batch(Op.FetchSub, index, val)
    def mul(self, index, val): return self._single(Op.Mul, index, val)
    def batch_mul(self, index, val): return self._batch(Op.Mul, index, val)
    def fetch_mul(self, index, val): return self._single(Op.FetchMul, index, val)
    def batch_fetch_mul(self, index, val): return self._batch(Op.FetchMul, index, val)
    def div(self, index, val): return self._single(Op.Div, index, val)
    def batch_div(self, index, val): return self._batch(Op.Div, index, val)
    def fetch_div(self, index, val): return self._single(Op.FetchDiv, index, val)
    def batch_fetch_div(self, index, val): return self._batch(Op.FetchDiv, index, val)
    def rem(self, index, val): return self._single(Op.Rem, index, val)
    def batch_rem(self, index, val): return self._batch(Op.Rem, index, val)
    def fetch_rem(self, index, val): return self._single(Op.FetchRem, index, val)
    def batch_fetch_rem(self, index, val): return self._batch(Op.FetchRem, index, val)


class _BitWiseOps:
    """BitWiseOps (src/array/operations/bitwise.rs:87-535)."""
    def bit_and(self, index, val): return self._single(Op.And, index, val)
    def batch_bit_and(self, index, val): return self._batch(Op.And, index, val)
    def fetch_bit_and(self, index, val): return self._single(Op.FetchAnd, index, val)
    def batch_fetch_bit_and(self, index, val): return self._batch(Op.FetchAnd, index, val)
    def bit_or(self, index, val): return self._single(Op.Or, index, val)
    def batch_bit_or(self, index, val): return self._batch(Op.Or, index, val)
    def fetch_bit_or(self, index, val): return self._single(Op.FetchOr, index, val)
    def batch_fetch_bit_or(self, index, val): return self._batch(Op.FetchOr, index, val)
    def bit_xor(self, index, val): return self._single(Op.Xor, index, val)
    def batch_bit_xor(self, index, val): return self._batch(Op.Xor, index, val)
    def fetch_bit_xor(self, index, val): return self._single(Op.FetchXor, index, val)
    def batch_fetch_bit_xor(self, index, val): return self._batch(Op.FetchXor, index, val)


class _ShiftOps:
    """ShiftOps (src/array/operations/shift.rs)."""
    def shl(self, index, val): return self._single(Op.Shl, index, val)
    def batch_shl(self, index, val): return self._batch(Op.Shl, index, val)
    def fetch_shl(self, index, val): return self._single(Op.FetchShl, index, val)
    def batch_fetch_shl(self, index, val): return self._batch(Op.FetchShl, index, val)
    def shr(self, index, val): return self._single(Op.Shr, index, val)
    def batch_shr(self, index, val): return self._batch(Op.Shr, index, val)
    def fetch_shr(self, index, val): return self._single(Op.FetchShr, index, val)
    def batch_fetch_shr(self, index, val): return self._batch(Op.FetchShr, index, val)


class _AccessOps:
    """AccessOps (src/array/operations/access.rs:72-212)."""
    def store(self, index, val): return self._single(Op.Store, index, val)
    def batch_store(self, index, val): return self._batch(Op.Store, index, val)
    def swap(self, index, val): return self._single(Op.Swap, index, val)
    def batch_swap(self, index, val): return self._batch(Op.Swap, index, val)


class _ReadOnlyOps:
    """ReadOnlyOps (src/array/operations/read_only.rs:50-125)."""
    def load(self, index): return self._single(Op.Load, index, self._dummy_val())
    def batch_load(self, index): return self._batch(Op.Load, index, self._dummy_val())


class _CompareExchangeOps:
    """CompareExchangeOps / CompareExchangeEpsilonOps (operations/compare_exchange.rs:96-348)."""
    def compare_exchange(self, index, current, new):
        return self._single(Op.CompareExchange, index, new, current=current)

    def batch_compare_exchange(self, index, current, new):
        return self._batch(Op.CompareExchange, index, new, current=current)

    def compare_exchange_epsilon(self, index, current, new, eps):
        return self._single(Op.CompareExchangeEps, index, new, current=current, eps=eps)

    def batch_compare_exchange_epsilon(self, index, current, new, eps):
        return self._batch(Op.CompareExchangeEps, index, new, current=current, eps=eps)


class _AllOps(_ArithmeticOps, _BitWiseOps, _ShiftOps, _AccessOps, _ReadOnlyOps, _CompareExchangeOps):
    pass


class UnsafeArray(_AllOps, LamellarArray):
    KIND = ArrayKind.Unsafe


class AtomicArray(_AllOps, LamellarArray):
    """NativeAtomicArray for integer T, GenericAtomicArray for f32/f64 (atomic.rs:867-878)."""

    def _kind(self):
        return ArrayKind.GenericAtomic if self.dtype.is_float else ArrayKind.NativeAtomic


class LocalLockArray(_AllOps, LamellarArray):
    KIND = ArrayKind.LocalLock


class GlobalLockArray(_AllOps, LamellarArray):
    KIND = ArrayKind.GlobalLock


class ReadOnlyArray(_ReadOnlyOps, LamellarArray):
    KIND = ArrayKind.ReadOnly


__all__ = ["UnsafeArray", "AtomicArray", "LocalLockArray", "GlobalLockArray", "ReadOnlyArray",
           "Ok", "Err", "BatchResult", "LamellarError", "Distribution", "LmrStatus"]
