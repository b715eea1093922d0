"""Vocabulary of the batched element-op path (mirrors include/lamellar_types.h)."""
from __future__ import annotations

import enum

import numpy as np


class ArrayOpCmd(enum.IntEnum):
    """src/array/operations.rs:86-114, declaration order."""
    Add = 0
    FetchAdd = 1
    Sub = 2
    FetchSub = 3
    Mul = 4
    FetchMul = 5
    Div = 6
    FetchDiv = 7
    Rem = 8
    FetchRem = 9
    And = 10
    FetchAnd = 11
    Or = 12
    FetchOr = 13
    Xor = 14
    FetchXor = 15
    Store = 16
    Load = 17
    Swap = 18
    Put = 19
    Get = 20
    CompareExchange = 21
    CompareExchangeEps = 22
    Shl = 23
    FetchShl = 24
    Shr = 25
    FetchShr = 26


class BatchReturnType(enum.IntEnum):
    """src/array/unsafe/operations.rs:850-854."""
    None_ = 0
    Vals = 1
    Result = 2


class Distribution(enum.IntEnum):
    """src/array.rs:247-252."""
    Block = 0
    Cyclic = 1


class ArrayKind(enum.IntEnum):
    Unsafe = 0
    NativeAtomic = 1
    GenericAtomic = 2
    LocalLock = 3
    GlobalLock = 4
    ReadOnly = 5


class Strategy(enum.IntEnum):
    Auto = 0
    Direct = 1
    Tiled = 2
    Ordered = 3


class LmrStatus(enum.IntEnum):
    OK = 0
    INVALID = 1
    OOB = 2
    DIVZERO = 3
    OVERFLOW = 4
    UNSUPPORTED = 5
    HIP = 6
    WORKSPACE = 7
    LENGTH = 8


ERRBIT_OOB = 0x1
ERRBIT_DIVZERO = 0x2
ERRBIT_OVERFLOW = 0x4
ERRBIT_UNSUPPORTED = 0x8
ERRBIT_TRANSPORT = 0x10


class DType:
    """One element type: lmr_dtype_t code, numpy dtype, torch storage dtype.

    Device storage uses the signed torch dtype of the same width (bit-identical);
    values are presented through the numpy dtype.
    """

    def __init__(self, name, code, np_dtype, torch_name, is_float, signed):
        self.name = name
        self.code = code
        self.np = np.dtype(np_dtype)
        self.torch_name = torch_name
        self.is_float = is_float
        self.signed = signed
        self.bytes = self.np.itemsize

    @property
    def torch(self):
        import torch
        return getattr(torch, self.torch_name)

    def __repr__(self):
        return f"DType({self.name})"

    def to_bits(self, value) -> int:
        """Raw little-endian bits of one element value, as a Python int."""
        a = np.array([value]).astype(self.np) if not isinstance(value, np.ndarray) else value.astype(self.np)
        u = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[self.bytes]
        return int(a.view(u)[0])

    def from_bits(self, bits: int):
        u = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[self.bytes]
        return np.array([bits], dtype=u).view(self.np)[0]

    def as_storage_scalar(self, value):
        """Value reinterpreted as the torch storage dtype (for fill_)."""
        st = {1: np.int8, 2: np.int16, 4: np.int32, 8: np.int64}[self.bytes]
        if self.is_float:
            return float(np.array([value], dtype=self.np)[0])
        return int(np.array([value]).astype(self.np).view(st)[0])


DTYPES = {
    "u8": DType("u8", 0, np.uint8, "uint8", False, False),
    "u16": DType("u16", 1, np.uint16, "int16", False, False),
    "u32": DType("u32", 2, np.uint32, "int32", False, False),
    "u64": DType("u64", 3, np.uint64, "int64", False, False),
    "usize": DType("usize", 3, np.uint64, "int64", False, False),
    "i8": DType("i8", 4, np.int8, "int8", False, True),
    "i16": DType("i16", 5, np.int16, "int16", False, True),
    "i32": DType("i32", 6, np.int32, "int32", False, True),
    "i64": DType("i64", 7, np.int64, "int64", False, True),
    "isize": DType("isize", 7, np.int64, "int64", False, True),
    "f32": DType("f32", 8, np.float32, "float32", True, True),
    "f64": DType("f64", 9, np.float64, "float64", True, True),
}


def dtype_of(t) -> DType:
    if isinstance(t, DType):
        return t
    if isinstance(t, str):
        return DTYPES[t]
    npd = np.dtype(t)
    for d in DTYPES.values():
        if d.np == npd:
            return d
    raise TypeError(f"unsupported element type {t!r}")


RET_KIND = {op: BatchReturnType.None_ for op in ArrayOpCmd}
for _op in (ArrayOpCmd.FetchAdd, ArrayOpCmd.FetchSub, ArrayOpCmd.FetchMul, ArrayOpCmd.FetchDiv,
            ArrayOpCmd.FetchRem, ArrayOpCmd.FetchAnd, ArrayOpCmd.FetchOr, ArrayOpCmd.FetchXor,
            ArrayOpCmd.Load, ArrayOpCmd.Swap, ArrayOpCmd.Get, ArrayOpCmd.FetchShl,
            ArrayOpCmd.FetchShr):
    RET_KIND[_op] = BatchReturnType.Vals
for _op in (ArrayOpCmd.CompareExchange, ArrayOpCmd.CompareExchangeEps):
    RET_KIND[_op] = BatchReturnType.Result


def op_supported(kind: int, dt: DType, op: int) -> bool:
    """src/array.rs:207-220 + impl/src/array_ops.rs:1503-1533."""
    if kind == ArrayKind.ReadOnly:
        return op == ArrayOpCmd.Load
    if not dt.is_float:
        return True
    return op not in (ArrayOpCmd.And, ArrayOpCmd.FetchAnd, ArrayOpCmd.Or, ArrayOpCmd.FetchOr,
                      ArrayOpCmd.Xor, ArrayOpCmd.FetchXor, ArrayOpCmd.CompareExchange,
                      ArrayOpCmd.Shl, ArrayOpCmd.FetchShl, ArrayOpCmd.Shr, ArrayOpCmd.FetchShr)
