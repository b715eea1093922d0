"""lmr_reduce: the per-PE step of array.sum / prod / max / min
(src/array/unsafe.rs:1414-1557, impl/src/array_reduce.rs:82-88, 283-319),
against the oracle's sequential fold of the same elements (orc_reduce, pinned
by dist_array_reduce.rs's known answer in test_oracle_known_answers.py). Integers (wrapping) and
max / min are bit-exact; float sum / prod within a relative tolerance of
n * eps (the device folds in a tree order)."""
import numpy as np
import pytest
import torch

from opgen import NP

pytestmark = pytest.mark.gpu

DTS = ["u8", "u16", "u32", "u64", "i8", "i16", "i32", "i64", "f32", "f64"]


CODES = {"u8": 0, "u16": 1, "u32": 2, "u64": 3, "i8": 4, "i16": 5, "i32": 6, "i64": 7, "f32": 8, "f64": 9}


def oracle_fold(op, dt, a):
    """The reference's per-PE step (array_reduce.rs:82-88), restated in the C oracle."""
    from oracle import oracle as o
    return o.reduce(CODES[dt], NP[dt], op, a)


STORAGE = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}


def store(a, x):
    """Write x into a's local slice (torch storage dtype view of the element bits)."""
    v = x if x.dtype.kind == "f" else x.view(STORAGE[x.itemsize])
    a.local_data().copy_(torch.from_numpy(np.ascontiguousarray(v)).cuda())


def make(dt, n, rng, op):
    t = NP[dt]
    if dt.startswith("f"):
        if op == "prod":
            return (1.0 + (rng.random(n) - 0.5) * 1e-3).astype(t)
        return (rng.random(n) * 200 - 100).astype(t)
    info = np.iinfo(t)
    return rng.integers(info.min, info.max, n, dtype=t, endpoint=True)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("op", ["sum", "prod", "max", "min"])
def test_reduce_local(world, lam, dt, op):
    rng = np.random.default_rng(hash((dt, op)) & 0xFFFF)
    for n in (0, 1, 7, 1000, 65537, (1 << 20) + 3):
        x = make(dt, n, rng, op)
        if n:
            a = lam.UnsafeArray(world.team(), n, lam.Distribution.Block, dt)
            store(a, x)
            got = a.reduce(op).block()
        else:
            a = lam.UnsafeArray(world.team(), 1, lam.Distribution.Block, dt)
            got = a.sub_array(0, 0).reduce(op).block()      # empty: the reference's None
        exp = oracle_fold(op, dt, x)
        if exp is None:
            assert got is None
            continue
        if dt.startswith("f") and op in ("sum", "prod"):
            # both the sequential fold and the device's tree fold are within n*eps of the exact
            # value (times sum|x| for a sum, |result| for a product of values near 1)
            eps = float(np.finfo(NP[dt]).eps)
            scale = float(np.abs(x.astype(np.float64)).sum()) if op == "sum" else abs(float(exp))
            assert abs(float(got) - float(exp)) <= 2 * n * eps * scale + 1e-30, (n, got, exp)
        else:
            assert np.array(got, dtype=NP[dt]).tobytes() == np.array(exp, dtype=NP[dt]).tobytes(), (n, got, exp)


def test_reduce_sub_array_and_atomic(world, lam):
    rng = np.random.default_rng(5)
    a = lam.AtomicArray(world.team(), 100003, lam.Distribution.Cyclic, "u64")
    x = rng.integers(0, 2**63, 100003).astype(np.uint64)
    store(a, x)
    s = a.sub_array(17, 90017)
    assert s.sum().block() == oracle_fold("sum", "u64", x[17:90017])
    assert s.max().block() == oracle_fold("max", "u64", x[17:90017])
    assert a.min().block() == oracle_fold("min", "u64", x)
