"""Shared input generators for parity tests (test-only helpers)."""
import numpy as np

DTYPE_NAMES = ["u8", "u16", "u32", "u64", "i8", "i16", "i32", "i64", "f32", "f64"]
NP = {"u8": np.uint8, "u16": np.uint16, "u32": np.uint32, "u64": np.uint64, "i8": np.int8,
      "i16": np.int16, "i32": np.int32, "i64": np.int64, "f32": np.float32, "f64": np.float64}
CODE = {n: i for i, n in enumerate(DTYPE_NAMES)}
IS_FLOAT = {n: n.startswith("f") for n in DTYPE_NAMES}

# ArrayOpCmd codes
ADD, FETCH_ADD, SUB, FETCH_SUB, MUL, FETCH_MUL, DIV, FETCH_DIV, REM, FETCH_REM = range(10)
AND, FETCH_AND, OR, FETCH_OR, XOR, FETCH_XOR, STORE, LOAD, SWAP, PUT, GET = range(10, 21)
CAS, CAS_EPS, SHL, FETCH_SHL, SHR, FETCH_SHR = range(21, 27)
ALL_OPS = list(range(27))
FLOAT_OPS = [ADD, FETCH_ADD, SUB, FETCH_SUB, MUL, FETCH_MUL, DIV, FETCH_DIV, REM, FETCH_REM, STORE,
             LOAD, SWAP, PUT, GET, CAS_EPS]
RET_VALS = {FETCH_ADD, FETCH_SUB, FETCH_MUL, FETCH_DIV, FETCH_REM, FETCH_AND, FETCH_OR, FETCH_XOR,
            LOAD, SWAP, GET, FETCH_SHL, FETCH_SHR}
RET_RESULT = {CAS, CAS_EPS}
# final state independent of application order (wrapping integer arithmetic)
COMMUTATIVE_INT = {ADD, FETCH_ADD, SUB, FETCH_SUB, MUL, FETCH_MUL, AND, FETCH_AND, OR, FETCH_OR,
                   XOR, FETCH_XOR, LOAD, GET}


def ops_for(dt):
    return FLOAT_OPS if IS_FLOAT[dt] else ALL_OPS


def ret_kind(op):
    return 2 if op in RET_RESULT else (1 if op in RET_VALS else 0)


def rand_elems(dt, n, rng, op=None):
    t = NP[dt]
    if IS_FLOAT[dt]:
        a = rng.uniform(1.0, 100.0, n) * rng.choice([-1.0, 1.0], n)
        return a.astype(t)
    info = np.iinfo(t)
    a = rng.integers(info.min, info.max, n, dtype=t, endpoint=True)
    if op in (DIV, FETCH_DIV, REM, FETCH_REM) and info.min < 0:
        a[a == info.min] = 7       # avoid MIN / -1 (tested separately)
    return a


def rand_vals(dt, n, rng, op):
    t = NP[dt]
    if IS_FLOAT[dt]:
        if op in (MUL, FETCH_MUL, DIV, FETCH_DIV, REM, FETCH_REM):
            return (rng.uniform(0.5, 4.0, n) * rng.choice([-1.0, 1.0], n)).astype(t)
        return (rng.uniform(1.0, 100.0, n) * rng.choice([-1.0, 1.0], n)).astype(t)
    info = np.iinfo(t)
    if op in (DIV, FETCH_DIV, REM, FETCH_REM):
        v = rng.integers(1, 10, n).astype(t)
        if info.min < 0:
            neg = rng.random(n) < 0.5
            v[neg] = (-(rng.integers(2, 10, int(neg.sum())))).astype(t)
        return v
    if op in (MUL, FETCH_MUL):
        return rng.integers(0, min(info.max, 1000), n).astype(t)
    return rng.integers(info.min, info.max, n, dtype=t, endpoint=True)


def cas_operands(dt, elems, vals, rng):
    """current value = a common value; make ~half of the target elements equal to it."""
    t = NP[dt]
    cur = t(3) if not IS_FLOAT[dt] else t(3.0)
    mask = rng.random(elems.size) < 0.5
    elems = elems.copy()
    elems[mask] = cur
    eps = t(2) if not IS_FLOAT[dt] else t(0.5)
    return cur, eps, elems


def record_dtype(iw, dt, rb, vo):
    it = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[iw]
    return np.dtype({"names": ["i", "v"], "formats": [it, NP[dt]], "offsets": [0, vo], "itemsize": rb})


def to_aos(idx, vals, iw, dt, rb, vo):
    rec = np.zeros(idx.size, dtype=record_dtype(iw, dt, rb, vo))
    rec["i"] = idx
    rec["v"] = vals
    return np.frombuffer(rec.tobytes(), dtype=np.uint8).copy()


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    u = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize]
    return np.array_equal(a.view(u), b.view(u))
