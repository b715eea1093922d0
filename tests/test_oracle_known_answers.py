"""Pin the CPU oracle against the reference's own known-answer tests.

The reference holds no golden vectors (its tests are unseeded); what pins the
oracle are the invariants its test programs check, restated
here over N simulated PEs, every (array type, distribution, element type,
PE count, length) combination of the reference's matrices:
  tests/array/arithmetic_ops/{add,sub,mul,div,fetch_add}_test.rs,
  tests/array/bitwise_ops/{and,or,xor,fetch_xor}_test.rs,
  tests/array/atomic_ops/{swap,compare_exchange}_test.rs.
Each PE's batch is applied in turn (the checks are order-independent).
"""
import numpy as np
import pytest

from opgen import (ADD, AND, CAS, DIV, FETCH_ADD, FETCH_XOR, LOAD, MUL, NP, OR, SUB, SWAP, XOR)
from simworld import SimArray

INT_TYPES = ["u8", "u16", "u32", "u64", "i8", "i16", "i32", "i64"]
ALL_TYPES = INT_TYPES + ["f32", "f64"]
LENS = [4, 19, 128]
PES = [1, 2, 3, 4]
ARRAYS = ["AtomicArray", "LocalLockArray", "UnsafeArray"]


def T(dt, v):
    return np.array([v]).astype(NP[dt])[0]


def wrap_mul(dt, a, b):
    return (np.array([a], dtype=NP[dt]) * np.array([b], dtype=NP[dt]))[0]


def check_close(vals, expect):
    """check_val!: ((val - max_val) as f64).abs() <= 0.0001 with T-wrapping subtraction."""
    d = (vals - np.array([expect], dtype=vals.dtype)).astype(np.float64)
    return bool(np.all(np.abs(d) <= 1e-4))


@pytest.mark.parametrize("array_type", ARRAYS)
@pytest.mark.parametrize("dist", [0, 1], ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", ALL_TYPES)
def test_add_known_answer(orc, dt, npes, dist, array_type):
    """add_test.rs:88-111 (+ shuffled batch :131-160, sub-arrays :166-290)."""
    for length in LENS:
        pe_max_val = 9 if dt == "f32" else 50
        max_val = np.zeros(1, dtype=NP[dt])[0]
        for pe in range(npes):
            max_val = (np.array([max_val]) + np.array([wrap_mul(dt, T(dt, 10 ** (2 * pe)), T(dt, pe_max_val))])
                       ).astype(NP[dt])[0]
        a = SimArray(orc, npes, length, dist, dt, array_type)
        a.fill(0)
        if length <= 19:   # per-element single adds: add(idx, 10^(2 my_pe)) (the 1x1 form)
            for my_pe in range(npes):
                for idx in range(a.len()):
                    for _ in range(pe_max_val):
                        st, _, _ = a.op(ADD, idx, T(dt, 10 ** (2 * my_pe)))
                        assert st == 0
            if array_type != "UnsafeArray":
                assert check_close(a.to_numpy(), max_val), (dt, npes, length)
        # shuffled batch: batch_add(indices, val)
        a.fill(0)
        rng = np.random.default_rng(length + npes)
        for my_pe in range(npes):
            ind = np.tile(np.arange(length, dtype=np.uint64), pe_max_val)
            rng.shuffle(ind)
            st, _, _ = a.op(ADD, ind, T(dt, 10 ** (2 * my_pe)))
            assert st == 0
        assert check_close(a.to_numpy(), max_val)
        # half sub-array
        a.fill(0)
        sub = a.sub_array(length // 2, length)
        for my_pe in range(npes):
            ind = np.tile(np.arange(sub.len(), dtype=np.uint64), pe_max_val)
            st, _, _ = sub.op(ADD, ind, T(dt, 10 ** (2 * my_pe)))
            assert st == 0
        got = a.to_numpy()
        assert check_close(got[length // 2:], max_val) and np.all(got[:length // 2] == 0)


@pytest.mark.parametrize("dist", [0, 1], ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", ALL_TYPES)
def test_sub_known_answer(orc, dt, npes, dist):
    """sub_test.rs:96-118: init 100*num_pes, every PE subtracts 1 a hundred times -> 0."""
    for length in LENS:
        pe_max_val = 100
        init = wrap_mul(dt, T(dt, pe_max_val), T(dt, npes))
        a = SimArray(orc, npes, length, dist, dt)
        a.fill(init)
        for _ in range(npes):
            ind = np.tile(np.arange(length, dtype=np.uint64), pe_max_val)
            assert a.op(SUB, ind, T(dt, 1))[0] == 0
        assert check_close(a.to_numpy(), 0)


def max_updates(dt, npes):
    """max_updates! (mul_test.rs:59-71): (128 - lz(T::MAX as u128 / npes) - 1) / npes."""
    tmax = {"u8": 2**8 - 1, "u16": 2**16 - 1, "u32": 2**32 - 1, "u64": 2**64 - 1, "i8": 2**7 - 1,
            "i16": 2**15 - 1, "i32": 2**31 - 1, "i64": 2**63 - 1,
            "f32": int(np.finfo(np.float32).max), "f64": 2**128 - 1}[dt]   # f64::MAX as u128 saturates
    q = tmax // npes
    lz = 128 - q.bit_length()
    return (128 - lz - 1) // npes


@pytest.mark.parametrize("dist", [0, 1], ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", ALL_TYPES)
def test_mul_div_known_answer(orc, dt, npes, dist):
    """mul_test.rs:99-117 (1 * 2^(updates*npes)) and div_test.rs:91-110 (back to 1)."""
    mu = max_updates(dt, npes)
    max_val = np.array([2 ** (mu * npes)]).astype(NP[dt])[0] if not dt.startswith("f") else \
        NP[dt](2.0 ** (mu * npes))
    for length in LENS:
        a = SimArray(orc, npes, length, dist, dt)
        a.fill(1)
        for _ in range(npes):
            assert a.op(MUL, np.tile(np.arange(length, dtype=np.uint64), mu), T(dt, 2))[0] == 0
        assert np.all(a.to_numpy() == max_val), (dt, npes, mu)
        for _ in range(npes):
            assert a.op(DIV, np.tile(np.arange(length, dtype=np.uint64), mu), T(dt, 2))[0] == 0
        assert np.all(a.to_numpy() == 1)


@pytest.mark.parametrize("dist", [0, 1], ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", INT_TYPES)
def test_bitwise_known_answers(orc, dt, npes, dist):
    """xor_test.rs:78-98, and_test.rs:80-97, or_test.rs, fetch_xor_test.rs:85-98."""
    t = NP[dt]
    for length in LENS:
        a = SimArray(orc, npes, length, dist, dt)
        a.fill(0)
        for p in range(npes):
            assert a.op(XOR, np.arange(length, dtype=np.uint64), t(1) << t(p))[0] == 0
        assert np.all(a.to_numpy() == t(~(~t(0) << t(npes))))
        a.fill(~t(0))
        for p in range(npes):
            assert a.op(AND, np.arange(length, dtype=np.uint64), t(~(t(1) << t(p))))[0] == 0
        assert np.all(a.to_numpy() == t(~t(0) << t(npes)))
        a.fill(0)
        for p in range(npes):
            assert a.op(OR, np.arange(length, dtype=np.uint64), t(1) << t(p))[0] == 0
        assert np.all(a.to_numpy() == t(~(~t(0) << t(npes))))
        # fetch_xor: the returned old never already holds the caller's bit
        a.fill(0)
        for p in range(npes):
            st, res, _ = a.op(FETCH_XOR, np.arange(length, dtype=np.uint64), t(1) << t(p))
            assert st == 0 and np.all((res & (t(1) << t(p))) == 0)


@pytest.mark.parametrize("dist", [0, 1], ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", ALL_TYPES)
def test_fetch_add_known_answer(orc, dt, npes, dist):
    """fetch_add_test.rs:134-149: 10 fetch_add(idx, 1) per element per PE; the olds a PE
    receives for one index are distinct, and the final value is 10 * num_pes."""
    for length in LENS:
        a = SimArray(orc, npes, length, dist, dt)
        a.fill(0)
        for _ in range(npes):
            ind = np.repeat(np.arange(length, dtype=np.uint64), 10)
            st, res, _ = a.op(FETCH_ADD, ind, T(dt, 1))
            assert st == 0
            r = res.reshape(length, 10)
            assert all(len(set(row.tolist())) == 10 for row in r)
        assert np.all(a.to_numpy() == T(dt, 10 * npes))


@pytest.mark.parametrize("dist", [0, 1], ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", ALL_TYPES)
def test_swap_known_answer(orc, dt, npes, dist):
    """swap_test.rs:70-106: PE p swaps p into indices = p (mod num_pes): the old value
    is the init value; afterwards load(idx) == idx % num_pes."""
    for length in LENS:
        a = SimArray(orc, npes, length, dist, dt)
        init = T(dt, npes)
        a.fill(init)
        for p in range(npes):
            ind = np.arange(p, length, npes, dtype=np.uint64)
            if ind.size == 0:
                continue
            st, res, _ = a.op(SWAP, ind, T(dt, p))
            assert st == 0 and np.all(res == init)
        st, res, _ = a.op(LOAD, np.arange(length, dtype=np.uint64), T(dt, 0))
        assert np.all(res == (np.arange(length) % npes).astype(NP[dt]))


@pytest.mark.parametrize("dist", [0, 1], ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", INT_TYPES)
def test_compare_exchange_known_answer(orc, dt, npes, dist):
    """compare_exchange_test.rs:70-116: round 1 on owned indices returns Ok(init);
    round 2 on every index fails."""
    for length in LENS:
        a = SimArray(orc, npes, length, dist, dt)
        init = T(dt, npes)
        a.fill(init)
        for p in range(npes):
            ind = np.arange(p, length, npes, dtype=np.uint64)
            if ind.size == 0:
                continue
            st, res, ok = a.op(CAS, ind, T(dt, p), current=init)
            assert st == 0 and np.all(ok == 1) and np.all(res == init)
        for p in range(npes):
            st, res, ok = a.op(CAS, np.arange(length, dtype=np.uint64), T(dt, p), current=init)
            assert st == 0 and np.all(ok == 0)


@pytest.mark.parametrize("npes", [1, 2, 3, 4])
@pytest.mark.parametrize("dist", [0, 1], ids=["Block", "Cyclic"])
@pytest.mark.parametrize("total_len", [100, 7, 1000])
def test_reduce_known_answer(orc, npes, dist, total_len):
    """examples/array_examples/dist_array_reduce.rs:36-109: an UnsafeArray<usize> holding
    0..total_len (put from PE 0), sum() == (total_len / 2) * (0 + 99) for the default 100
    elements, Block and Cyclic alike; min / max the ends. The oracle's per-PE fold
    (array_reduce.rs:82-88) and cross-PE tree (:90-107) must give it on every layout."""
    from oracle import oracle as o
    a = SimArray(orc, npes, total_len, dist, "u64", "UnsafeArray")
    g = np.arange(total_len, dtype=np.uint64)
    for pe in range(npes):                      # place element i at its owner's local offset
        for i in g:
            p, off = orc.pe_and_offset(a.L, int(i))
            if p == pe:
                a.shards[pe][off] = i
    sl = a.slices()
    per = {op: [o.reduce(3, np.uint64, op, s) for s in sl] for op in ("sum", "min", "max", "prod")}
    assert o.reduce_tree(3, np.uint64, "sum", per["sum"]) == total_len * (total_len - 1) // 2
    if total_len == 100:
        assert o.reduce_tree(3, np.uint64, "sum", per["sum"]) == (total_len // 2) * (0 + 99)
    assert o.reduce_tree(3, np.uint64, "min", per["min"]) == 0
    assert o.reduce_tree(3, np.uint64, "max", per["max"]) == total_len - 1
    assert o.reduce_tree(3, np.uint64, "prod", per["prod"]) == 0


@pytest.mark.parametrize("dt", ["u8", "i8", "u16", "i32", "u64", "i64", "f32", "f64"])
def test_reduce_oracle_vs_sequential_fold(orc, dt):
    """orc_reduce is the left fold of the reference closures: wrapping integers, float
    rounding in sequence; None for an empty slice."""
    from oracle import oracle as o
    rng = np.random.default_rng(3)
    t = NP[dt]
    x = (rng.random(2000) * 100 - 50).astype(t) if dt.startswith("f") else \
        rng.integers(np.iinfo(t).min, np.iinfo(t).max, 2000, dtype=t, endpoint=True)
    code = {"u8": 0, "u16": 1, "u32": 2, "u64": 3, "i8": 4, "i16": 5, "i32": 6, "i64": 7, "f32": 8, "f64": 9}[dt]
    with np.errstate(over="ignore"):
        acc_s, acc_p = x[0], x[0]
        for v in x[1:]:
            acc_s = t(acc_s + v)
            acc_p = t(acc_p * v)
    assert np.array([o.reduce(code, t, "sum", x)], t).tobytes() == np.array([acc_s], t).tobytes()
    assert np.array([o.reduce(code, t, "prod", x)], t).tobytes() == np.array([acc_p], t).tobytes()
    assert o.reduce(code, t, "max", x) == x.max() and o.reduce(code, t, "min", x) == x.min()
    assert o.reduce(code, t, "sum", x[:0]) is None
