"""The oracle's linearisability checker (oracle/linearize.c), on the CPU.

It decides, per element, whether the returned values / Ok flags and the final value
of a batch come from some serial order of that element's records — what every
reference array kind guarantees (impl/src/array_ops.rs:327-545: one SeqCst RMW, CAS
loop, per-element mutex or shard lock per record; no order promised,
src/array/operations/arithmetic.rs:57-58). Histories made by applying the records in
a random serial order with the oracle must pass; tampered ones must fail.
"""
import numpy as np
import pytest

from opgen import (CAS, CAS_EPS, CODE, FETCH_ADD, FETCH_AND, FETCH_DIV, FETCH_MUL, FETCH_OR, FETCH_REM,
                   FETCH_SHL, FETCH_SHR, FETCH_SUB, FETCH_XOR, IS_FLOAT, LOAD, NP, SWAP, rand_elems,
                   rand_vals)

KIND_NATIVE, KIND_GENERIC, KIND_LOCAL_LOCK = 1, 2, 3
ORDER_DEP = [FETCH_ADD, FETCH_SUB, FETCH_MUL, FETCH_DIV, FETCH_REM, FETCH_AND, FETCH_OR, FETCH_XOR,
             FETCH_SHL, FETCH_SHR, SWAP, LOAD, CAS, CAS_EPS]


def serial_history(orc, dt, op, kind, shard0, idx, vals, cur, eps, rng):
    """Apply the records one at a time in a random order (the oracle's semantics):
    returns (final shard, per-record results, per-record ok) in record order."""
    t = NP[dt]
    L = orc.layout_new(shard0.size, 1, 0, 0)
    perm = rng.permutation(idx.size)
    ref = shard0.copy()
    st, res, ok = orc.batch_op(L, [ref], kind, CODE[dt], t, op, idx[perm], vals[perm], cur, eps)
    assert st == 0
    r = np.empty_like(res)
    o = np.empty_like(ok)
    r[perm] = res
    o[perm] = ok
    return ref, r, o


def make_inputs(dt, op, rng, slice_len, n):
    t = NP[dt]
    shard0 = rand_elems(dt, slice_len, rng, op)
    idx = rng.integers(0, slice_len, n).astype(np.uint64)
    vals = rand_vals(dt, n, rng, op)
    cur = eps = None
    if op in (FETCH_SHL, FETCH_SHR):
        vals = rng.integers(0, 3, n).astype(t)           # small shifts: states stay distinct
    if op in (CAS, CAS_EPS):
        cur = t(3) if not IS_FLOAT[dt] else t(3.0)
        eps = t(2) if not IS_FLOAT[dt] else t(0.5)
        shard0[rng.random(slice_len) < 0.5] = cur
        vals[rng.random(n) < 0.3] = cur                   # some records write `current` back
    return shard0, idx, vals, cur, eps


@pytest.mark.parametrize("dt", ["u8", "u16", "u32", "u64", "i8", "i32", "i64", "f32", "f64"])
def test_serial_histories_pass(orc, dt):
    rng = np.random.default_rng(100 + CODE[dt])
    for op in ORDER_DEP:
        if IS_FLOAT[dt] and op in (FETCH_AND, FETCH_OR, FETCH_XOR, FETCH_SHL, FETCH_SHR, CAS):
            continue
        if IS_FLOAT[dt] and op in (FETCH_MUL, FETCH_DIV, FETCH_REM):
            continue                                      # float products drift into denormals
        kind = KIND_GENERIC if IS_FLOAT[dt] else KIND_NATIVE
        for kd in ([kind, KIND_LOCAL_LOCK] if op == CAS_EPS else [kind]):
            shard0, idx, vals, cur, eps = make_inputs(dt, op, rng, 300, 3000)
            fin, res, ok = serial_history(orc, dt, op, kd, shard0, idx, vals, cur, eps, rng)
            st, bad = orc.check_linearizable(kd, CODE[dt], NP[dt], op, shard0, fin, idx, vals, res, ok, cur, eps)
            assert st == 0, (dt, op, kd, bad)


def test_hot_element_is_fast(orc):
    """One element with 200k fetch_add records (Zipf-like hot spot): linear time."""
    rng = np.random.default_rng(3)
    n = 200000
    idx = np.zeros(n, dtype=np.uint64)
    idx[::7] = rng.integers(0, 1000, idx[::7].size).astype(np.uint64)
    vals = rng.integers(0, 2**40, n).astype(np.uint64)
    shard0 = rng.integers(0, 2**60, 1000).astype(np.uint64)
    fin, res, ok = serial_history(orc, "u64", FETCH_ADD, KIND_NATIVE, shard0, idx, vals, None, None, rng)
    st, _ = orc.check_linearizable(KIND_NATIVE, CODE["u64"], np.uint64, FETCH_ADD, shard0, fin, idx, vals, res)
    assert st == 0


def test_block_serial_histories_pass(orc):
    """Records applied as contiguous blocks (the device's delta mode: a workgroup's
    records combined, then applied at once) are still one serial order."""
    rng = np.random.default_rng(9)
    shard0 = np.zeros(16, dtype=np.uint64)
    idx = rng.integers(0, 16, 5000).astype(np.uint64)
    vals = np.ones(5000, dtype=np.uint64)
    fin, res, ok = serial_history(orc, "u64", FETCH_ADD, KIND_NATIVE, shard0, idx, vals, None, None, rng)
    st, _ = orc.check_linearizable(KIND_NATIVE, CODE["u64"], np.uint64, FETCH_ADD, shard0, fin, idx, vals, res)
    assert st == 0


@pytest.mark.parametrize("op", [FETCH_ADD, FETCH_XOR, FETCH_MUL, SWAP, FETCH_SHL])
def test_tampered_histories_fail(orc, op):
    rng = np.random.default_rng(50 + op)
    dt = "u32"
    shard0, idx, vals, cur, eps = make_inputs(dt, op, rng, 50, 2000)
    fin, res, ok = serial_history(orc, dt, op, KIND_NATIVE, shard0, idx, vals, cur, eps, rng)
    # a returned value that no serial order produces
    r2 = res.copy()
    k = int(np.nonzero(idx == idx[0])[0][-1])
    r2[k] ^= np.uint32(0x80000001)
    st, bad = orc.check_linearizable(KIND_NATIVE, CODE[dt], NP[dt], op, shard0, fin, idx, vals, r2, ok, cur, eps)
    assert st == 1 and bad == int(idx[0])
    # a wrong final value
    f2 = fin.copy()
    f2[int(idx[5])] ^= np.uint32(1)
    st, bad = orc.check_linearizable(KIND_NATIVE, CODE[dt], NP[dt], op, shard0, f2, idx, vals, res, ok, cur, eps)
    assert st == 1 and bad == int(idx[5])


def test_known_small_cases(orc):
    u64 = np.uint64
    c = CODE["u64"]
    # fetch_add(1) x3 from 0: olds must be {0, 1, 2}
    idx = np.zeros(3, dtype=u64)
    ones = np.ones(3, dtype=u64)
    assert orc.check_linearizable(1, c, u64, FETCH_ADD, [0], [3], idx, ones, [2, 0, 1])[0] == 0
    assert orc.check_linearizable(1, c, u64, FETCH_ADD, [0], [3], idx, ones, [0, 1, 1])[0] == 1
    # swap: olds chain init -> v -> v'
    assert orc.check_linearizable(1, c, u64, SWAP, [7], [9], idx[:2], [9, 8], [8, 7])[0] == 0
    assert orc.check_linearizable(1, c, u64, SWAP, [7], [8], idx[:2], [9, 8], [8, 7])[0] == 1
    # compare_exchange(current = 5): one success 5 -> 6, the other fails seeing 6
    cas = dict(current=5)
    assert orc.check_linearizable(1, c, u64, CAS, [5], [6], idx[:2], [6, 4], [5, 6], [1, 0], **cas)[0] == 0
    assert orc.check_linearizable(1, c, u64, CAS, [5], [4], idx[:2], [6, 4], [5, 6], [1, 0], **cas)[0] == 1
    # two successes are impossible once the first writes a value != current
    assert orc.check_linearizable(1, c, u64, CAS, [5], [4], idx[:2], [6, 4], [5, 5], [1, 1], **cas)[0] == 1
    # NativeAtomic compare_exchange_epsilon (array_ops.rs:391-419): exact match -> Ok(new)
    eps = dict(current=5, eps=2)
    assert orc.check_linearizable(1, c, u64, CAS_EPS, [5], [9], idx[:1], [9], [9], [1], **eps)[0] == 0
    assert orc.check_linearizable(1, c, u64, CAS_EPS, [6], [9], idx[:1], [9], [6], [1], **eps)[0] == 0
    # the generic kinds return Ok(current) (array_ops.rs:521-535)
    assert orc.check_linearizable(3, c, u64, CAS_EPS, [6], [9], idx[:1], [9], [5], [1], **eps)[0] == 0
    assert orc.check_linearizable(3, c, u64, CAS_EPS, [6], [9], idx[:1], [9], [6], [1], **eps)[0] == 1


def test_cas_eps_record_that_is_a_noop_at_one_state_and_a_change_at_another(orc):
    """NativeAtomic compare_exchange_epsilon(current = 3, eps = 2) of new = 4 returns
    4 both at state 3 (exact match: Ok(new), 3 -> 4) and at state 4 (|4 - 3| < 2:
    Ok(old), no change). From 4: C = cas_eps(new = 3) moves 4 -> 3 returning Ok(4),
    then A = cas_eps(new = 4) moves 3 -> 4 returning Ok(4). Taking A as a no-op at the
    initial 4 would strand the search at 3; the only order is C, A."""
    u8 = np.uint8
    c = CODE["u8"]
    idx = np.zeros(2, dtype=np.uint64)
    eps = dict(current=u8(3), eps=u8(2))
    # records: A (new 4, Ok(4)), C (new 3, Ok(4)); 4 -> 3 -> 4
    assert orc.check_linearizable(1, c, u8, CAS_EPS, np.array([4], u8), np.array([4], u8), idx,
                                  np.array([4, 3], u8), np.array([4, 4], u8), np.array([1, 1], np.uint8),
                                  **eps)[0] == 0
    # ... they may also end at 3 (A as a no-op at 4, then C), never at 5
    assert orc.check_linearizable(1, c, u8, CAS_EPS, np.array([4], u8), np.array([3], u8), idx,
                                  np.array([4, 3], u8), np.array([4, 4], u8), np.array([1, 1], np.uint8),
                                  **eps)[0] == 0
    assert orc.check_linearizable(1, c, u8, CAS_EPS, np.array([4], u8), np.array([5], u8), idx,
                                  np.array([4, 3], u8), np.array([4, 4], u8), np.array([1, 1], np.uint8),
                                  **eps)[0] == 1


@pytest.mark.parametrize("dt,op", [("u16", FETCH_ADD), ("u8", FETCH_XOR), ("i16", FETCH_SUB), ("u8", SWAP),
                                   ("u16", CAS)])
def test_small_type_hot_element_revisits_states(orc, dt, op):
    """400k records on one 8/16-bit element revisit every state many times, so a
    search would branch without end; with returned values that name the state they
    ran at, the check is an Eulerian-trail question and stays exact and linear."""
    rng = np.random.default_rng(77 + op)
    t = NP[dt]
    n = 400000
    idx = np.zeros(n, dtype=np.uint64)
    info = np.iinfo(t)
    vals = rng.integers(info.min, info.max, n, dtype=t, endpoint=True)
    cur = t(3) if op == CAS else None
    shard0 = np.array([3], dtype=t)
    if op == CAS:
        vals[rng.random(n) < 0.5] = t(3)        # successes keep the state at `current` ...
        vals[-1] = t(9)                          # ... until one of them writes 9
    fin, res, ok = serial_history(orc, dt, op, KIND_NATIVE, shard0, idx, vals, cur, None, rng)
    st, _ = orc.check_linearizable(KIND_NATIVE, CODE[dt], t, op, shard0, fin, idx, vals, res, ok, cur)
    assert st == 0
    r2 = res.copy()
    r2[rng.integers(0, n)] ^= t(1)
    st, _ = orc.check_linearizable(KIND_NATIVE, CODE[dt], t, op, shard0, fin, idx, vals, r2, ok, cur)
    assert st == 1
