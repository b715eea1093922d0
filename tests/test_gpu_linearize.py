"""Order-dependent ops under colliding indices: the device's results must be a valid
linearisation, checked by the oracle's checker (oracle/linearize.c) per element.

The reference applies each record with one SeqCst RMW / CAS loop (NativeAtomic,
impl/src/array_ops.rs:327-458; swap and compare_exchange :379-419; mul/div/rem
:339-368, native_atomic.rs:42-74), a per-element mutex (GenericAtomic,
generic_atomic.rs:286-293) or a shard lock per AM (LocalLock, array_ops.rs:557-560),
and promises no order (operations/arithmetic.rs:57-58). So for swap,
compare_exchange(_epsilon), every fetch_* and load the only contract is: per element,
the returned olds / Result<T,T>s and the final value come from one serial order of
that element's records. Checked on every device path: direct atomics, the one-level
and two-level tiled partitions, the staged pipeline, and delta mode (hot tiles split
over workgroups). Plus reduced-size twins of BASELINE configs C5 (u32 and/or/xor/swap/
compare_exchange batches through the array API) and C3 (f64 fetch_add, Zipf 0.99).
"""
import numpy as np
import pytest
import torch

from opgen import (ADD, CAS, CAS_EPS, CODE, FETCH_ADD, FETCH_AND, FETCH_DIV, FETCH_MUL, FETCH_OR,
                   FETCH_REM, FETCH_SHL, FETCH_SHR, FETCH_SUB, FETCH_XOR, IS_FLOAT, LOAD, NP, SWAP,
                   bits_equal, rand_elems, rand_vals)
from test_gpu_parity import Case, KIND_LOCAL_LOCK, kind_for

pytestmark = pytest.mark.gpu

INT_OPS = [FETCH_ADD, FETCH_SUB, FETCH_MUL, FETCH_DIV, FETCH_REM, FETCH_AND, FETCH_OR, FETCH_XOR,
           FETCH_SHL, FETCH_SHR, SWAP, LOAD, CAS, CAS_EPS]
FLT_OPS = [FETCH_ADD, FETCH_SUB, FETCH_MUL, FETCH_DIV, SWAP, LOAD, CAS_EPS]
TILE = {1: 16384, 2: 16384, 4: 16384, 8: 8192}


def lin_inputs(dt, op, rng, shard_len, n, hot_set):
    """Colliding records: indices drawn from `hot_set` (~10 records per element).
    Float values are exact in every order (small integers, powers of two), so a serial
    order reproduces the device's bits exactly."""
    t = NP[dt]
    shard0 = rand_elems(dt, shard_len, rng, op)
    idx = hot_set[rng.integers(0, hot_set.size, n)].astype(np.uint64)
    vals = rand_vals(dt, n, rng, op)
    cur = eps = None
    if IS_FLOAT[dt]:
        shard0 = rng.integers(-1000, 1000, shard_len).astype(t)
        if op in (FETCH_MUL, FETCH_DIV):
            vals = rng.choice(np.array([0.5, 2.0, -1.0, 1.0, 4.0], dtype=t), n)
        else:
            vals = rng.integers(-64, 64, n).astype(t)
    if op in (FETCH_SHL, FETCH_SHR):
        vals = rng.integers(0, 3, n).astype(t)
    if op in (CAS, CAS_EPS):
        cur = t(3) if not IS_FLOAT[dt] else t(3.0)
        eps = t(2) if not IS_FLOAT[dt] else t(0.5)
        shard0[hot_set[rng.random(hot_set.size) < 0.5]] = cur
        vals[rng.random(n) < 0.2] = cur             # some records write `current` back
    return shard0, idx, vals, cur, eps


def check(orc, c, dt, op, kind, shard0, idx, vals, cur, eps, what):
    assert c.err == 0, (what, dt, op, c.err)
    st, bad = orc.check_linearizable(kind, CODE[dt], NP[dt], op, shard0, c.got, idx, vals, c.res_d,
                                     c.ok_d if c.rk == 2 else None, cur, eps)
    assert st == 0, (what, dt, op, "status", st, "element", bad)


def run_path(k, orc, lam, dt, path, monkeypatch):
    rng = np.random.default_rng(700 + CODE[dt] + 31 * ["direct", "tiled1", "tiled2", "staged"].index(path))
    eb = NP[dt](0).itemsize
    tile = TILE[eb]
    if path == "tiled1":
        shard_len = 5 * tile + 17                      # <= 128 tiles: one-level partition
    elif path == "direct":
        shard_len = 50000
    else:
        shard_len = 129 * tile + 77                    # > 128 tiles: two-level partition
    hot = rng.choice(shard_len, 20000, replace=False)
    n = 200000
    monkeypatch.setenv("LMR_STAGED", "1" if path == "staged" else "0")
    monkeypatch.setenv("LMR_STAGE_SPLIT", "3")
    strategy = 1 if path == "direct" else 2
    for op in (FLT_OPS if IS_FLOAT[dt] else INT_OPS):
        kinds = [kind_for(dt)] + ([KIND_LOCAL_LOCK] if op == CAS_EPS else [])
        for kind in kinds:
            shard0, idx, vals, cur, eps = lin_inputs(dt, op, rng, shard_len, n, hot)
            c = Case(k, orc, lam, dt, op, shard0, idx, vals, "soa", strategy, kind=kind, cur=cur, eps=eps)
            check(orc, c, dt, op, kind, shard0, idx, vals, cur, eps, path)


@pytest.mark.parametrize("path", ["direct", "tiled1", "tiled2", "staged"])
@pytest.mark.parametrize("dt", ["u32", "u64", "i32", "i64", "u8", "i16", "f32", "f64"])
def test_order_dependent_ops_linearizable(world, orc, lam, dt, path, monkeypatch):
    """swap, compare_exchange(_epsilon), load and every fetch_* on colliding streams:
    per element, returned values, Ok flags and the final value form one serial order."""
    k = world.team().kernels
    k.reserve(1 << 20)
    run_path(k, orc, lam, dt, path, monkeypatch)


@pytest.mark.parametrize("dt", ["u64", "i32", "u16", "f64", "f32"])
def test_delta_mode_fetch_linearizable(world, orc, lam, dt, monkeypatch):
    """A hot element (40 % of 2^20 records) makes its tile split into delta-mode work
    items for the combinable ops: each workgroup combines its records in LDS and
    applies them with one device atomic; fetch results = returned base (+) LDS prefix.
    The olds of every combinable fetch op must still form one serial order per element,
    on the one-level and the two-level partition."""
    monkeypatch.setenv("LMR_STAGED", "0")
    k = world.team().kernels
    k.reserve(1 << 21)
    rng = np.random.default_rng(17 + CODE[dt])
    t = NP[dt]
    ops = [FETCH_ADD, FETCH_SUB] if IS_FLOAT[dt] else [FETCH_ADD, FETCH_SUB, FETCH_AND, FETCH_OR, FETCH_XOR]
    eb = t(0).itemsize
    for shard_len in (1 << 16, 129 * TILE[eb] + 5):
        n = 1 << 20
        idx = rng.integers(0, shard_len, n).astype(np.uint64)
        idx[rng.random(n) < 0.4] = 12345
        for op in ops:
            if IS_FLOAT[dt]:
                shard0 = rng.integers(-100, 100, shard_len).astype(t)
                vals = rng.integers(-8, 8, n).astype(t)        # exact sums in any order
            else:
                shard0 = rand_elems(dt, shard_len, rng)
                vals = rand_vals(dt, n, rng, op)
            c = Case(k, orc, lam, dt, op, shard0, idx, vals, "soa", 2)
            check(orc, c, dt, op, kind_for(dt), shard0, idx, vals, None, None, "delta")


def test_c5_twin_mixed_u32_stream(world, orc, lam):
    """Reduced C5 (BASELINE configs[4]): AtomicArray<u32> of 2^22 elements, five
    batches in sequence -- bit_and, bit_or, bit_xor, swap, compare_exchange(current=0)
    -- each 2^22 / 2.5 records uniform over the array (C5's density: 0.4 records per
    element and batch), through the op-builder API with the default strategy. and/or/
    xor: bit-exact final state against the oracle; swap and compare_exchange: the
    olds / Results form one serial order per element, ending at the observed state."""
    team = world.team()
    rng = np.random.default_rng(0xC5)
    n_el = 1 << 22
    m = int(n_el * 0.4)
    arr = lam.AtomicArray(team, n_el, lam.Distribution.Block, "u32")
    init = rng.integers(0, 4, n_el).astype(np.uint32)        # many zeros: compare_exchange(0) succeeds
    arr.local_data().copy_(torch.from_numpy(init.view(np.int32)).cuda())
    L = orc.layout_new(n_el, 1, 0, 0)
    ref = init.copy()
    u32 = np.uint32
    for op, fn in ((10, "batch_bit_and"), (12, "batch_bit_or"), (14, "batch_bit_xor")):
        idx = rng.integers(0, n_el, m).astype(np.uint64)
        vals = rng.integers(0, 2**32, m, dtype=np.uint64).astype(u32)
        getattr(arr, fn)(idx, vals).block()
        st, _, _ = orc.batch_op(L, [ref], 1, CODE["u32"], u32, op, idx, vals)
        assert st == 0
        assert np.array_equal(arr.local_numpy(), ref), fn
    # swap
    before = arr.local_numpy().copy()
    idx = rng.integers(0, n_el, m).astype(np.uint64)
    vals = rng.integers(0, 2**32, m, dtype=np.uint64).astype(u32)
    olds = arr.batch_swap(idx, vals).block().cpu().numpy().view(u32)
    after = arr.local_numpy().copy()
    st, bad = orc.check_linearizable(1, CODE["u32"], u32, SWAP, before, after, idx, vals, olds)
    assert st == 0, ("swap", bad)
    # compare_exchange(current = 0): mostly fails on the swapped values, succeeds on zeros
    arr.local_data()[: n_el // 8] = 0
    before = arr.local_numpy().copy()
    idx = rng.integers(0, n_el, m).astype(np.uint64)
    vals = rng.integers(0, 2**32, m, dtype=np.uint64).astype(u32)
    vals[rng.random(m) < 0.1] = 0
    res, ok = arr.batch_compare_exchange(idx, 0, vals).block().numpy()
    after = arr.local_numpy().copy()
    assert ok.any() and (~ok).any()
    st, bad = orc.check_linearizable(1, CODE["u32"], u32, CAS, before, after, idx, vals, res, ok.astype(np.uint8),
                                     current=u32(0))
    assert st == 0, ("compare_exchange", bad)


def zipf_indices(rng, n_el, n, s=0.99):
    ranks = np.arange(1, n_el + 1, dtype=np.float64)
    cdf = np.cumsum(ranks ** -s)
    cdf /= cdf[-1]
    r = np.minimum(np.searchsorted(cdf, rng.random(n)), n_el - 1)
    return rng.permutation(n_el)[r].astype(np.uint64)


def test_c3_twin_zipf_f64_fetch_add(world, orc, lam):
    """Reduced C3 (BASELINE configs[2]): AtomicArray<f64>, fetch_add of 2^22 records,
    Zipf(0.99) ranks (randomly permuted) over 2^20 elements -- a long tail of moderately
    hot tiles, not one hot element. vals = 1.0: exact final state and olds that form one
    serial order per element. Random vals in [0, 1): final state within the float
    tolerance |device - serial| <= m * eps * sum|terms| per element (m = its records)."""
    team = world.team()
    rng = np.random.default_rng(0xC3)
    n_el, n = 1 << 20, 1 << 22
    idx = zipf_indices(rng, n_el, n)
    arr = lam.AtomicArray(team, n_el, lam.Distribution.Block, "f64")
    init = rng.integers(0, 1000, n_el).astype(np.float64)
    arr.local_data().copy_(torch.from_numpy(init).cuda())
    ones = np.ones(n, dtype=np.float64)
    olds = arr.batch_fetch_add(idx, ones).block().cpu().numpy().view(np.float64)
    got = arr.local_numpy().copy()
    exp = init + np.bincount(idx.astype(np.int64), minlength=n_el)
    assert np.array_equal(got, exp)
    st, bad = orc.check_linearizable(2, CODE["f64"], np.float64, FETCH_ADD, init, got, idx, ones, olds)
    assert st == 0, bad
    # random values: tolerance on the final state
    arr.local_data().copy_(torch.from_numpy(init).cuda())
    vals = rng.random(n)
    arr.batch_fetch_add(idx, vals).block()
    got = arr.local_numpy().astype(np.float64)
    exp = init.copy()
    np.add.at(exp, idx.astype(np.int64), vals)
    m = np.bincount(idx.astype(np.int64), minlength=n_el)
    mag = np.abs(init).astype(np.float64)
    np.add.at(mag, idx.astype(np.int64), np.abs(vals))
    tol = m * np.finfo(np.float64).eps * mag + np.finfo(np.float64).tiny
    assert np.all(np.abs(got - exp) <= tol)
