"""Small-batch ordering contract: a buffer that is one reference AM is applied per element
in buffer order, so order-dependent ops give exactly the reference's result.

The reference's apply AM walks its op buffer sequentially (impl/src/array_ops.rs:203-250),
and at 1 PE every batch below 1000 records is one OpInput chunk (src/array/operations.rs:
462-469) that fits one AM (unsafe/operations.rs:679-681): `batch_swap([5, 5], [1, 2])`
deterministically leaves 2 and returns [old, 1]. The device applies such batches with
LMR_STRATEGY_ORDERED (AUTO below 1000 records; any size on request): per element in
record order, as one atomic block. Larger batches keep the unordered (linearisable)
contract, checked in test_gpu_linearize.py.

Bar: bit-exact against the oracle's sequential apply -- final state, fetch values, Ok
flags -- for every op and type, floats included, on colliding indices.
"""
import numpy as np
import pytest

from opgen import (CAS, CAS_EPS, CODE, DTYPE_NAMES, IS_FLOAT, NP, STORE, SWAP, bits_equal,
                   ops_for, rand_elems, rand_vals)
from test_gpu_parity import Case, KIND_LOCAL_LOCK, kind_for

pytestmark = pytest.mark.gpu

AUTO, ORDERED = 0, 3


def colliding(dt, op, rng, shard_len, n):
    t = NP[dt]
    shard0 = rand_elems(dt, shard_len, rng, op)
    idx = rng.integers(0, max(1, shard_len // 4), n).astype(np.uint64)   # ~4n/shard_len records per element
    vals = rand_vals(dt, n, rng, op)
    cur = eps = None
    if op in (CAS, CAS_EPS):
        cur = t(3) if not IS_FLOAT[dt] else t(3.0)
        eps = t(2) if not IS_FLOAT[dt] else t(0.5)
        shard0[rng.random(shard_len) < 0.5] = cur
        vals[rng.random(n) < 0.3] = cur
    return shard0, idx, vals, cur, eps


def check_exact(c, what):
    assert c.err == 0 and c.st_o == 0, (what, c.err, c.st_o)
    assert bits_equal(c.got, c.ref), (what, "state")
    if c.rk:
        assert bits_equal(c.res_d, c.res_o), (what, "results")
    if c.rk == 2:
        assert np.array_equal(c.ok_d, c.ok_o), (what, "ok")


@pytest.mark.parametrize("shape", ["soa", "aos", "svmi"])
@pytest.mark.parametrize("dt", DTYPE_NAMES)
def test_small_batch_in_buffer_order(world, orc, lam, dt, shape):
    """AUTO, 999 colliding records (one reference AM): every op bit-exact against the
    sequential oracle, including swap / store / compare_exchange(_epsilon) / rem / floats."""
    k = world.team().kernels
    rng = np.random.default_rng(303 + CODE[dt])
    for op in ops_for(dt):
        shard0, idx, vals, cur, eps = colliding(dt, op, rng, 400, 999)
        if shape == "svmi":
            vals[:] = vals[0]
        kinds = [kind_for(dt)] + ([KIND_LOCAL_LOCK] if op == CAS_EPS else [])
        for kind in kinds:
            c = Case(k, orc, lam, dt, op, shard0, idx, vals, shape, AUTO, kind=kind, cur=cur, eps=eps)
            check_exact(c, (dt, op, shape, kind))


@pytest.mark.parametrize("n", [1025, 6250, 100000, 1 << 20])
@pytest.mark.parametrize("dt", ["u64", "u8", "i32", "f32", "f64"])
def test_ordered_strategy_large_buffers(world, orc, lam, dt, n):
    """LMR_STRATEGY_ORDERED on buffers above one workgroup (sort by index, then each
    element's run in input order): one AM of 6250 16-B records, 100000 u8-indexed records,
    and 2^20 records -- bit-exact against the sequential oracle."""
    k = world.team().kernels
    rng = np.random.default_rng(404 + CODE[dt] + n)
    ops = [1, SWAP, STORE, CAS_EPS if IS_FLOAT[dt] else CAS, 9, 5]      # fetch_add, swap, store, cas, fetch_rem, fetch_mul
    for op in ops:
        shard0, idx, vals, cur, eps = colliding(dt, op, rng, max(64, n // 8), n)
        if IS_FLOAT[dt] and op == 5:
            vals = rng.choice(np.array([0.5, 2.0, -1.0, 1.25], dtype=NP[dt]), n)
        c = Case(k, orc, lam, dt, op, shard0, idx, vals, "aos" if n == 6250 else "soa", ORDERED, cur=cur, eps=eps)
        check_exact(c, (dt, op, n))


def test_ordered_errors_and_oob(world, orc, lam):
    """Records that panic in the reference (div by zero, out of bounds) are skipped with the
    error bit raised; the rest of the element's records still apply in order."""
    k = world.team().kernels
    rng = np.random.default_rng(9)
    for n in (500, 5000):
        shard0 = rng.integers(1, 1000, 64).astype(np.int32)
        idx = rng.integers(0, 64, n).astype(np.uint64)
        vals = rng.integers(1, 4, n).astype(np.int32)
        vals[rng.random(n) < 0.05] = 0                   # division by zero
        c = Case(k, orc, lam, "i32", 7, shard0, idx, vals, "soa", ORDERED)   # fetch_div
        assert c.err & 0x2
        good = vals != 0
        ref = shard0.copy()
        L = orc.layout_new(64, 1, 0, 0)
        st, res_o, _ = orc.batch_op(L, [ref], 1, CODE["i32"], np.int32, 7, idx[good], vals[good])
        assert st == 0
        assert np.array_equal(c.got, ref)
        assert np.array_equal(c.res_d[good], res_o)
        idx2 = idx.copy()
        idx2[::97] = 64 + 5                              # out of bounds
        c = Case(k, orc, lam, "i32", 18, shard0, idx2, vals, "soa", ORDERED)  # swap
        assert c.err & 0x1
        keep = idx2 < 64
        ref = shard0.copy()
        st, res_o, _ = orc.batch_op(L, [ref], 1, CODE["i32"], np.int32, 18, idx2[keep], vals[keep])
        assert np.array_equal(c.got, ref) and np.array_equal(c.res_d[keep], res_o)


def test_array_api_small_batches_deterministic(world, lam):
    """Through the op-builder API at 1 PE (AUTO): the reference's deterministic outcomes."""
    team = world.team()
    a = lam.AtomicArray(team, 16, lam.Distribution.Block, "u64")
    a.fill(7)
    olds = a.batch_swap([5, 5], [1, 2]).block().cpu().numpy().view(np.uint64)
    assert list(olds) == [7, 1] and int(a.local_numpy()[5]) == 2
    a.batch_store([3, 3, 3], [10, 20, 30]).block()
    assert int(a.local_numpy()[3]) == 30
    res, ok = a.batch_compare_exchange([4, 4, 4], 7, [8, 9, 7]).block().numpy()
    assert list(ok) == [True, False, False] and list(res) == [7, 8, 8] and int(a.local_numpy()[4]) == 8
    f = lam.AtomicArray(team, 4, lam.Distribution.Block, "f64")
    vals = [1e16, 1.0, -1e16, 1.0]                        # order-dependent rounding
    olds = f.batch_fetch_add([0, 0, 0, 0], vals).block().cpu().numpy().view(np.float64)
    s = 0.0
    exp = []
    for v in vals:
        exp.append(s)
        s = s + v
    assert list(olds) == exp and float(f.local_numpy()[0]) == s
    r = a.batch_rem([2, 2], [5, 3]).block()
    assert r is None


@pytest.mark.parametrize("dt,op", [("u64", SWAP), ("f64", 1), ("i32", CAS)])
def test_ordered_apply_in_pieces(world, orc, lam, dt, op):
    """An ordered stream longer than the reserved sort capacity (2^22 records) runs piece after
    piece; every record of a piece is applied before any of the next, so each element still
    sees its records in input order: bit-exact against the sequential oracle, including the
    records of an element that straddle the piece boundary."""
    k = world.team().kernels
    rng = np.random.default_rng(505 + CODE[dt])
    n = (1 << 22) + 4099
    shard0, idx, vals, cur, eps = colliding(dt, op, rng, 1 << 16, n)
    if dt == "f64":
        vals = rng.random(n) * 8.0 - 4.0                   # inexact sums: the order shows in the bits
    c = Case(k, orc, lam, dt, op, shard0, idx, vals, "soa", ORDERED, cur=cur, eps=eps)
    check_exact(c, (dt, op, n))
