"""Device parity: liblamellar_gpu_ops.so (through the C ABI) vs the CPU oracle.

Bar: bit-exact for every integer op; for f32/f64 bit-exact where each element
sees one record (conflict-free streams), and within a stated relative bound
where records collide (float addition is not associative).
"""
import numpy as np
import pytest
import torch

from opgen import (ADD, AND, CAS, CAS_EPS, CODE, COMMUTATIVE_INT, DIV, DTYPE_NAMES, FETCH_ADD,
                   FETCH_SUB, IS_FLOAT, MUL, NP, OR, REM, SUB, XOR, bits_equal, cas_operands,
                   ops_for, rand_elems, rand_vals, ret_kind, to_aos)

pytestmark = pytest.mark.gpu

KIND_NATIVE, KIND_GENERIC, KIND_LOCAL_LOCK, KIND_UNSAFE = 1, 2, 3, 0


def kind_for(dt):
    return KIND_GENERIC if IS_FLOAT[dt] else KIND_NATIVE


def to_dev(a):
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(np.uint8).copy()).cuda()


def from_dev(t, dt, n):
    return t[: n * np.dtype(NP[dt]).itemsize].cpu().numpy().view(NP[dt])


class Case:
    """One kernel-level apply: device vs oracle on identical inputs."""

    def __init__(self, k, orc, lam, dt, op, shard0, idx, vals, shape, strategy, kind=None,
                 cur=None, eps=None):
        self.dt, self.op = dt, op
        kind = kind_for(dt) if kind is None else kind
        t = NP[dt]
        n = idx.size if shape != "mvsi" else vals.size
        L = orc.layout_new(shard0.size, 1, 0, 0)
        iw = orc.index_size(L)
        # ---- oracle (sequential, input order) ----
        ref = shard0.copy()
        if shape == "mvsi":
            st_o, res_o, ok_o = orc.apply_mvsi(ref, kind, CODE[dt], t, op, vals, int(idx[0]), cur, eps)
        elif shape == "svmi":
            st_o, res_o, ok_o = orc.batch_op(L, [ref], kind, CODE[dt], t, op, idx, vals[:1], cur, eps)
        else:
            st_o, res_o, ok_o = orc.batch_op(L, [ref], kind, CODE[dt], t, op, idx, vals, cur, eps)
        # ---- device ----
        old_strategy = k.strategy
        k.strategy = strategy
        try:
            dt_obj = lam.dtype_of(dt)
            d_shard = to_dev(shard0)
            eb = np.dtype(t).itemsize
            d_res = torch.zeros(max(n, 1) * eb, dtype=torch.uint8, device="cuda")
            d_ok = torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")
            rk = ret_kind(op)
            res_arg = d_res if rk else None
            ok_arg = d_ok if rk == 2 else None
            cb = dt_obj.to_bits(cur) if cur is not None else 0
            ebits = dt_obj.to_bits(eps) if eps is not None else 0
            if shape == "soa":
                k.apply_soa(d_shard, shard0.size, kind, dt_obj, op, to_dev(idx.astype(np.uint64)), 8,
                            to_dev(vals), 0, n, res_arg, ok_arg, cb, ebits)
            elif shape == "svmi":
                ii = idx.astype({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[iw])
                k.apply_svmi(d_shard, shard0.size, kind, dt_obj, op, dt_obj.to_bits(vals[0]),
                             to_dev(ii), n, iw, res_arg, ok_arg, cb, ebits)
            elif shape == "aos":
                rb, vo = orc.record_bytes(iw, CODE[dt]), orc.record_val_offset(iw, CODE[dt])
                buf = to_aos(idx, vals, iw, dt, rb, vo)
                k.apply_mvmi(d_shard, shard0.size, kind, dt_obj, op, to_dev(buf), buf.size, iw,
                             res_arg, ok_arg, cb, ebits)
            elif shape == "mvsi":
                k.apply_mvsi(d_shard, shard0.size, kind, dt_obj, op, to_dev(vals), n, int(idx[0]),
                             res_arg, ok_arg, cb, ebits)
            k.synchronize()
            self.err = k.errors(clear=True)
        finally:
            k.strategy = old_strategy
        self.st_o = st_o
        self.ref, self.res_o, self.ok_o = ref, res_o, ok_o
        self.got = from_dev(d_shard, dt, shard0.size)
        self.res_d = from_dev(d_res, dt, n) if rk else None
        self.ok_d = d_ok[:n].cpu().numpy() if rk == 2 else None
        self.rk = rk


def _perm_inputs(dt, op, rng, shard_len, n):
    shard0 = rand_elems(dt, shard_len, rng, op)
    idx = rng.permutation(shard_len)[:n].astype(np.uint64)
    vals = rand_vals(dt, n, rng, op)
    cur = eps = None
    if op in (CAS, CAS_EPS):
        cur, eps, shard0 = cas_operands(dt, shard0, vals, rng)
    return shard0, idx, vals, cur, eps


@pytest.mark.parametrize("shape", ["soa", "svmi", "aos"])
@pytest.mark.parametrize("strategy", [1, 2, 3], ids=["direct", "tiled", "staged"])
@pytest.mark.parametrize("dt", DTYPE_NAMES)
def test_apply_conflict_free_bit_exact(world, orc, lam, dt, strategy, shape, monkeypatch):
    """Every op, every type: one record per element -> bit-exact state and results.
    staged: the tiled path through the staged pipeline, each call cut into 3 regions."""
    if strategy == 3:
        monkeypatch.setenv("LMR_STAGED", "1")
        monkeypatch.setenv("LMR_STAGE_SPLIT", "3")
        strategy = 2
    k = world.team().kernels
    k.reserve(1 << 20)
    rng = np.random.default_rng(1234 + CODE[dt])
    for op in ops_for(dt):
        shard0, idx, vals, cur, eps = _perm_inputs(dt, op, rng, 40000, 30000)
        if shape == "svmi" and op in (DIV, REM, 7, 9):
            vals[:] = vals[0]
        c = Case(k, orc, lam, dt, op, shard0, idx, vals, shape, strategy, cur=cur, eps=eps)
        assert c.err == 0 and c.st_o == 0, (dt, op, c.err, c.st_o)
        assert bits_equal(c.got, c.ref), (dt, op, shape, strategy)
        if c.rk:
            assert bits_equal(c.res_d, c.res_o), (dt, op, "results")
        if c.rk == 2:
            assert np.array_equal(c.ok_d, c.ok_o), (dt, op, "ok")


@pytest.mark.parametrize("dt", DTYPE_NAMES)
def test_apply_cas_eps_generic_kind(world, orc, lam, dt):
    """compare_exchange_epsilon on non-native kinds (LocalLock): array_ops.rs:521-535."""
    k = world.team().kernels
    rng = np.random.default_rng(77)
    shard0, idx, vals, cur, eps = _perm_inputs(dt, CAS_EPS, rng, 4096, 3000)
    c = Case(k, orc, lam, dt, CAS_EPS, shard0, idx, vals, "soa", 1, kind=KIND_LOCAL_LOCK, cur=cur, eps=eps)
    assert bits_equal(c.got, c.ref) and bits_equal(c.res_d, c.res_o) and np.array_equal(c.ok_d, c.ok_o)


@pytest.mark.parametrize("dt", DTYPE_NAMES)
def test_apply_mvsi_in_order(world, orc, lam, dt):
    """Many values at one index are applied in buffer order: bit-exact even for floats."""
    k = world.team().kernels
    rng = np.random.default_rng(5 + CODE[dt])
    for op in ops_for(dt):
        shard0 = rand_elems(dt, 64, rng, op)
        vals = rand_vals(dt, 300, rng, op)
        cur = eps = None
        if op in (CAS, CAS_EPS):
            cur, eps, shard0 = cas_operands(dt, shard0, vals, rng)
            shard0[17] = cur
            vals[::3] = cur
        if op in (MUL, 5) and IS_FLOAT[dt]:
            vals = np.abs(vals) * 0 + NP[dt](1.0009765625)
        c = Case(k, orc, lam, dt, op, shard0, np.array([17], dtype=np.uint64), vals, "mvsi", 1,
                 cur=cur, eps=eps)
        assert c.err == 0 and c.st_o == 0
        assert bits_equal(c.got, c.ref), (dt, op)
        if c.rk:
            assert bits_equal(c.res_d, c.res_o), (dt, op)


@pytest.mark.parametrize("strategy", [1, 2], ids=["direct", "tiled"])
@pytest.mark.parametrize("dt", ["u8", "u16", "u32", "u64", "i8", "i16", "i32", "i64"])
def test_apply_collisions_order_independent(world, orc, lam, dt, strategy):
    """Colliding indices: wrapping integer add/sub/mul/and/or/xor give a bit-exact final state."""
    k = world.team().kernels
    k.reserve(1 << 20)
    rng = np.random.default_rng(99 + CODE[dt])
    for op in sorted(COMMUTATIVE_INT):
        shard0 = rand_elems(dt, 5000, rng, op)
        idx = rng.integers(0, 5000, 200000).astype(np.uint64)
        vals = rand_vals(dt, idx.size, rng, op)
        c = Case(k, orc, lam, dt, op, shard0, idx, vals, "soa", strategy)
        assert c.err == 0
        assert bits_equal(c.got, c.ref), (dt, op)


@pytest.mark.parametrize("strategy", [1, 2], ids=["direct", "tiled"])
@pytest.mark.parametrize("dt", ["u32", "u64", "i32", "i64", "u16"])
def test_fetch_add_linearizable(world, orc, lam, dt, strategy):
    """Colliding fetch_add / fetch_sub: per element the returned olds are exactly the
    prefix states of some serial order (each old distinct, chain closes at the final value)."""
    k = world.team().kernels
    k.reserve(1 << 20)
    rng = np.random.default_rng(3)
    t = NP[dt]
    for op in (FETCH_ADD, FETCH_SUB):
        shard0 = rand_elems(dt, 1000, rng)
        idx = rng.integers(0, 1000, 100000).astype(np.uint64)
        vals = np.ones(idx.size, dtype=t)
        c = Case(k, orc, lam, dt, op, shard0, idx, vals, "soa", strategy)
        assert bits_equal(c.got, c.ref)
        # with v = 1 the olds for element e must be {a0, a0±1, ..., a0±(m-1)} (wrapping)
        order = np.lexsort((c.res_d.astype(np.uint64), idx))
        cnt = np.bincount(idx.astype(np.int64), minlength=1000)
        start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
        olds = c.res_d[order]
        step = 1 if op == FETCH_ADD else -1
        for e in np.nonzero(cnt)[0][:200]:
            m = cnt[e]
            got = np.sort(olds[start[e]:start[e] + m].astype(np.uint64))
            exp = np.sort((np.uint64(shard0[e].astype(np.int64).astype(np.uint64))
                           + np.arange(m, dtype=np.int64).astype(np.uint64) * np.uint64(step & 0xFFFFFFFFFFFFFFFF))
                          .astype(t).astype(np.uint64))
            assert np.array_equal(got, exp), (dt, op, e)


@pytest.mark.parametrize("strategy", [1, 2], ids=["direct", "tiled"])
@pytest.mark.parametrize("dt", ["f32", "f64"])
def test_float_add_collisions_tolerance(world, orc, lam, dt, strategy):
    """Colliding float adds: exact with exactly representable values (1.0); random
    values within |err| <= m * eps_mach * sum|terms| per element (m = updates)."""
    k = world.team().kernels
    k.reserve(1 << 20)
    rng = np.random.default_rng(11)
    t = NP[dt]
    shard0 = np.zeros(3000, dtype=t)
    idx = rng.integers(0, 3000, 120000).astype(np.uint64)
    c = Case(k, orc, lam, dt, ADD, shard0, idx, np.ones(idx.size, dtype=t), "soa", strategy)
    assert bits_equal(c.got, c.ref)
    vals = rng.uniform(-1, 1, idx.size).astype(t)
    c = Case(k, orc, lam, dt, ADD, shard0, idx, vals, "soa", strategy)
    m = np.bincount(idx.astype(np.int64), minlength=3000)
    mag = np.zeros(3000)
    np.add.at(mag, idx.astype(np.int64), np.abs(vals.astype(np.float64)))
    tol = m * np.finfo(t).eps * mag + np.finfo(t).tiny
    assert np.all(np.abs(c.got.astype(np.float64) - c.ref.astype(np.float64)) <= tol)


def test_pack_matches_oracle(world, orc, lam):
    """lmr_pack: per-PE record streams == concatenation of the reference's op buffers."""
    k = world.team().kernels
    rng = np.random.default_rng(21)
    import ctypes
    from lamellar_runtime_amd import _capi
    for npes, dist, size, sub in [(2, 0, 1000, None), (3, 1, 997, None), (4, 0, 100003, None),
                                  (8, 1, 65536 * 3 + 5, None), (4, 0, 5000, (123, 4000)),
                                  (3, 1, 5000, (7, 4444)), (8, 0, 7, None), (5, 0, 300000, None)]:
        Lo = orc.layout_new(size, npes, 0, dist)
        Ld = _capi.lmr_layout_t()
        _capi.lib().lmr_layout_new(ctypes.byref(Ld), size, npes, 0, dist)
        if sub:
            Lo = orc.layout_sub(Lo, *sub)
            Ld2 = _capi.lmr_layout_t()
            _capi.lib().lmr_layout_sub(ctypes.byref(Ld), sub[0], sub[1], ctypes.byref(Ld2))
            Ld = Ld2
        assert Lo.as_tuple() == Ld.as_tuple()
        n_len = Lo.size
        iw = orc.index_size(Lo)
        gidx = rng.integers(0, n_len, 20000).astype(np.uint64)
        vals = rng.integers(0, 2**63, 20000).astype(np.uint64)
        st, ams = orc.pack(Lo, CODE["u64"], np.uint64, gidx, vals, iw)
        assert st == 0
        dt_obj = lam.dtype_of("u64")
        out_idx, out_vals, out_pos, counts = k.pack(Ld, to_dev(gidx).view(torch.int64), gidx.size,
                                                    to_dev(vals), dt_obj, iw)
        k.synchronize()
        counts = counts.cpu().numpy()
        oi = out_idx.cpu().numpy().view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[iw])
        ov = out_vals.cpu().numpy().view(np.uint64)
        op_ = out_pos.cpu().numpy().view(np.uint32)
        off = 0
        rb, vo = orc.record_bytes(iw, CODE["u64"]), orc.record_val_offset(iw, CODE["u64"])
        from opgen import record_dtype
        for p in range(npes):
            recs = [a for a in ams if a[0] == p]
            if recs:
                b = np.concatenate([a[1] for a in recs]).view(record_dtype(iw, "u64", rb, vo))
                pos = np.concatenate([a[2] for a in recs])
            else:
                b = np.zeros(0, dtype=record_dtype(iw, "u64", rb, vo))
                pos = np.zeros(0, dtype=np.uint64)
            assert counts[p] == b.size
            assert np.array_equal(oi[off:off + b.size], b["i"]), (npes, dist, p)
            assert np.array_equal(ov[off:off + b.size], b["v"])
            assert np.array_equal(op_[off:off + b.size].astype(np.uint64), pos)
            off += b.size
        assert k.errors() == 0


def test_pack_unordered_matches_oracle_per_pe(world, orc, lam):
    """lmr_pack_unordered: same per-PE record sets as the reference's op buffers
    (order inside a PE free; each record keeps its input position)."""
    k = world.team().kernels
    rng = np.random.default_rng(22)
    import ctypes
    from lamellar_runtime_amd import _capi
    from opgen import record_dtype
    for npes, dist, size, nrec, dt in [(2, 0, 1000, 20000, "u64"), (3, 1, 997, 20000, "u32"),
                                       (8, 0, 1 << 20, 300000, "u64"), (8, 1, 65536 * 3 + 5, 100000, "u16"),
                                       (5, 0, 300000, 70000, "f64"), (128, 1, 1 << 22, 200000, "u8"),
                                       (200, 0, 1 << 20, 50000, "u64"), (7, 0, 7, 1000, "i32")]:
        Lo = orc.layout_new(size, npes, 0, dist)
        Ld = _capi.lmr_layout_t()
        _capi.lib().lmr_layout_new(ctypes.byref(Ld), size, npes, 0, dist)
        iw = orc.index_size(Lo)
        npt = NP[dt]
        gidx = rng.integers(0, size, nrec).astype(np.uint64)
        vals = rng.integers(0, 120, nrec).astype(npt)
        st, ams = orc.pack(Lo, CODE[dt], npt, gidx, vals, iw)
        assert st == 0
        dt_obj = lam.dtype_of(dt)
        for with_vals in (True, False):
            out_idx, out_vals, out_pos, counts = k.pack(Ld, to_dev(gidx).view(torch.int64), nrec,
                                                        to_dev(vals) if with_vals else None, dt_obj, iw,
                                                        stable=False)
            k.synchronize()
            counts = counts.cpu().numpy()
            oi = out_idx.cpu().numpy().view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[iw])
            ov = out_vals.cpu().numpy().view(npt) if with_vals else None
            op_ = out_pos.cpu().numpy().view(np.uint32)
            rb, vo = orc.record_bytes(iw, CODE[dt]), orc.record_val_offset(iw, CODE[dt])
            off = 0
            for p in range(npes):
                recs = [a for a in ams if a[0] == p]
                c = int(sum(len(a[2]) for a in recs))
                assert counts[p] == c, (npes, p)
                if c == 0:
                    continue
                b = np.concatenate([a[1] for a in recs]).view(record_dtype(iw, dt, rb, vo))
                pos = np.concatenate([a[2] for a in recs])
                order = np.argsort(op_[off:off + c], kind="stable")
                assert np.array_equal(op_[off:off + c][order].astype(np.uint64), pos), (npes, dist, p)
                assert np.array_equal(oi[off:off + c][order], b["i"]), (npes, dist, p)
                if with_vals:
                    assert np.array_equal(ov[off:off + c][order], b["v"])
                off += c
            assert off == nrec
        assert k.errors() == 0


def test_scatter_results(world):
    k = world.team().kernels
    rng = np.random.default_rng(2)
    for eb, t in ((1, np.uint8), (2, np.uint16), (4, np.uint32), (8, np.uint64)):
        n = 5000
        pos = rng.permutation(n).astype(np.uint32)
        vals = rng.integers(0, 200, n).astype(t)
        ok = rng.integers(0, 2, n).astype(np.uint8)
        out = torch.zeros(n * eb, dtype=torch.uint8, device="cuda")
        ook = torch.zeros(n, dtype=torch.uint8, device="cuda")
        k.scatter_results(to_dev(vals), to_dev(pos), n, eb, out, to_dev(ok), ook)
        k.synchronize()
        exp = np.zeros(n, dtype=t)
        exp[pos] = vals
        eok = np.zeros(n, dtype=np.uint8)
        eok[pos] = ok
        assert np.array_equal(out.cpu().numpy().view(t), exp)
        assert np.array_equal(ook.cpu().numpy(), eok)


@pytest.mark.parametrize("strategy", [1, 2], ids=["direct", "tiled"])
def test_device_errors(world, lam, strategy):
    """Where Rust panics the device raises the matching error bit and skips the record."""
    k = world.team().kernels
    k.reserve(1 << 20)
    old = k.strategy
    k.strategy = strategy
    try:
        dt = lam.dtype_of("i32")
        shard = to_dev(np.array([10, -2**31, 5, 6], dtype=np.int32))
        k.apply_soa(shard, 4, 1, dt, DIV, to_dev(np.array([0, 2], np.uint64)), 8,
                    to_dev(np.array([0, 1], np.int32)), 0, 2)
        assert k.errors() == 0x2
        k.apply_soa(shard, 4, 1, dt, REM, to_dev(np.array([1], np.uint64)), 8,
                    to_dev(np.array([-1], np.int32)), 0, 1)
        assert k.errors() == 0x4
        k.apply_soa(shard, 4, 1, dt, ADD, to_dev(np.array([4, 1 << 40], np.uint64)), 8,
                    to_dev(np.array([1, 1], np.int32)), 0, 2)
        assert k.errors() == 0x1
        got = shard.cpu().numpy().view(np.int32)
        assert list(got[:4]) == [10, -2**31, 5, 6]   # nothing applied
        with pytest.raises(lam.LamellarError):
            k.apply_soa(shard, 4, 2, lam.dtype_of("f32"), XOR, to_dev(np.array([0], np.uint64)), 8,
                        to_dev(np.array([1], np.float32)), 0, 1)
    finally:
        k.strategy = old


@pytest.fixture(params=["count", "free", "staged"])
def partition(request, monkeypatch):
    """Two-level partition variant: count pass + bucket-major temp ("count"), the
    staged pipeline (coarse pass, then fixed-size pieces counted and sorted by tile)
    with every call cut into 3 regions applied in one sweep ("staged"), or the default
    selection, where order-insensitive integer ops that return nothing take the
    count-free partition ("free"; "count" switches it off)."""
    monkeypatch.setenv("LMR_FREE", "0" if request.param == "count" else "1")
    monkeypatch.setenv("LMR_STAGED", "0")          # the segment-based fine pass unless "staged"
    if request.param == "staged":
        monkeypatch.setenv("LMR_STAGED", "1")
        monkeypatch.setenv("LMR_STAGE_SPLIT", "3")
    return request.param


@pytest.mark.parametrize("dt", ["u64", "u32", "u8", "i16", "i64", "f32", "f64"])
def test_tiled_two_level_partition_bit_exact(world, orc, lam, dt, partition):
    """> 128 tiles: coarse + fine LDS-staged partition before the tile apply."""
    k = world.team().kernels
    k.reserve(1 << 21)
    rng = np.random.default_rng(4321 + CODE[dt])
    shard_len = (1 << 21) + 1234
    for op in ops_for(dt):
        shard0, idx, vals, cur, eps = _perm_inputs(dt, op, rng, shard_len, 1 << 20)
        c = Case(k, orc, lam, dt, op, shard0, idx, vals, "soa", 2, cur=cur, eps=eps)
        assert c.err == 0 and c.st_o == 0
        assert bits_equal(c.got, c.ref), (dt, op)
        if c.rk:
            assert bits_equal(c.res_d, c.res_o), (dt, op)
        if c.rk == 2:
            assert np.array_equal(c.ok_d, c.ok_o)


@pytest.mark.parametrize("dt,op", [("u64", ADD), ("i64", XOR), ("u64", FETCH_ADD), ("u32", ADD), ("i64", FETCH_ADD)])
def test_tiled_ragged_batch_lengths(world, orc, lam, dt, op, partition):
    """Odd batch lengths, not a multiple of any LDS round: the coarse pass's paired 16-B
    record loads end on a single record, and the tile apply's 4-record groups start and end
    on unaligned bin ranges (head and tail records one per thread). Colliding streams:
    exact final state (integers) and, for fetch_add with v = 1, exact olds per element."""
    k = world.team().kernels
    k.reserve(1 << 21)
    rng = np.random.default_rng(77 + CODE[dt] + op)
    shard_len = (1 << 21) + 37
    t = NP[dt]
    for n in (1, 3, 65537, (1 << 20) + 777):
        idx = rng.integers(0, shard_len, n).astype(np.uint64)
        shard0 = rand_elems(dt, shard_len, rng, op)
        vals = np.ones(n, dtype=t) if op == FETCH_ADD else rand_vals(dt, n, rng, op)
        c = Case(k, orc, lam, dt, op, shard0, idx, vals, "soa", 2)
        assert c.err == 0 and c.st_o == 0, (dt, op, n)
        assert bits_equal(c.got, c.ref), (dt, op, n)
        if op == FETCH_ADD:                  # olds of an element: base, base + 1, ..., base + m - 1
            olds = c.res_d.view(np.uint64)
            order = np.lexsort((olds, idx))
            si, so = idx[order], olds[order]
            first = np.r_[0, np.flatnonzero(si[1:] != si[:-1]) + 1]
            start = np.repeat(first, np.diff(np.r_[first, n]))
            rank = (np.arange(n) - start).astype(np.uint64)
            assert np.array_equal(so, shard0.view(np.uint64)[si.astype(np.int64)] + rank), (dt, n)


def test_tiled_two_level_collisions(world, orc, lam, partition):
    """Colliding u64 fetch_add over > 128 tiles: exact final state; each element's olds
    are exactly init, init+1, ..., init+m-1 (v = 1)."""
    k = world.team().kernels
    k.reserve(1 << 22)
    rng = np.random.default_rng(8)
    shard_len = (1 << 21) + 5
    shard0 = rng.integers(0, 2**62, shard_len, dtype=np.uint64)
    idx = rng.integers(0, shard_len, 1 << 22).astype(np.uint64)
    vals = np.ones(idx.size, dtype=np.uint64)
    c = Case(k, orc, lam, "u64", FETCH_ADD, shard0, idx, vals, "soa", 2)
    assert bits_equal(c.got, c.ref)
    order = np.lexsort((c.res_d, idx))
    si, so = idx[order], c.res_d[order]
    first = np.ones(si.size, dtype=bool)
    first[1:] = si[1:] != si[:-1]
    grp_start = np.maximum.accumulate(np.where(first, np.arange(si.size), 0))
    rank = np.arange(si.size) - grp_start
    assert np.array_equal(so, shard0[si] + rank.astype(np.uint64))


@pytest.mark.parametrize("dt", ["u64", "i32", "u16", "f64", "f32"])
def test_hot_tile_delta_mode(world, orc, lam, dt, partition):
    """Skewed stream: one element takes ~40 % of all records, so its tile is split into
    delta-mode work items (LDS combine + one global atomic per element per item).
    Integer ops: exact final state, fetch olds a valid chain; floats: exact with 1.0."""
    k = world.team().kernels
    k.reserve(1 << 21)
    rng = np.random.default_rng(17)
    shard_len = 1 << 18
    n = 1 << 20
    idx = rng.integers(0, shard_len, n).astype(np.uint64)
    idx[rng.random(n) < 0.4] = 12345
    t = NP[dt]
    ops = [ADD, FETCH_ADD, SUB, FETCH_SUB] if IS_FLOAT[dt] else \
        [ADD, FETCH_ADD, SUB, FETCH_SUB, AND, 11, OR, 13, XOR, 15]
    for op in ops:
        shard0 = rand_elems(dt, shard_len, rng) if not IS_FLOAT[dt] else np.zeros(shard_len, t)
        vals = np.ones(n, dtype=t) if (IS_FLOAT[dt] or op in (ADD, FETCH_ADD, SUB, FETCH_SUB)) else \
            rand_vals(dt, n, rng, op)
        c = Case(k, orc, lam, dt, op, shard0, idx, vals, "soa", 2)
        assert c.err == 0
        assert bits_equal(c.got, c.ref), (dt, op)
        if op in (FETCH_ADD, FETCH_SUB):
            hot = idx == 12345
            olds = np.sort(c.res_d[hot].astype(np.float64 if IS_FLOAT[dt] else np.int64)
                           if IS_FLOAT[dt] else c.res_d[hot].astype(np.uint64))
            m = int(hot.sum())
            step = 1 if op == FETCH_ADD else -1
            base = shard0[12345]
            exp = (np.array([base]).astype(t)[0] + (np.arange(m) * step).astype(t)) if IS_FLOAT[dt] else \
                (np.uint64(base.astype(np.int64).astype(np.uint64)) +
                 (np.arange(m, dtype=np.int64) * step).astype(np.uint64)).astype(t)
            exp = np.sort(exp.astype(np.float64) if IS_FLOAT[dt] else exp.astype(np.uint64))
            assert np.array_equal(olds, exp), (dt, op)


def test_two_level_out_of_bounds_fetch(world, orc, lam, partition):
    """Out-of-bounds records in a two-level tiled fetch_add: the error bit is raised, every
    in-bounds record is applied exactly once and returns a valid old value, and the
    un-partition never reads a hole (round-major temp slots of dropped records)."""
    k = world.team().kernels
    k.reserve(1 << 21)
    rng = np.random.default_rng(77)
    shard_len = (1 << 21) + 3
    n = 1 << 20
    idx = rng.permutation(shard_len)[:n].astype(np.uint64)
    bad = rng.random(n) < 0.01
    idx[bad] = shard_len + rng.integers(0, 1000, int(bad.sum())).astype(np.uint64)
    shard0 = rng.integers(0, 2**40, shard_len).astype(np.uint64)
    vals = rng.integers(0, 2**20, n).astype(np.uint64)
    d_shard = to_dev(shard0)
    d_res = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
    old = k.strategy
    k.strategy = 2
    try:
        k.apply_soa(d_shard, shard_len, 1, lam.dtype_of("u64"), FETCH_ADD, to_dev(idx), 8, to_dev(vals), 0, n,
                    d_res, None)
        k.synchronize()
        assert k.errors(clear=True) & 1
    finally:
        k.strategy = old
    got = d_shard.cpu().numpy().view(np.uint64)[:shard_len]
    exp = shard0.copy()
    good = ~bad
    exp[idx[good].astype(np.int64)] += vals[good]
    assert np.array_equal(got, exp)
    res = d_res.cpu().numpy().view(np.uint64)
    assert np.array_equal(res[good], shard0[idx[good].astype(np.int64)])


FREE_OPS = [ADD, SUB, MUL, AND, OR, XOR]


@pytest.mark.parametrize("shape", ["soa", "svmi", "aos"])
@pytest.mark.parametrize("dt", ["u64", "i64", "u32", "i32", "u16", "u8", "i8"])
def test_free_partition_collisions_bit_exact(world, orc, lam, dt, shape, monkeypatch):
    """Count-free partition (order-insensitive integer ops, nothing returned): colliding
    records in any order give the oracle's state bit for bit, for array values, one
    scalar value and AoS records, next to the counted partition on the same inputs."""
    k = world.team().kernels
    k.reserve(1 << 22)
    rng = np.random.default_rng(99 + CODE[dt])
    shard_len = (1 << 22) + 777 if NP[dt](0).itemsize >= 4 else (1 << 23) + 777
    n = 1 << 21
    for op in FREE_OPS:
        shard0 = rand_elems(dt, shard_len, rng, op)
        idx = rng.integers(0, shard_len, n).astype(np.uint64)
        vals = rand_vals(dt, n, rng, op)
        if shape == "svmi":
            vals[:] = vals[0]
        for free in ("1", "0"):
            monkeypatch.setenv("LMR_FREE", free)
            c = Case(k, orc, lam, dt, op, shard0, idx, vals, shape, 2)
            assert c.err == 0 and c.st_o == 0, (dt, op, free)
            assert bits_equal(c.got, c.ref), (dt, op, shape, free)


@pytest.mark.parametrize("dt", ["u64", "u16"])
def test_free_partition_bucket_overflow_spills(world, orc, lam, dt, monkeypatch):
    """Records concentrated on one coarse bucket (128 tiles) overflow its region in the
    count-free partition: the records that find the region full are applied at once with
    device atomics (spill), the rest through the tiles, and the state is still the
    oracle's. The batch holds at least twice the region, so the spill surely runs (the
    region size follows the reserved workspace, which earlier tests may have grown). Also
    a batch split over two buckets and one with 1 % out-of-bounds records (error bit
    raised, the rest applied)."""
    monkeypatch.setenv("LMR_FREE", "1")
    k = world.team().kernels
    k.reserve(1 << 22)
    R = k.reserved
    rng = np.random.default_rng(5)
    t = NP[dt]
    tile = 8192 if t(0).itemsize == 8 else 16384
    shard_len = 640 * tile + 3                     # 641 tiles: 6 coarse buckets
    C = 6
    capc = (2 * R + R // 4 + 128 * 8192) // C       # one coarse bucket's region of the temp arrays
    n = min(max(1 << 21, 2 * capc + 4096), R)
    assert n >= 2 * capc, "workspace too large for a forced spill"
    shard0 = rand_elems(dt, shard_len, rng, ADD)
    cases = [rng.integers(0, 128 * tile, n),                                   # all in bucket 0
             np.where(rng.random(n) < 0.5, rng.integers(0, 50, n),
                      rng.integers(5 * 128 * tile, shard_len, n)),              # buckets 0 and 5
             rng.integers(0, shard_len, n)]                                     # uniform
    for j, idx in enumerate(cases):
        idx = idx.astype(np.uint64)
        vals = rand_vals(dt, n, rng, ADD)
        c = Case(k, orc, lam, dt, ADD, shard0, idx, vals, "soa", 2)
        assert c.err == 0 and c.st_o == 0, j
        assert bits_equal(c.got, c.ref), (dt, j)
    # out-of-bounds records
    idx = rng.integers(0, shard_len, n).astype(np.uint64)
    bad = rng.random(n) < 0.01
    idx[bad] = shard_len + rng.integers(0, 99, int(bad.sum())).astype(np.uint64)
    vals = rand_vals(dt, n, rng, ADD)
    d_shard = to_dev(shard0)
    old = k.strategy
    k.strategy = 2
    try:
        k.apply_soa(d_shard, shard_len, 1, lam.dtype_of(dt), ADD, to_dev(idx), 8, to_dev(vals), 0, n, None, None)
        k.synchronize()
        assert k.errors(clear=True) & 1
    finally:
        k.strategy = old
    exp = shard0.copy()
    good = ~bad
    np.add.at(exp, idx[good].astype(np.int64), vals[good])
    assert bits_equal(from_dev(d_shard, dt, shard_len), exp)


@pytest.mark.parametrize("dt", ["u64", "u32", "u16", "i8", "f64", "f32"])
def test_staged_session_regions(world, orc, lam, dt):
    """lmr_stage_*: several record streams of one op staged as regions (array values,
    a scalar value, out-of-bounds records, one stream below the tiled threshold that is
    applied at once) and applied in one sweep; final shard, per-stream results in
    arrival order and the OOB error bit against the oracle (conflict-free: bit-exact)."""
    k = world.team().kernels
    k.reserve(1 << 21)
    rng = np.random.default_rng(606 + CODE[dt])
    t = NP[dt]
    shard_len = (1 << 20) + 77
    dt_obj = lam.dtype_of(dt)
    eb = np.dtype(t).itemsize
    for op in (FETCH_ADD, ADD, 18, CAS if not IS_FLOAT[dt] else CAS_EPS):
        shard0, _, _, cur, eps = _perm_inputs(dt, op, rng, shard_len, 10)
        perm = rng.permutation(shard_len)
        sizes = [300000, 70000, 1000, 200000]
        streams, o = [], 0
        for j, m in enumerate(sizes):
            idx = perm[o:o + m].astype(np.uint64)
            o += m
            vals = rand_vals(dt, m, rng, op)
            if op in (CAS, CAS_EPS):
                vals = rand_vals(dt, m, rng, 18)
            scalar = (j == 1)
            if scalar:
                vals[:] = vals[0]
            if j == 3:                                     # a few out-of-bounds records
                idx[rng.random(m) < 0.01] = shard_len + 5
            streams.append((idx, vals, scalar))
        # oracle: streams in order (conflict-free across streams)
        ref = shard0.copy()
        L = orc.layout_new(shard_len, 1, 0, 0)
        exp = []
        for idx, vals, scalar in streams:
            good = idx < shard_len
            st, res, okk = orc.batch_op(L, [ref], kind_for(dt), CODE[dt], t, op, idx[good], vals[good], cur, eps)
            assert st == 0
            exp.append((good, res, okk))
        d_shard = to_dev(shard0)
        rk = ret_kind(op)
        cb = dt_obj.to_bits(cur) if cur is not None else 0
        ebits = dt_obj.to_bits(eps) if eps is not None else 0
        outs = []
        k.stage_begin(d_shard, shard_len, kind_for(dt), dt_obj, op, cb, ebits)
        for idx, vals, scalar in streams:
            m = idx.size
            d_res = torch.zeros(m * eb, dtype=torch.uint8, device="cuda") if rk else None
            d_ok = torch.zeros(m, dtype=torch.uint8, device="cuda") if rk == 2 else None
            if scalar:
                k.stage_soa(to_dev(idx), 8, None, dt_obj.to_bits(vals[0]), m, d_res, d_ok)
            else:
                k.stage_soa(to_dev(idx), 8, to_dev(vals), 0, m, d_res, d_ok)
            outs.append((d_res, d_ok))
        k.stage_finish()
        k.synchronize()
        assert k.errors(clear=True) == 1, (dt, op)
        assert bits_equal(from_dev(d_shard, dt, shard_len), ref), (dt, op)
        for (good, res, okk), (d_res, d_ok), (idx, _, _) in zip(exp, outs, streams):
            if rk:
                got = from_dev(d_res, dt, idx.size)[good]
                assert bits_equal(got, res), (dt, op, "results")
            if rk == 2:
                assert np.array_equal(d_ok[:idx.size].cpu().numpy()[good], okk), (dt, op, "ok")


def test_staged_session_collisions_many_regions(world, orc, lam):
    """40 colliding u64 fetch_add streams (more than the 32-region table and the
    reserved workspace hold: staged records are applied in several sweeps): exact final
    state; per element the olds are exactly init, init+1, ... (v = 1)."""
    k = world.team().kernels
    k.reserve(1 << 21)
    rng = np.random.default_rng(31)
    shard_len = (1 << 19) + 3
    shard0 = rng.integers(0, 2**60, shard_len, dtype=np.uint64)
    d_shard = to_dev(shard0)
    dt_obj = lam.dtype_of("u64")
    k.stage_begin(d_shard, shard_len, 1, dt_obj, FETCH_ADD)
    idxs, outs = [], []
    for j in range(40):
        m = 70000 + 1000 * j
        idx = rng.integers(0, shard_len, m).astype(np.uint64)
        d_res = torch.zeros(m * 8, dtype=torch.uint8, device="cuda")
        k.stage_soa(to_dev(idx), 8, None, 1, m, d_res, None)
        idxs.append(idx)
        outs.append(d_res)
    k.stage_finish()
    k.synchronize()
    assert k.errors(clear=True) == 0
    idx = np.concatenate(idxs)
    res = np.concatenate([o.cpu().numpy().view(np.uint64) for o in outs])
    exp = shard0.copy()
    np.add.at(exp, idx.astype(np.int64), np.uint64(1))
    assert np.array_equal(d_shard.cpu().numpy().view(np.uint64)[:shard_len], exp)
    order = np.lexsort((res, idx))
    si, so = idx[order], res[order]
    first = np.ones(si.size, dtype=bool)
    first[1:] = si[1:] != si[:-1]
    grp_start = np.maximum.accumulate(np.where(first, np.arange(si.size), 0))
    rank = np.arange(si.size) - grp_start
    assert np.array_equal(so, shard0[si] + rank.astype(np.uint64))


@pytest.mark.parametrize("dt,op", [("u64", ADD), ("i32", XOR), ("u8", MUL), ("i64", SUB)])
def test_staged_free_session_spill_and_flush(world, orc, lam, dt, op):
    """Count-free staged regions (order-insensitive integer op, nothing returned):
    colliding streams, the first ones all on one coarse bucket until twice its region's
    records are staged (the rest of them are applied at once by device atomics: spill),
    more records than the workspace holds (staged records applied in several sweeps),
    one scalar-valued stream; exact final state against numpy's unbuffered ufunc.at."""
    k = world.team().kernels
    k.reserve(1 << 20)
    R = k.reserved                                   # the workspace only grows: earlier tests may hold more
    rng = np.random.default_rng(404 + CODE[dt])
    t = NP[dt]
    shard_len = (1 << 22) + 5
    tile = 8192 if t(0).itemsize == 8 else 16384
    C = -(-(-(-shard_len // tile)) // 128)
    capc = (2 * R + R // 4 + 128 * 8192) // C       # a coarse bucket's region (temp-array headroom)
    m = 150000
    n_skew = -(-2 * capc // m)                       # twice what bucket 0's region holds
    n_all = max(n_skew + 8, R // m + 4)              # more than the workspace: several sweeps
    shard0 = rand_elems(dt, shard_len, rng, op)
    d_shard = to_dev(shard0)
    dt_obj = lam.dtype_of(dt)
    k.stage_begin(d_shard, shard_len, KIND_NATIVE, dt_obj, op)
    exp = shard0.copy()
    ufunc = {ADD: np.add, SUB: np.subtract, XOR: np.bitwise_xor, MUL: np.multiply}[op]
    for j in range(n_all):
        hi = 128 * tile if j < n_skew else shard_len
        idx = rng.integers(0, hi, m).astype(np.uint64)
        vals = rand_vals(dt, m, rng, op)
        if j == n_skew + 1:
            vals[:] = vals[0]
            k.stage_soa(to_dev(idx), 8, None, dt_obj.to_bits(vals[0]), m, None, None)
        else:
            k.stage_soa(to_dev(idx), 8, to_dev(vals), 0, m, None, None)
        with np.errstate(over="ignore"):
            ufunc.at(exp, idx.astype(np.int64), vals)
    k.stage_finish()
    k.synchronize()
    assert k.errors(clear=True) == 0
    assert bits_equal(from_dev(d_shard, dt, shard_len), exp), (dt, op)
