"""Float special values on every float apply path: NaN, +-inf, +-0.0, subnormals, the
largest finites.

The reference's f32/f64 arrays are GenericAtomic: each record is a plain IEEE RMW under a
per-element mutex (impl/src/array_ops.rs:482-535, generic_atomic.rs:286-293): `+=`, `-=`,
`*=`, `/=`, `%` (fmod), swap, store, and compare_exchange_epsilon's `|a - current| < eps`.
So subnormals are kept, NaN propagates and -0.0 + -0.0 = -0.0. The device adds through
hardware FP atomics (global `unsafeAtomicAdd` on the direct path, LDS `ds_add_rtn_f32/f64`
in the tile kernel, an identity-initialised LDS delta tile plus one device atomic per
element for hot tiles), built with -munsafe-fp-atomics; these tests pin what they do.

Bar: bit-exact against the oracle, NaN-aware -- any NaN matches any NaN. A NaN's sign and
payload are not part of the contract: x86 SSE (where the reference runs) makes a negative
default NaN for inf - inf, gfx950 a positive one.

* conflict-free: every (element special, record special) pair, one record per element;
  final state, fetch results and Ok flags -- direct, one-level tiled, two-level tiled and
  staged paths; MVSI (values applied in buffer order at one index).
* colliding: element classes whose outcome is the same in every order -- subnormal
  multiples (exact), -0.0 chains, +inf absorbing finite values, +inf meets -inf (NaN),
  NaN absorbing everything, overflow of positive values to +inf -- add / sub / fetch_add /
  fetch_sub / swap, on the same paths plus delta mode (one hot subnormal element takes
  40 % of the records, so its tile is split into delta work items). Delta pieces sum their
  records in an LDS tile initialised with -0.0, the identity of IEEE addition (+0.0 would
  turn -0.0 + -0.0 into +0.0), and a float sub piece sums -v: a - v is a + (-v) bit for bit.
"""
import numpy as np
import pytest

from opgen import (ADD, CAS_EPS, CODE, DIV, FETCH_ADD, FETCH_DIV, FETCH_MUL, FETCH_REM, FETCH_SUB,
                   LOAD, MUL, NP, REM, STORE, SUB, SWAP)
from test_gpu_parity import Case, KIND_GENERIC, KIND_LOCAL_LOCK

pytestmark = pytest.mark.gpu

TILE = {4: 16384, 8: 8192}
PATHS = ["direct", "tiled1", "tiled2", "staged"]


def specials(t):
    fi = np.finfo(t)
    tiny_sub = fi.smallest_subnormal
    vals = [np.nan, np.inf, -np.inf, 0.0, -0.0, tiny_sub, -tiny_sub, tiny_sub * 3, fi.tiny - tiny_sub,
            -(fi.tiny - tiny_sub) / 2, fi.tiny, fi.max, -fi.max, 1.0, -1.5, 3.0]
    return np.array(vals, dtype=t)


def nan_aware_equal(a, b):
    """Bit-exact, except that any NaN matches any NaN."""
    a, b = np.asarray(a), np.asarray(b)
    u = {4: np.uint32, 8: np.uint64}[a.dtype.itemsize]
    both_nan = np.isnan(a) & np.isnan(b)
    return bool(np.all((a.view(u) == b.view(u)) | both_nan))


def first_mismatch(a, b):
    u = {4: np.uint32, 8: np.uint64}[a.dtype.itemsize]
    bad = np.flatnonzero(~((a.view(u) == b.view(u)) | (np.isnan(a) & np.isnan(b))))
    return None if bad.size == 0 else (int(bad[0]), a[bad[0]], b[bad[0]], int(bad.size))


def _setup_path(path, monkeypatch):
    monkeypatch.setenv("LMR_STAGED", "1" if path == "staged" else "0")
    monkeypatch.setenv("LMR_STAGE_SPLIT", "2")
    return 1 if path == "direct" else 2


def _shard_len(path, eb):
    if path == "tiled1":
        return 3 * TILE[eb] + 11            # <= 128 tiles: one-level partition
    if path == "direct":
        return 70001
    return 129 * TILE[eb] + 77              # > 128 tiles: two-level partition


CF_OPS = [ADD, FETCH_ADD, SUB, FETCH_SUB, MUL, FETCH_MUL, DIV, FETCH_DIV, REM, FETCH_REM, STORE, LOAD, SWAP]


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("dt", ["f32", "f64"])
def test_specials_conflict_free(world, orc, lam, dt, path, monkeypatch):
    k = world.team().kernels
    k.reserve(1 << 20)
    strategy = _setup_path(path, monkeypatch)
    t = NP[dt]
    eb = t(0).itemsize
    S = specials(t)
    rng = np.random.default_rng(1000 + CODE[dt] + 7 * PATHS.index(path))
    shard_len = _shard_len(path, eb)
    pa, pb = np.meshgrid(np.arange(S.size), np.arange(S.size), indexing="ij")
    pa, pb = pa.ravel(), pb.ravel()
    reps = max(1, min(shard_len // 2, 1 << 16) // pa.size)
    ea, vb = np.tile(S[pa], reps), np.tile(S[pb], reps)     # every pair, `reps` times
    n = ea.size
    idx = rng.permutation(shard_len)[:n].astype(np.uint64)
    shard0 = rng.integers(-100, 100, shard_len).astype(t)
    shard0[idx.astype(np.int64)] = ea
    ops = CF_OPS + [CAS_EPS]
    with np.errstate(all="ignore"):
        for op in ops:
            for kind in ([KIND_GENERIC, KIND_LOCAL_LOCK] if op == CAS_EPS else [KIND_GENERIC]):
                cur = eps = None
                if op == CAS_EPS:
                    cur, eps = t(0.0), np.finfo(t).tiny       # +-0.0 and subnormals are within eps of 0.0
                c = Case(k, orc, lam, dt, op, shard0, idx, vb, "soa", strategy, kind=kind, cur=cur, eps=eps)
                assert c.err == 0 and c.st_o == 0, (dt, op, c.err, c.st_o)
                assert nan_aware_equal(c.got, c.ref), (dt, path, op, "state", first_mismatch(c.got, c.ref))
                if c.rk:
                    assert nan_aware_equal(c.res_d, c.res_o), (dt, path, op, "results",
                                                               first_mismatch(c.res_d, c.res_o))
                if c.rk == 2:
                    assert np.array_equal(c.ok_d, c.ok_o), (dt, path, op, "ok")


@pytest.mark.parametrize("dt", ["f32", "f64"])
def test_specials_mvsi_in_order(world, orc, lam, dt):
    """Many values at one index, applied in buffer order: the same bits as the reference's
    sequential loop for every op, with special values among the values and the element."""
    k = world.team().kernels
    t = NP[dt]
    S = specials(t)
    rng = np.random.default_rng(55)
    with np.errstate(all="ignore"):
        for start in S:
            for op in CF_OPS:
                vals = rng.choice(S, 40)
                if op in (MUL, FETCH_MUL, DIV, FETCH_DIV, REM, FETCH_REM):
                    vals = rng.choice(np.concatenate([S, np.array([2.0, 0.5, -3.0], dtype=t)]), 40)
                shard0 = np.zeros(64, dtype=t)
                shard0[17] = start
                c = Case(k, orc, lam, dt, op, shard0, np.array([17], dtype=np.uint64), vals, "mvsi", 1)
                assert c.err == 0 and c.st_o == 0
                assert nan_aware_equal(c.got, c.ref), (dt, op, start, first_mismatch(c.got, c.ref))
                if c.rk:
                    assert nan_aware_equal(c.res_d, c.res_o), (dt, op, start, first_mismatch(c.res_d, c.res_o))


def colliding_inputs(t, rng, shard_len, n, op, hot=False):
    """Element classes whose outcome does not depend on the order of their records."""
    fi = np.finfo(t)
    sub = fi.smallest_subnormal
    n_el = min(shard_len // 2, 6000)
    el = rng.choice(shard_len, n_el, replace=False)
    cls = rng.integers(0, 6, n_el)
    shard0 = rng.integers(-50, 50, shard_len).astype(t)
    idx = el[rng.integers(0, n_el, n)]
    pos = {int(e): i for i, e in enumerate(el)}
    c_rec = cls[np.fromiter((pos[int(e)] for e in idx), dtype=np.int64, count=n)]
    vals = np.empty(n, dtype=t)
    sign = -1.0 if op in (SUB, FETCH_SUB) else 1.0       # a - v: the classes hold for a + (-v)
    # class 0: subnormal multiples (exact in any order); element 3*sub, records 1..7 * sub
    m = c_rec == 0
    vals[m] = (rng.integers(1, 8, int(m.sum())) * sub * sign).astype(t)
    shard0[el[cls == 0]] = t(3 * sub)
    # class 1: -0.0 element, -0.0 records (sub: +0.0 records; -0.0 - +0.0 = -0.0)
    m = c_rec == 1
    vals[m] = t(-0.0) if sign > 0 else t(0.0)
    shard0[el[cls == 1]] = t(-0.0)
    # class 2: +inf absorbs finite records (one +inf record per element at least)
    m = c_rec == 2
    vals[m] = rng.integers(-100, 100, int(m.sum())).astype(t)
    # class 3: +inf and -inf records meet -> NaN
    m = c_rec == 3
    vals[m] = rng.integers(-100, 100, int(m.sum())).astype(t)
    # class 4: NaN element absorbs everything
    m = c_rec == 4
    vals[m] = rng.integers(-100, 100, int(m.sum())).astype(t)
    shard0[el[cls == 4]] = t(np.nan)
    # class 5: max finite element, positive records (half of max): overflow to +inf in any order
    m = c_rec == 5
    vals[m] = t(fi.max / 2 * sign)
    shard0[el[cls == 5]] = fi.max
    # plant the infinities: for every class-2 / class-3 element, one record of its first
    # occurrence becomes +inf (class 3: also the second one -inf)
    first = {}
    for j in range(n):
        e = int(idx[j])
        if c_rec[j] in (2, 3):
            first.setdefault(e, []).append(j)
    for e, js in first.items():
        vals[js[0]] = t(np.inf * sign)
        if c_rec[js[0]] == 3:
            if len(js) > 1:
                vals[js[1]] = t(-np.inf * sign)
            else:
                shard0[e] = t(-np.inf)                   # lone record: the element is -inf
    if hot:                                              # delta mode: 40 % on one class-0 element
        h = int(el[cls == 0][0])
        hm = rng.random(n) < 0.4
        idx[hm] = h
        vals[hm] = t(sub * sign)
        c_rec[hm] = 0
    return shard0, idx.astype(np.uint64), vals, el, cls


CPATHS = PATHS + ["delta", "delta_staged"]


@pytest.mark.parametrize("path", CPATHS)
@pytest.mark.parametrize("dt", ["f32", "f64"])
def test_specials_colliding(world, orc, lam, dt, path, monkeypatch):
    """delta / delta_staged: 64 tiles, 2^19 records, 40 % of them on one element: its tile
    holds far more than 4x the average tile's records, so the combinable ops split it into
    delta pieces (one-shot tiled path / staged pipeline)."""
    k = world.team().kernels
    k.reserve(1 << 21)
    hot = path.startswith("delta")
    strategy = _setup_path({"delta": "tiled1", "delta_staged": "staged"}.get(path, path), monkeypatch)
    t = NP[dt]
    eb = t(0).itemsize
    rng = np.random.default_rng(2000 + CODE[dt] + 11 * CPATHS.index(path))
    shard_len = 64 * TILE[eb] + 11 if hot else _shard_len(path, eb)
    n = 1 << 19 if hot else 1 << 18
    with np.errstate(all="ignore"):
        for op in (ADD, FETCH_ADD, SUB, FETCH_SUB, SWAP):
            shard0, idx, vals, el, cls = colliding_inputs(t, rng, shard_len, n, op, hot=hot)
            if op == SWAP:
                vals = rng.choice(specials(t), n)
            c = Case(k, orc, lam, dt, op, shard0, idx, vals, "soa", strategy)
            assert c.err == 0 and c.st_o == 0
            if op != SWAP:
                assert nan_aware_equal(c.got, c.ref), (dt, path, op, first_mismatch(c.got, c.ref))
            if op in (FETCH_ADD, FETCH_SUB, SWAP):
                # per element one serial order; elements that turn NaN through arithmetic are
                # left out (a NaN's sign / payload differs between x86 and gfx950)
                keep = np.ones(idx.size, dtype=bool)
                init, fin = shard0.copy(), c.got.copy()
                if op != SWAP:
                    drop = el[(cls == 3) | (cls == 4)]
                    keep = ~np.isin(idx, drop)
                    init[drop] = 0
                    fin[drop] = 0
                st, bad = orc.check_linearizable(KIND_GENERIC, CODE[dt], t, op, init, fin, idx[keep], vals[keep],
                                                 c.res_d[keep])
                assert st == 0, (dt, path, op, "element", bad)
