"""The one-level ("wide") staged partition for 1/2/4-byte element shards (lmr_wide.hip, round 6):
shards of at most 2048 tiles of 128 KiB of 32-bit LDS words (2^26 elements: C5's u32 shard) are
partitioned in one pass straight into their tiles (16K-record LDS rounds) and their olds come back
in one gather, where larger shards (and LMR_WIDE4=0) take the two-level path. Every case checks that
the wide path ran (no fine pass in the stage profile) and its results against the oracle / numpy:
  * final shard = the serial replay, bit for bit (f32 sums of small integers are exact);
  * returned olds / Results are a valid linearisation (oracle/linearize.c);
  * one tile, a ragged shard, the 2048-tile maximum, u32 and u64 indices, scalar values, u8 / i16
    sub-word elements (widened LDS words), hot tiles in delta pieces, out-of-bounds indices;
  * a mixed C5-shaped session (and / or / xor / swap / compare_exchange) whose first count-free
    phase joins the counted phases (one partition, one sweep), op phases in staging order;
  * the same records through the two-level path (LMR_WIDE4=0) give the same final shard.
Reference semantics: olds returned in input order, `src/array/operations/handle.rs:293-325`; the
NativeAtomic u32 and/or/xor and swap / compare_exchange bodies, `native_atomic.rs:75-89`,
`impl/src/array_ops.rs:379-390`."""
import numpy as np
import pytest
import torch

from opgen import ADD, AND, CAS, CODE, FETCH_ADD, FETCH_XOR, NP, OR, SWAP, XOR
from test_gpu_parity import to_dev

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _wide4(monkeypatch):
    """The wide path for 1/2/4-byte elements is switched per session (LMR_WIDE4, read by the
    library at each session's first partition)."""
    monkeypatch.setenv("LMR_WIDE4", "1")


def _skewed(rng, n_el, n, hot_share=0.1):
    u = rng.integers(0, n_el, n)
    hot = int(rng.integers(0, n_el))
    warm = rng.choice(n_el, min(256, n_el), replace=False)
    r = rng.random(n)
    out = np.where(r < hot_share, hot, np.where(r < 2 * hot_share, warm[rng.integers(0, warm.size, n)], u))
    return out.astype(np.uint64)


def _run(k, shard, n_el, dt, phases, stage_profile=True):
    """phases: (op, idx, iw, vals or None, scalar, results, ok, cmp) staged into one session."""
    if stage_profile:
        k.profile(True)
        k.profile_read(reset=True)
    try:
        for j, (op, idx, iw, vals, scalar, res, ok, cmp) in enumerate(phases):
            if j == 0:
                k.stage_begin(shard, n_el, 1, dt, op, cmp)
            else:
                k.stage_op(op, cmp)
            i = idx if iw == 8 else idx.astype(np.uint32)
            k.stage_soa(to_dev(i), iw, None if vals is None else to_dev(vals), scalar, idx.size, res, ok)
        k.stage_finish()
        return k.profile_read(reset=True) if stage_profile else None
    finally:
        if stage_profile:
            k.profile(False)


def _assert_wide(stages, sweeps=None):
    assert stages.get("bin_scatter", (0, 0))[1] >= 1, stages
    assert stages.get("fine_scatter", (0, 0))[1] == 0, stages      # one level: no fine pass
    if sweeps is not None:
        assert stages["tile_apply"][1] == sweeps, stages


@pytest.mark.parametrize("n_el", [(1 << 15) - 5, (1 << 22) + 77, 1 << 26], ids=["one-tile", "ragged", "max"])
def test_wide4_u32_fetch_add_linearizable(world, lam, orc, n_el):
    k = world.team().kernels
    dt = lam.dtype_of("u32")
    rng = np.random.default_rng(n_el)
    n = 1 << 21
    idx = _skewed(rng, n_el, n)
    vals = rng.integers(1, 1 << 20, n, dtype=np.uint64).astype(np.uint32)
    s0 = rng.integers(0, 1 << 31, n_el, dtype=np.uint64).astype(np.uint32)
    shard = to_dev(s0)
    res = k.empty(n, torch.int32)
    k.reserve(n)
    stages = _run(k, shard, n_el, dt, [(FETCH_ADD, idx, 8, vals, 0, res, None, 0)])
    assert k.errors() == 0
    _assert_wide(stages, 1)
    final = shard.cpu().numpy().view(np.uint32)
    exp = s0.copy()
    np.add.at(exp, idx.astype(np.int64), vals)
    assert np.array_equal(final, exp)
    st, bad = orc.check_linearizable(1, CODE["u32"], np.uint32, FETCH_ADD, s0, final, idx, vals,
                                     res.cpu().numpy().view(np.uint32))
    assert st == 0, bad


@pytest.mark.parametrize("dtn,op", [("u8", FETCH_ADD), ("i16", SWAP), ("f32", FETCH_ADD), ("i32", FETCH_XOR)])
def test_wide4_element_types(world, lam, orc, dtn, op):
    """Sub-word elements (8/16-bit, widened to 32-bit LDS words in the 128 KiB tiles), f32 (exact
    small-integer sums) and i32 fetch_xor with a hot tile (delta pieces), u32 local indices and a
    scalar-valued region in the same session."""
    k = world.team().kernels
    dt = lam.dtype_of(dtn)
    t = NP[dtn]
    rng = np.random.default_rng(CODE[dtn] * 31 + op)
    n_el, n = (1 << 21) + 11, 1 << 20
    if dtn == "f32":
        s0 = rng.integers(0, 64, n_el).astype(np.float32)
        mk = lambda m: rng.integers(1, 8, m).astype(np.float32)
    else:
        info = np.iinfo(t)
        s0 = rng.integers(info.min, info.max, n_el, dtype=t, endpoint=True)
        mk = lambda m: rng.integers(info.min, info.max, m, dtype=t, endpoint=True)
    i1, i2 = _skewed(rng, n_el, n, 0.05), _skewed(rng, n_el, n // 2, 0.05)
    v1 = mk(n)
    sc = mk(1)[0]
    v2 = np.full(n // 2, sc, t)
    r1, r2 = k.empty(n, dt.torch), k.empty(n // 2, dt.torch)
    shard = to_dev(s0)
    k.reserve(2 * n)
    bits = int(np.array([sc], t).view({1: np.uint8, 2: np.uint16, 4: np.uint32}[t().itemsize])[0])
    stages = _run(k, shard, n_el, dt, [(op, i1, 8, v1, 0, r1, None, 0), (op, i2, 4, None, bits, r2, None, 0)])
    assert k.errors() == 0
    _assert_wide(stages, 1)
    final = shard.cpu().numpy().view(t)
    iall, vall = np.concatenate([i1, i2]), np.concatenate([v1, v2])
    rall = np.concatenate([r1.cpu().numpy().view(t), r2.cpu().numpy().view(t)])
    st, bad = orc.check_linearizable(1, CODE[dtn], t, op, s0, final, iall, vall, rall)
    assert st == 0, bad
    if op in (FETCH_ADD, FETCH_XOR):
        exp = s0.copy()
        (np.add if op == FETCH_ADD else np.bitwise_xor).at(exp, iall.astype(np.int64), vall)
        assert np.array_equal(final, exp)


def test_wide4_oob_indices_reported(world, lam):
    k = world.team().kernels
    dt = lam.dtype_of("u32")
    rng = np.random.default_rng(91)
    n_el, n = (1 << 18) + 3, 1 << 20
    idx = rng.integers(0, n_el, n).astype(np.uint64)
    bad = rng.choice(n, 1000, replace=False)
    idx[bad] = n_el + rng.integers(0, 1 << 30, bad.size).astype(np.uint64)
    shard = to_dev(np.zeros(n_el, np.uint32))
    res = k.empty(n, torch.int32)
    res.fill_(-1)
    k.reserve(n)
    stages = _run(k, shard, n_el, dt, [(FETCH_ADD, idx, 8, None, 1, res, None, 0)])
    from lamellar_runtime_amd.types import ERRBIT_OOB
    assert k.errors() & ERRBIT_OOB
    _assert_wide(stages, 1)
    good = np.ones(n, bool)
    good[bad] = False
    exp = np.bincount(idx[good].astype(np.int64), minlength=n_el).astype(np.uint32)
    assert np.array_equal(shard.cpu().numpy().view(np.uint32), exp)
    r = res.cpu().numpy()
    assert np.all(r[bad] == -1)                        # out-of-bounds records return nothing
    order = np.lexsort((r[good], idx[good]))
    ii, rr = idx[good][order], r[good][order]
    first = np.r_[True, ii[1:] != ii[:-1]]
    start = np.maximum.accumulate(np.where(first, np.arange(ii.size), 0))
    assert np.array_equal(rr, np.arange(ii.size) - start)


def test_wide4_c5_session_one_sweep(world, lam, orc):
    """The C5 shape at reduced size: u32 bit_and / bit_or / bit_xor / swap / compare_exchange(0)
    staged into one session. The first (count-free) phase is not partitioned yet at the switch, so
    it joins the counted phases: one partition pass per group and one sweep. Each phase is checked
    from the state the earlier ones left (phase order per element): and / or / xor bit for bit, swap
    and compare_exchange as linearisations."""
    k = world.team().kernels
    dt = lam.dtype_of("u32")
    rng = np.random.default_rng(0xC5)
    n_el, m = (1 << 22) + 5, 1 << 19
    s0 = rng.integers(0, 1 << 32, n_el, dtype=np.uint64).astype(np.uint32)
    hot = rng.choice(n_el, 20000, replace=False)

    def idx():
        return np.where(rng.random(m) < 0.5, rng.integers(0, n_el, m), hot[rng.integers(0, hot.size, m)]).astype(np.uint64)

    r32 = lambda: rng.integers(0, 1 << 32, m, dtype=np.uint64).astype(np.uint32)
    iA, vA = idx(), r32() | np.uint32(0x0F0F0F0F)
    iO, vO = idx(), r32() & np.uint32(0x00FF00FF)
    iX, vX = idx(), r32()
    iS, vS = idx(), rng.integers(0, 4, m, dtype=np.uint64).astype(np.uint32)
    iC, vC = idx(), rng.integers(0, 4, m, dtype=np.uint64).astype(np.uint32)
    rS, rC, okC = k.empty(m, torch.int32), k.empty(m, torch.int32), k.empty(m, torch.uint8)
    shard = to_dev(s0)
    k.reserve(8 * m)
    stages = _run(k, shard, n_el, dt, [(AND, iA, 8, vA, 0, None, None, 0), (OR, iO, 8, vO, 0, None, None, 0),
                                      (XOR, iX, 8, vX, 0, None, None, 0), (SWAP, iS, 8, vS, 0, rS, None, 0),
                                      (CAS, iC, 8, vC, 0, rC, okC, 0)])
    assert k.errors() == 0
    _assert_wide(stages, 1)
    assert stages["bin_count"][1] == 1, stages          # the five regions partitioned as one group
    final = shard.cpu().numpy().view(np.uint32)
    ii = lambda a: a.astype(np.int64)
    s3 = s0.copy()
    np.bitwise_and.at(s3, ii(iA), vA)
    np.bitwise_or.at(s3, ii(iO), vO)
    np.bitwise_xor.at(s3, ii(iX), vX)
    u = lambda t: t.cpu().numpy().view(np.uint32)
    s4 = s3.astype(np.uint64)                           # swap: start + sum(vals) - sum(returned)
    np.add.at(s4, ii(iS), vS.astype(np.uint64))
    np.subtract.at(s4, ii(iS), u(rS).astype(np.uint64))
    s4 = s4.astype(np.uint32)
    st, bad = orc.check_linearizable(1, CODE["u32"], np.uint32, SWAP, s3, s4, iS, vS, u(rS))
    assert st == 0, ("swap", st, bad)
    st, bad = orc.check_linearizable(1, CODE["u32"], np.uint32, CAS, s4, final, iC, vC, u(rC), okC.cpu().numpy(),
                                     current=np.uint32(0))
    assert st == 0, ("compare_exchange", st, bad)
    assert okC.cpu().numpy().any() and (~okC.cpu().numpy().astype(bool)).any()


@pytest.mark.parametrize("op", [AND, ADD], ids=["and", "add"])
def test_wide4_matches_two_level(world, lam, monkeypatch, op):
    """The same two-phase session (op, then xor) through the wide path and the two-level path
    (LMR_WIDE4=0): identical final shards."""
    k = world.team().kernels
    dt = lam.dtype_of("u32")
    rng = np.random.default_rng(op + 100)
    n_el, m = (1 << 23) + 3, 1 << 20
    s0 = rng.integers(0, 1 << 32, n_el, dtype=np.uint64).astype(np.uint32)
    i1, i2 = _skewed(rng, n_el, m, 0.02), rng.integers(0, n_el, m).astype(np.uint64)
    v1, v2 = (rng.integers(0, 1 << 32, m, dtype=np.uint64).astype(np.uint32) for _ in range(2))
    k.reserve(2 * m)
    out = []
    for wide in ("1", "0"):
        monkeypatch.setenv("LMR_WIDE4", wide)
        shard = to_dev(s0)
        stages = _run(k, shard, n_el, dt, [(op, i1, 8, v1, 0, None, None, 0), (XOR, i2, 4, v2, 0, None, None, 0)])
        assert k.errors() == 0
        assert (stages.get("fine_scatter", (0, 0))[1] == 0) == (wide == "1"), stages
        out.append(shard.cpu().numpy().view(np.uint32).copy())
    assert np.array_equal(out[0], out[1])
    exp = s0.copy()
    (np.bitwise_and if op == AND else np.add).at(exp, i1.astype(np.int64), v1)
    np.bitwise_xor.at(exp, i2.astype(np.int64), v2)
    assert np.array_equal(out[0], exp)
