"""The one-level ("wide") staged partition (lmr_wide.hip): 8-byte element shards of at most
1024 tiles of 128 KiB (2^24 elements) are partitioned in one pass straight into their tiles and
their olds come back in one gather, where other shards take the two-level path (count, coarse,
fine, two gathers). Every case checks that the wide path ran (no fine pass in the stage profile)
and its results against the oracle:
  * final shard = the serial replay (bit for bit for integers; f64 sums of 1.0 are exact);
  * returned olds / Results are a valid linearisation (oracle/linearize.c);
  * ragged shards (a partial last tile), one tile, the 1024-tile maximum, u32 and u64 indices,
    scalar values, several regions in one session (deferred batches), out-of-bounds indices
    (reported, the in-bounds records applied), a RESULT op (compare_exchange) with ok flags.
Reference semantics: olds returned in input order, `src/array/operations/handle.rs:293-325`;
concurrent batches' olds one valid serial order per element (`impl/src/array_ops.rs:863-1408`)."""
import numpy as np
import pytest
import torch

from opgen import ADD, CAS, CODE, FETCH_ADD, FETCH_XOR, SWAP
from test_gpu_parity import to_dev

pytestmark = pytest.mark.gpu


def _skewed(rng, n_el, n, hot_share=0.1):
    """Uniform records plus a hot element and 256 warm ones (the delta pieces and the owner's
    warm elements both run)."""
    u = rng.integers(0, n_el, n)
    hot = int(rng.integers(0, n_el))
    warm = rng.choice(n_el, min(256, n_el), replace=False)
    r = rng.random(n)
    out = np.where(r < hot_share, hot, np.where(r < 2 * hot_share, warm[rng.integers(0, warm.size, n)], u))
    return out.astype(np.uint64)


def _stages(k):
    return k.profile_read(reset=True)


def _assert_wide(stages):
    assert stages.get("bin_scatter", (0, 0))[1] >= 1, stages
    assert stages.get("fine_scatter", (0, 0))[1] == 0, stages      # one level: no fine pass


@pytest.mark.parametrize("n_el", [(1 << 14) - 5, (1 << 20) + 77, 1 << 24], ids=["one-tile", "ragged", "max"])
def test_wide_u64_fetch_add_linearizable(world, lam, orc, n_el):
    k = world.team().kernels
    dt = lam.dtype_of("u64")
    rng = np.random.default_rng(n_el)
    n = 1 << 21
    idx = _skewed(rng, n_el, n)
    vals = rng.integers(1, 1 << 20, n, dtype=np.uint64)
    s0 = rng.integers(0, 1 << 40, n_el, dtype=np.uint64)
    shard = to_dev(s0)
    res = k.empty(n, torch.int64)
    k.reserve(n)
    k.profile(True)
    k.profile_read(reset=True)
    try:
        k.stage_begin(shard, n_el, 1, dt, FETCH_ADD)
        k.stage_soa(to_dev(idx), 8, to_dev(vals), 0, n, res)
        k.stage_finish()
        stages = _stages(k)
    finally:
        k.profile(False)
    assert k.errors() == 0
    _assert_wide(stages)
    final = shard.cpu().numpy().view(np.uint64)
    exp = s0.copy()
    np.add.at(exp, idx.astype(np.int64), vals)
    assert np.array_equal(final, exp)
    olds = res.cpu().numpy().view(np.uint64)
    st, bad = orc.check_linearizable(1, CODE["u64"], np.uint64, FETCH_ADD, s0, final, idx, vals, olds)
    assert st == 0, bad


def test_wide_session_of_regions_mixed_widths_scalars(world, lam, orc):
    """Five fetch_add regions in one session: u64 and u32 indices, array and scalar values, one
    region without a results buffer (the session still returns the others' olds)."""
    k = world.team().kernels
    dt = lam.dtype_of("i64")
    rng = np.random.default_rng(5)
    n_el = (1 << 22) + 1234
    s0 = rng.integers(-(1 << 40), 1 << 40, n_el, dtype=np.int64)
    sizes = [1 << 20, 300000, (1 << 19) + 17, 1 << 20, 70000]
    idxs = [_skewed(rng, n_el, m, 0.05) for m in sizes]
    vals = [rng.integers(1, 1000, m, dtype=np.int64) for m in sizes]
    scalar = [False, True, False, False, True]
    want = [True, True, False, True, True]
    widths = [8, 4, 8, 4, 8]
    shard = to_dev(s0)
    k.reserve(sum(sizes))
    ress = [k.empty(m, torch.int64) if w else None for m, w in zip(sizes, want)]
    k.profile(True)
    k.profile_read(reset=True)
    try:
        k.stage_begin(shard, n_el, 1, dt, FETCH_ADD)
        for j, m in enumerate(sizes):
            i = idxs[j] if widths[j] == 8 else idxs[j].astype(np.uint32)
            if scalar[j]:
                vals[j][:] = 7
                k.stage_soa(to_dev(i), widths[j], None, 7, m, ress[j])
            else:
                k.stage_soa(to_dev(i), widths[j], to_dev(vals[j]), 0, m, ress[j])
        k.stage_finish()
        stages = _stages(k)
    finally:
        k.profile(False)
    assert k.errors() == 0
    _assert_wide(stages)
    assert stages["tile_apply"][1] == 1, stages
    final = shard.cpu().numpy().view(np.int64)
    exp = s0.copy()
    for i, v in zip(idxs, vals):
        np.add.at(exp, i.astype(np.int64), v)
    assert np.array_equal(final, exp)
    # the silent region's records interleave with the others' anywhere, so the returning
    # regions' olds are checked for what every serial order gives: on each element they are
    # distinct (the values are positive) and lie in [start, final)
    sel = [j for j in range(len(sizes)) if want[j]]
    iall = np.concatenate([idxs[j] for j in sel]).astype(np.int64)
    rall = np.concatenate([ress[j].cpu().numpy().view(np.int64) for j in sel])
    order = np.lexsort((rall, iall))
    i_s, r_s = iall[order], rall[order]
    assert not np.any((i_s[1:] == i_s[:-1]) & (r_s[1:] == r_s[:-1])), "two records saw one state"
    assert np.all((rall >= s0[iall]) & (rall < final[iall]))
    # every region returning: the session's olds are jointly a valid linearisation
    k.reserve(sum(sizes))
    shard.copy_(to_dev(s0))
    ress = [k.empty(m, torch.int64) for m in sizes]
    k.stage_begin(shard, n_el, 1, dt, FETCH_ADD)
    for j, m in enumerate(sizes):
        i = idxs[j] if widths[j] == 8 else idxs[j].astype(np.uint32)
        k.stage_soa(to_dev(i), widths[j], None if scalar[j] else to_dev(vals[j]), 7 if scalar[j] else 0, m, ress[j])
    k.stage_finish()
    assert k.errors() == 0
    assert np.array_equal(shard.cpu().numpy().view(np.int64), final)
    iall = np.concatenate(idxs)
    vall = np.concatenate(vals)
    rall = np.concatenate([r.cpu().numpy().view(np.int64) for r in ress])
    st, bad = orc.check_linearizable(1, CODE["i64"], np.int64, FETCH_ADD, s0, final, iall, vall, rall)
    assert st == 0, bad


def test_wide_deferred_f64_batches_one_sweep(world, lam, orc):
    """Three deferred f64 fetch_add batches (the C3 pattern) applied in one sweep."""
    team = world.team()
    k = team.kernels
    n_el = 1 << 20
    arr = lam.AtomicArray(team, n_el, lam.Distribution.Block, "f64")
    rng = np.random.default_rng(0xC3)
    init = rng.integers(0, 1000, n_el).astype(np.float64)
    arr.local_data().copy_(torch.from_numpy(init).to(k.device))
    nb = 1 << 20
    idxs = [_skewed(rng, n_el, nb) for _ in range(3)]
    ones = np.ones(nb, np.float64)
    k.reserve(3 * nb)
    k.profile(True)
    k.profile_read(reset=True)
    try:
        hs = [arr.batch_fetch_add(i, ones).spawn() for i in idxs]
        rs = [h.block() for h in hs]
        stages = _stages(k)
    finally:
        k.profile(False)
    _assert_wide(stages)
    assert stages["tile_apply"][1] == 1, stages
    final = arr.local_numpy().copy()
    iall = np.concatenate(idxs)
    exp = init + np.bincount(iall.astype(np.int64), minlength=n_el)
    assert np.array_equal(final, exp)
    rall = np.concatenate([r.cpu().numpy().view(np.float64) for r in rs])
    st, bad = orc.check_linearizable(1, CODE["f64"], np.float64, FETCH_ADD, init, final, iall,
                                     np.ones(iall.size), rall)
    assert st == 0, bad


def test_wide_oob_indices_reported(world, lam):
    k = world.team().kernels
    dt = lam.dtype_of("u64")
    rng = np.random.default_rng(9)
    n_el, n = (1 << 18) + 3, 1 << 20
    idx = rng.integers(0, n_el, n).astype(np.uint64)
    bad = rng.choice(n, 1000, replace=False)
    idx[bad] = n_el + rng.integers(0, 1 << 30, bad.size).astype(np.uint64)
    shard = to_dev(np.zeros(n_el, np.uint64))
    res = k.empty(n, torch.int64)
    res.fill_(-1)
    k.reserve(n)
    k.stage_begin(shard, n_el, 1, dt, FETCH_ADD)
    k.stage_soa(to_dev(idx), 8, None, 1, n, res)
    k.stage_finish()
    from lamellar_runtime_amd.types import ERRBIT_OOB
    assert k.errors() & ERRBIT_OOB
    good = np.ones(n, bool)
    good[bad] = False
    exp = np.bincount(idx[good].astype(np.int64), minlength=n_el).astype(np.uint64)
    assert np.array_equal(shard.cpu().numpy().view(np.uint64), exp)
    r = res.cpu().numpy()
    assert np.all(r[bad] == -1)                        # out-of-bounds records return nothing
    # in-bounds olds: per element exactly 0..count-1
    order = np.lexsort((r[good], idx[good]))
    ii, rr = idx[good][order], r[good][order]
    first = np.r_[True, ii[1:] != ii[:-1]]
    start = np.maximum.accumulate(np.where(first, np.arange(ii.size), 0))
    assert np.array_equal(rr, np.arange(ii.size) - start)


@pytest.mark.parametrize("op", [CAS, SWAP, FETCH_XOR], ids=["cas", "swap", "fetch_xor"])
def test_wide_non_add_ops(world, lam, orc, op):
    """compare_exchange (Results with ok flags), swap (no delta pieces: owner tiles only) and
    fetch_xor (delta pieces) through the wide path, checked as linearisations."""
    k = world.team().kernels
    dt = lam.dtype_of("u64")
    rng = np.random.default_rng(op)
    n_el, n = (1 << 21) + 9, 1 << 20
    idx = _skewed(rng, n_el, n, 0.03)
    s0 = rng.integers(0, 4, n_el, dtype=np.uint64)
    vals = rng.integers(0, 4, n, dtype=np.uint64) if op != FETCH_XOR else rng.integers(0, 1 << 63, n, dtype=np.uint64)
    cur = 2
    shard = to_dev(s0)
    res = k.empty(n, torch.int64)
    ok = k.empty(n, torch.uint8) if op == CAS else None
    k.reserve(n)
    k.profile(True)
    k.profile_read(reset=True)
    try:
        k.stage_begin(shard, n_el, 1, dt, op, cur if op == CAS else 0)
        k.stage_soa(to_dev(idx), 8, to_dev(vals), 0, n, res, ok)
        k.stage_finish()
        stages = _stages(k)
    finally:
        k.profile(False)
    assert k.errors() == 0
    _assert_wide(stages)
    final = shard.cpu().numpy().view(np.uint64)
    rets = res.cpu().numpy().view(np.uint64)
    kw = {}
    if op == CAS:
        kw = dict(current=cur)
        st, bad = orc.check_linearizable(1, CODE["u64"], np.uint64, op, s0, final, idx, vals, rets,
                                         ok.cpu().numpy(), **kw)
    else:
        st, bad = orc.check_linearizable(1, CODE["u64"], np.uint64, op, s0, final, idx, vals, rets)
    assert st == 0, bad


def test_wide_mixed_session_returning_phases(world, lam, orc):
    """A mixed session on a wide shard (u64, 2^20 - 3 elements: <= 128 two-level tiles, so even
    the first, order-insensitive phase is a counted region): and, swap, xor, compare_exchange,
    fetch_add and add phases staged into one session, partitioned one-level and applied in one
    sweep, op phase by op phase in staging order per element (as test_gpu_stage_mixed does on a
    two-level shard). Each returning phase's olds / Results are a valid linearisation from the
    state the earlier phases left."""
    from opgen import AND, XOR
    k = world.team().kernels
    dt = lam.dtype_of("u64")
    n_el, n = (1 << 20) - 3, 1 << 18
    rng = np.random.default_rng(2024)
    hot = rng.choice(n_el, 30000, replace=False)

    def idx():
        u = rng.integers(0, n_el, n)
        h = hot[rng.integers(0, hot.size, n)]
        return np.where(rng.random(n) < 0.5, u, h).astype(np.uint64)

    r64 = lambda hi: rng.integers(0, hi, n, dtype=np.uint64)
    s0 = rng.integers(0, 8, n_el, dtype=np.uint64)
    iA, vA = idx(), r64(2**63) | np.uint64(0xFFFFFFFFFFFFFFF0)
    iS, vS = idx(), r64(8)
    iX, vX = idx(), r64(8)
    iC, vC = idx(), r64(8)
    iF, vF = idx(), r64(1000)
    iD, vD = idx(), r64(2**63)
    cur = 3
    k.reserve(8 * n)
    shard = to_dev(s0)
    rS, rC, okC, rF = (k.empty(n, torch.int64), k.empty(n, torch.int64), k.empty(n, torch.uint8),
                       k.empty(n, torch.int64))
    k.profile(True)
    k.profile_read(reset=True)
    try:
        k.stage_begin(shard, n_el, 1, dt, AND)
        k.stage_soa(to_dev(iA), 8, to_dev(vA), 0, n)
        k.stage_op(SWAP)
        k.stage_soa(to_dev(iS), 8, to_dev(vS), 0, n, rS)
        k.stage_op(XOR)
        k.stage_soa(to_dev(iX), 8, to_dev(vX), 0, n)
        k.stage_op(CAS, cur)
        k.stage_soa(to_dev(iC), 8, to_dev(vC), 0, n, rC, okC)
        k.stage_op(FETCH_ADD)
        k.stage_soa(to_dev(iF), 8, to_dev(vF), 0, n, rF)
        k.stage_op(ADD)
        k.stage_soa(to_dev(iD), 8, to_dev(vD), 0, n)
        k.stage_finish()
        stages = _stages(k)
    finally:
        k.profile(False)
    assert k.errors() == 0
    _assert_wide(stages)
    final = shard.cpu().numpy().view(np.uint64)
    u = lambda t: t.cpu().numpy().view(np.uint64)
    ii = lambda a: a.astype(np.int64)
    s1 = s0.copy()
    np.bitwise_and.at(s1, ii(iA), vA)
    s2 = s1.copy()                                    # swap: init + sum(vals) - sum(returned)
    np.add.at(s2, ii(iS), vS)
    np.subtract.at(s2, ii(iS), u(rS))
    st, bad = orc.check_linearizable(1, CODE["u64"], np.uint64, SWAP, s1, s2, iS, vS, u(rS))
    assert st == 0, ("swap", st, bad)
    s3 = s2.copy()
    np.bitwise_xor.at(s3, ii(iX), vX)
    s5 = final.copy()
    np.subtract.at(s5, ii(iD), vD)                    # undo the last add phase
    s4 = s5.copy()
    np.subtract.at(s4, ii(iF), vF)                    # the fetch_add phase's start state
    st, bad = orc.check_linearizable(1, CODE["u64"], np.uint64, FETCH_ADD, s4, s5, iF, vF, u(rF))
    assert st == 0, ("fetch_add", st, bad)
    st, bad = orc.check_linearizable(1, CODE["u64"], np.uint64, CAS, s3, s4, iC, vC, u(rC), okC.cpu().numpy(),
                                     current=np.uint64(cur))
    assert st == 0, ("compare_exchange", st, bad)
    assert okC.cpu().numpy().any() and (~okC.cpu().numpy().astype(bool)).any()
