"""Mixed staged sessions (lmr_stage_op) and the deferred batches of the op-builder API.

Batches of different ops on one shard staged into one session are applied in one sweep,
op phase by op phase in staging order per element. Checked against the oracle:
  * order-insensitive phases (and / or / xor / add / sub, count-free first phase, counted
    later ones): the final shard equals the serial per-phase replay, bit for bit;
  * returning phases between them (swap, compare_exchange, fetch_add): each phase's
    returned olds / Results are a valid linearisation (oracle/linearize.c) from the state
    the earlier phases left, and the phase's final state is the one the later phases
    started from (derived: swap's leftover value, or the later invertible phases undone).
  * the array API: spawned batches are deferred and applied at the next flush point
    (block, wait_all, to_numpy, local_data), results valid after block().
Reference: consecutive batches on one array reach the owner as separate op AMs applied
concurrently (impl/src/array_ops.rs:863-1408), so per-phase order is one allowed outcome."""
import numpy as np
import pytest
import torch

from opgen import ADD, AND, CAS, FETCH_ADD, OR, STORE, SUB, SWAP, XOR
from test_gpu_parity import to_dev

pytestmark = pytest.mark.gpu

U32 = 2
L = (1 << 22) + 333                     # 129 wide tiles (LMR_WIDE4=1) / 257 two-level tiles of 16K u32
N = 1 << 18


def _idx(rng, n, hot):
    """Half uniform over the shard, half on `hot` elements (~4 records each)."""
    u = rng.integers(0, L, n)
    h = hot[rng.integers(0, hot.size, n)]
    return np.where(rng.random(n) < 0.5, u, h).astype(np.uint64)


def _fold(op, init, idx, vals):
    out = init.copy()
    i = idx.astype(np.int64)
    if op == AND:
        np.bitwise_and.at(out, i, vals)
    elif op == OR:
        np.bitwise_or.at(out, i, vals)
    elif op == XOR:
        np.bitwise_xor.at(out, i, vals)
    elif op == ADD:
        np.add.at(out, i, vals)
    elif op == SUB:
        np.subtract.at(out, i, vals)
    return out


@pytest.mark.parametrize("wide4", ["1", "0"], ids=["wide", "two-level"])
def test_mixed_session_order_insensitive_phases(world, lam, monkeypatch, wide4):
    monkeypatch.setenv("LMR_WIDE4", wide4)
    k = world.team().kernels
    dt = lam.dtype_of("u32")
    rng = np.random.default_rng(4242)
    hot = rng.choice(L, 40000, replace=False)
    s0 = rng.integers(0, 2**32, L, dtype=np.uint64).astype(np.uint32)
    phases = [(AND, rng.integers(0, 2**32, N, dtype=np.uint64).astype(np.uint32) | np.uint32(0x0F0F0000)),
              (OR, rng.integers(0, 2**32, N, dtype=np.uint64).astype(np.uint32) & np.uint32(0x00FF00FF)),
              (XOR, rng.integers(0, 2**32, N, dtype=np.uint64).astype(np.uint32)),
              (ADD, rng.integers(0, 2**32, N, dtype=np.uint64).astype(np.uint32)),
              (AND, rng.integers(0, 2**32, N, dtype=np.uint64).astype(np.uint32) | np.uint32(0xF0F00F0F)),
              (SUB, rng.integers(0, 2**32, N, dtype=np.uint64).astype(np.uint32))]
    idxs = [_idx(rng, N, hot) for _ in phases]
    k.reserve(4 * N)                       # workspace holds 4 phases: the session also flushes when full
    shard = to_dev(s0)
    k.profile(True)
    k.profile_read(reset=True)
    try:
        for j, ((op, v), i) in enumerate(zip(phases, idxs)):
            if j == 0:
                k.stage_begin(shard, L, 1, dt, op)
            else:
                k.stage_op(op)
            k.stage_soa(to_dev(i), 8, to_dev(v), 0, N)
        k.stage_finish()
        stages = k.profile_read(reset=True)
    finally:
        k.profile(False)
    assert k.errors() == 0
    got = shard.cpu().numpy().view(np.uint32)
    ref = s0.copy()
    for (op, v), i in zip(phases, idxs):
        ref = _fold(op, ref, i, v)
    assert np.array_equal(got, ref)
    # two-level: the count-free first phase is applied at the switch; the counted phases 2..6
    # share one sweep, or two when the workspace (at least 4 phases) fills; wide: the first phase
    # joins the others
    assert stages["tile_apply"][1] in ((1, 2) if wide4 == "1" else (2, 3)), stages


def _swap_final(init, idx, vals, rets):
    """The state a linearisable swap phase leaves: per element init + sum(vals) - sum(rets)
    (the one value no later swap returned)."""
    acc = init.astype(np.uint64).copy()
    np.add.at(acc, idx.astype(np.int64), vals.astype(np.uint64))
    np.subtract.at(acc, idx.astype(np.int64), rets.astype(np.uint64))
    return acc.astype(np.uint32)


@pytest.mark.parametrize("wide4", ["1", "0"], ids=["wide", "two-level"])
def test_mixed_session_returning_phases(world, lam, orc, monkeypatch, wide4):
    monkeypatch.setenv("LMR_WIDE4", wide4)
    k = world.team().kernels
    dt = lam.dtype_of("u32")
    rng = np.random.default_rng(777)
    hot = rng.choice(L, 30000, replace=False)
    s0 = rng.integers(0, 8, L, dtype=np.uint64).astype(np.uint32)
    r32 = lambda hi: rng.integers(0, hi, N, dtype=np.uint64).astype(np.uint32)
    iA, vA = _idx(rng, N, hot), r32(2**32) | np.uint32(0xFFFFFFF0)
    iS, vS = _idx(rng, N, hot), r32(8)
    iX, vX = _idx(rng, N, hot), r32(8)
    iC, vC = _idx(rng, N, hot), r32(8)
    iF, vF = _idx(rng, N, hot), r32(1000)
    iD, vD = _idx(rng, N, hot), r32(2**32)
    cur = np.uint32(3)
    k.reserve(8 * N)
    shard = to_dev(s0)
    rS, rC, okC, rF = (k.empty(N, torch.int32), k.empty(N, torch.int32), k.empty(N, torch.uint8),
                       k.empty(N, torch.int32))
    k.stage_begin(shard, L, 1, dt, AND)
    k.stage_soa(to_dev(iA), 8, to_dev(vA), 0, N)
    k.stage_op(SWAP)
    k.stage_soa(to_dev(iS), 8, to_dev(vS), 0, N, rS)
    k.stage_op(XOR)
    k.stage_soa(to_dev(iX), 8, to_dev(vX), 0, N)
    k.stage_op(CAS, int(cur))
    k.stage_soa(to_dev(iC), 8, to_dev(vC), 0, N, rC, okC)
    k.stage_op(FETCH_ADD)
    k.stage_soa(to_dev(iF), 8, to_dev(vF), 0, N, rF)
    k.stage_op(ADD)
    k.stage_soa(to_dev(iD), 8, to_dev(vD), 0, N)
    k.stage_finish()
    assert k.errors() == 0
    final = shard.cpu().numpy().view(np.uint32)
    u = lambda t: t.cpu().numpy().view(np.uint32)
    s1 = _fold(AND, s0, iA, vA)
    s2 = _swap_final(s1, iS, vS, u(rS))
    st, bad = orc.check_linearizable(1, U32, np.uint32, SWAP, s1, s2, iS, vS, u(rS))
    assert st == 0, ("swap", st, bad)
    s3 = _fold(XOR, s2, iX, vX)
    s5 = _fold(SUB, final, iD, vD)                     # undo the last add phase
    # fetch_add phase: its start state = its end state minus the phase's sum
    s4 = _fold(SUB, s5, iF, vF)
    st, bad = orc.check_linearizable(1, U32, np.uint32, FETCH_ADD, s4, s5, iF, vF, u(rF))
    assert st == 0, ("fetch_add", st, bad)
    st, bad = orc.check_linearizable(1, U32, np.uint32, CAS, s3, s4, iC, vC, u(rC), okC.cpu().numpy(),
                                     current=cur)
    assert st == 0, ("compare_exchange", st, bad)
    assert okC.cpu().numpy().any() and (~okC.cpu().numpy().astype(bool)).any()


@pytest.mark.parametrize("wide4", ["1", "0"], ids=["wide", "two-level"])
def test_deferred_batches_array_api(world, lam, orc, monkeypatch, wide4):
    """Spawned batches are staged and applied at the next flush point, in issue order. On the wide
    path (the default for this u32 shard) the first, count-free batch is not partitioned yet at the
    op switch and joins the later ones: one sweep; on the two-level path it is applied at the
    switch."""
    monkeypatch.setenv("LMR_WIDE4", wide4)
    team = world.team()
    arr = lam.AtomicArray(team, L, lam.Distribution.Block, "u32")
    rng = np.random.default_rng(99)
    hot = rng.choice(L, 30000, replace=False)
    s0 = rng.integers(0, 8, L, dtype=np.uint64).astype(np.uint32)
    arr.local_data().copy_(torch.from_numpy(s0.view(np.int32)).to(team.kernels.device))
    r32 = lambda hi: rng.integers(0, hi, N, dtype=np.uint64).astype(np.uint32)
    iA, vA = _idx(rng, N, hot), r32(2**32)
    iS, vS = _idx(rng, N, hot), r32(8)
    iO, vO = _idx(rng, N, hot), r32(2**32)
    ti = lambda a: torch.from_numpy(a.astype(np.int64)).to(team.kernels.device)
    tv = lambda a: torch.from_numpy(a.view(np.int32)).to(team.kernels.device)
    k = team.kernels
    k.profile(True)
    k.profile_read(reset=True)
    try:
        # wide: the inputs handed over (Owned), so nothing is partitioned before the flush and the
        # count-free first batch joins the others; two-level: plain (borrowed) tensors, each batch
        # partitioned at its spawn
        own = (lambda t: lam.Owned(t)) if wide4 == "1" else (lambda t: t)
        arr.batch_bit_xor(own(ti(iA)), own(tv(vA))).spawn()
        hS = arr.batch_swap(own(ti(iS)), own(tv(vS))).spawn()
        arr.batch_bit_or(own(ti(iO)), own(tv(vO))).spawn()
        assert k._deferred is not None                    # nothing applied yet
        rS = hS.block()                                   # flush point
        stages = k.profile_read(reset=True)
    finally:
        k.profile(False)
    assert k._deferred is None
    # two-level: xor (count-free) applied at the switch, swap + or in one sweep; wide: one sweep
    assert stages["tile_apply"][1] == (1 if wide4 == "1" else 2), stages
    final = arr.to_numpy()
    s1 = _fold(XOR, s0, iA, vA)
    rs = rS.cpu().numpy().view(np.uint32)
    s2 = _swap_final(s1, iS, vS, rs)
    st, bad = orc.check_linearizable(1, U32, np.uint32, SWAP, s1, s2, iS, vS, rs)
    assert st == 0, ("swap", st, bad)
    assert np.array_equal(final, _fold(OR, s2, iO, vO))
    # a read flushes too: a batch followed by local_data() sees the batch applied
    arr.batch_add(ti(iA), tv(vA)).spawn()
    after = arr.local_data().cpu().numpy().view(np.uint32)
    assert np.array_equal(after, _fold(ADD, final, iA, vA))


def test_small_stream_after_other_op_phase(world, lam):
    """A small stream (applied at once) staged after records of another op is applied
    after them: the session's earlier phases go first."""
    k = world.team().kernels
    dt = lam.dtype_of("u32")
    rng = np.random.default_rng(5)
    shard = to_dev(np.zeros(L, np.uint32))
    i0 = rng.integers(0, 1000, N).astype(np.uint64)
    res = k.empty(N, torch.int32)
    k.stage_begin(shard, L, 1, dt, FETCH_ADD)
    k.stage_soa(to_dev(i0), 8, None, 1, N, res)            # staged (counted region)
    k.stage_op(STORE)
    k.stage_soa(to_dev(np.arange(1000, dtype=np.uint64)), 8, None, 7, 1000)   # small: applied now
    k.stage_op(ADD)
    k.stage_soa(to_dev(i0), 8, None, 1, N)                 # staged again, after the store
    k.stage_finish()
    assert k.errors() == 0
    got = shard.cpu().numpy().view(np.uint32)[:1000]
    ref = np.full(1000, 7, np.uint32)
    np.add.at(ref, i0.astype(np.int64), 1)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("wide4", ["1", "0"], ids=["wide", "two-level"])
def test_fused_partition_groups(world, lam, monkeypatch, wide4):
    """Counted regions are partitioned together at the finish: one count / coarse / fine
    launch per group of up to 8 pending regions of one index width (u64 global and u32
    local indices here, 11 counted phases -> groups of 2, 3 and 6 regions: 3 launches per
    pass), each region with its own count rows, tile totals and tables; the final shard is
    the serial per-phase replay, bit for bit. On the wide path (LMR_WIDE4=1, the default for this
    shard) the count-free first phase joins the counted ones (groups of 3, 3 and 6 regions: 3 count
    and 3 scatter launches, no fine pass)."""
    monkeypatch.setenv("LMR_WIDE4", wide4)
    k = world.team().kernels
    dt = lam.dtype_of("u32")
    rng = np.random.default_rng(31337)
    hot = rng.choice(L, 20000, replace=False)
    s0 = rng.integers(0, 2**32, L, dtype=np.uint64).astype(np.uint32)
    widths = [8, 8, 4, 4, 4, 8, 8, 8, 8, 8, 8]
    ops = [XOR] + [ADD if j % 2 == 0 else XOR for j in range(len(widths))]
    n = N // 2
    vals = [rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) for _ in ops]
    idxs = [_idx(rng, n, hot) for _ in ops]
    k.reserve(16 * n)
    shard = to_dev(s0)
    k.profile(True)
    k.profile_read(reset=True)
    try:
        k.stage_begin(shard, L, 1, dt, ops[0])
        k.stage_soa(to_dev(idxs[0]), 8, to_dev(vals[0]), 0, n)       # count-free, applied at the switch
        for j, w in enumerate(widths):
            k.stage_op(ops[j + 1])
            i = idxs[j + 1] if w == 8 else idxs[j + 1].astype(np.uint32)
            k.stage_soa(to_dev(i), w, to_dev(vals[j + 1]), 0, n)
        k.stage_finish()
        stages = k.profile_read(reset=True)
    finally:
        k.profile(False)
    assert k.errors() == 0
    ref = s0.copy()
    for op, v, i in zip(ops, vals, idxs):
        ref = _fold(op, ref, i, v)
    assert np.array_equal(shard.cpu().numpy().view(np.uint32), ref)
    if wide4 == "1":
        assert stages["bin_count"][1] == 3 and stages.get("fine_scatter", (0, 0))[1] == 0, stages
        assert stages["tile_apply"][1] == 1, stages
    else:
        assert stages["bin_count"][1] == 3 and stages["fine_scatter"][1] == 4, stages   # (+1: the free phase)


def test_deferred_fetch_add_batches_one_sweep(world, lam, orc):
    """Four deferred fetch_add batches (the bench's C3 pattern with a 4-batch workspace) with a
    hot element (12 % of the records) and 64 warm ones: one session, one shard sweep (the hot
    tile in delta pieces over the four regions, beside the owner tiles); the final state is the
    sum and the four batches' olds are jointly a valid linearisation (concurrent batches, as the
    reference's op AMs are)."""
    team = world.team()
    k = team.kernels
    arr = lam.AtomicArray(team, L, lam.Distribution.Block, "u32")
    rng = np.random.default_rng(4242)
    nb = 1 << 19
    s0 = rng.integers(0, 2**32, L, dtype=np.uint64).astype(np.uint32)
    arr.local_data().copy_(torch.from_numpy(s0.view(np.int32)).to(k.device))
    hot_el = int(rng.integers(0, L))
    warm = rng.choice(L, 64, replace=False)
    idxs, vals = [], []
    for _ in range(4):
        r = rng.random(nb)
        w = warm[rng.integers(0, warm.size, nb)]
        idxs.append(np.where(r < 0.12, hot_el, np.where(r < 0.3, w, rng.integers(0, L, nb))).astype(np.uint64))
        vals.append(rng.integers(1, 9, nb, dtype=np.uint64).astype(np.uint32))
    ti = lambda a: torch.from_numpy(a.astype(np.int64)).to(k.device)
    tv = lambda a: torch.from_numpy(a.view(np.int32)).to(k.device)
    k.reserve(4 * nb)
    k.profile(True)
    k.profile_read(reset=True)
    try:
        hs = [arr.batch_fetch_add(ti(i), tv(v)).spawn() for i, v in zip(idxs, vals)]
        assert k._deferred is not None                    # nothing applied yet
        rs = [h.block() for h in hs]
        stages = k.profile_read(reset=True)
    finally:
        k.profile(False)
    assert k.errors() == 0
    assert stages["tile_apply"][1] == 1, stages         # one sweep for the four batches
    final = arr.to_numpy()
    iall, vall = np.concatenate(idxs), np.concatenate(vals)
    rall = np.concatenate([r.cpu().numpy().view(np.uint32) for r in rs])
    assert np.array_equal(final, _fold(ADD, s0, iall, vall))
    st, bad = orc.check_linearizable(1, U32, np.uint32, FETCH_ADD, s0, final, iall, vall, rall)
    assert st == 0, (st, bad)
