"""Deferred 1-PE batches and who owns their input (engine._local, DeviceKernels.defer_soa).

The reference consumes a batch's input when the batch is built: the pack copies every record
into op buffers before batch_* returns (src/array/unsafe/operations.rs:663-811), and a Vec input
is moved in. So a caller may change its own buffers right after spawn(). Here a deferred batch
whose input is the caller's device tensor is partitioned at spawn, in stream order, and shares
only the shard sweep with the batches after it; inputs handed over with Owned(...) (Rust's
by-value Vec) stay with the session, which partitions them together at the flush.

Also C2's headline path at scale: two deferred 2^22-record u64 batch_add batches from distinct
input buffers in one session (count-free staged regions, one shard sweep), the final shard
bit-exact against the oracle's serial replay (orc.batch_op, the reference's sequential apply)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

L = (1 << 21) + 77              # u64: 257 tiles of 8192 elements (two-level partition)
N = 1 << 18


def _ti(a):
    return torch.from_numpy(np.ascontiguousarray(a).astype(np.int64)).cuda()


def _tv(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()


def _replay(orc, lam, s0, batches, op):
    """The oracle's sequential apply of the batches, in issue order (1 PE, Block)."""
    Lo = orc.layout_new(s0.size, 1, 0, 0)
    ref = s0.copy()
    rets = []
    for i, v in batches:
        st, res, _ = orc.batch_op(Lo, [ref], 1, lam.dtype_of("u64").code, np.uint64, op, i, v)
        assert st == 0
        rets.append(res)
    return ref, rets


def test_borrowed_inputs_changed_after_spawn(world, lam, orc):
    """batch_add, then the caller overwrites its index and value tensors in place and spawns
    again, then a fetch_add over the same (overwritten again) tensors: every batch applies the
    records its tensors held at its spawn. The final shard is the serial replay bit for bit
    (wrapping adds commute); fetch_add's olds are exact because its indices are a permutation."""
    team = world.team()
    k = team.kernels
    arr = lam.AtomicArray(team, L, lam.Distribution.Block, "u64")
    rng = np.random.default_rng(515)
    s0 = rng.integers(0, 2**63, L, dtype=np.uint64)
    arr.local_data().copy_(_tv(s0))
    i0, v0 = rng.integers(0, L, N).astype(np.uint64), rng.integers(0, 2**63, N, dtype=np.uint64)
    i1, v1 = rng.integers(0, L, N).astype(np.uint64), rng.integers(0, 2**63, N, dtype=np.uint64)
    i2, v2 = rng.permutation(L)[:N].astype(np.uint64), rng.integers(0, 2**63, N, dtype=np.uint64)
    k.reserve(4 * N)
    idx, vals = _ti(i0), _tv(v0)
    arr.batch_add(idx, vals).spawn()
    idx.copy_(_ti(i1))
    vals.copy_(_tv(v1))
    arr.batch_add(idx, vals).spawn()
    idx.copy_(_ti(i2))
    vals.copy_(_tv(v2))
    h = arr.batch_fetch_add(idx, vals).spawn()
    idx.fill_(0)                                          # changed again before anything is applied
    vals.fill_(1)
    olds = h.block().cpu().numpy().view(np.uint64)
    ref2 = s0.copy()
    Lo = orc.layout_new(L, 1, 0, 0)
    for (i, v), op in zip([(i0, v0), (i1, v1), (i2, v2)], [0, 0, 1]):
        st, res, _ = orc.batch_op(Lo, [ref2], 1, lam.dtype_of("u64").code, np.uint64, op, i, v)
        assert st == 0
    assert k.errors() == 0
    assert np.array_equal(arr.to_numpy(), ref2)
    assert np.array_equal(olds, res)


def test_owned_inputs_share_the_partition(world, lam, orc):
    """Owned inputs stay with the session: three batch_add batches are partitioned by one fused
    launch per pass and applied in one sweep; the final shard is the serial replay."""
    team = world.team()
    k = team.kernels
    arr = lam.AtomicArray(team, L, lam.Distribution.Block, "u64")
    rng = np.random.default_rng(616)
    s0 = rng.integers(0, 2**63, L, dtype=np.uint64)
    arr.local_data().copy_(_tv(s0))
    batches = [(rng.integers(0, L, N).astype(np.uint64), rng.integers(0, 2**63, N, dtype=np.uint64))
               for _ in range(3)]
    k.reserve(4 * N)
    arr.local_data()                                      # flush point: nothing pending
    k.profile(True)
    k.profile_read(reset=True)
    try:
        for i, v in batches:
            arr.batch_add(lam.Owned(_ti(i)), lam.Owned(_tv(v))).spawn()
        world.wait_all()
        owned = k.profile_read(reset=True)
        for i, v in batches:                              # the same batches borrowed
            arr.batch_add(_ti(i), _tv(v)).spawn()
        world.wait_all()
        borrowed = k.profile_read(reset=True)
    finally:
        k.profile(False)
    assert k.errors() == 0
    ref, _ = _replay(orc, lam, s0, batches + batches, 0)
    assert np.array_equal(arr.to_numpy(), ref)
    assert owned["tile_apply"][1] == 1 and borrowed["tile_apply"][1] == 1, (owned, borrowed)
    assert owned["bin_scatter"][1] == 1, owned            # one fused coarse launch for the three
    assert borrowed["bin_scatter"][1] == 3, borrowed      # one per batch, at its spawn


@pytest.mark.parametrize("owned", [False, True])
def test_c2_headline_session_matches_oracle(world, lam, orc, owned):
    """C2's bench path at 2^22 records per batch: AtomicArray<u64> of 2^23 elements (1024 tiles),
    uniform random indices, random u64 values, two batches from distinct buffers deferred into
    one session (count-free staged regions: no count pass, one shard sweep), as bench.py issues
    them. Final shard == the oracle's serial replay, bit for bit."""
    team = world.team()
    k = team.kernels
    Lc, n = 1 << 23, 1 << 22
    arr = lam.AtomicArray(team, Lc, lam.Distribution.Block, "u64")
    rng = np.random.default_rng(2828 + owned)
    s0 = rng.integers(0, 2**64 - 1, Lc, dtype=np.uint64)
    arr.local_data().copy_(_tv(s0))
    batches = [(rng.integers(0, Lc, n).astype(np.uint64), rng.integers(0, 2**64 - 1, n, dtype=np.uint64))
               for _ in range(2)]
    k.reserve(2 * n)
    dev = [(_ti(i), _tv(v)) for i, v in batches]
    arr.local_data()
    k.profile(True)
    k.profile_read(reset=True)
    try:
        for i, v in dev:
            arr.batch_add(lam.Owned(i) if owned else i, lam.Owned(v) if owned else v).spawn()
        world.wait_all()
        stages = k.profile_read(reset=True)
    finally:
        k.profile(False)
    assert k.errors() == 0
    assert stages["tile_apply"][1] == 1, stages           # one sweep for both batches
    assert stages["bin_count"][1] == 0, stages            # count-free regions
    ref, _ = _replay(orc, lam, s0, batches, 0)
    assert np.array_equal(arr.to_numpy(), ref)
