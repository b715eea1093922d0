"""Shards above one tiled window (2^14 tiles: 2^27 u64 / 2^28 u32 elements).

The reference puts no limit on a PE's shard (src/array/unsafe.rs:178-274). Here a
larger shard is applied window by window (csrc/lmr_window.hip): records are
grouped by window, each window takes the tiled path on its slice. These tests run
AUTO on shards just above the window, at a reduced record count, and assert via
lmr_ctx_profile that the window partition and the tiled stages ran (no direct
atomics); results are checked against the oracle on the touched elements (final
state serially replayed; returned values against the linearizability checker).
"""
import numpy as np
import pytest
import torch

from opgen import ADD, CODE, FETCH_ADD, NP, SWAP
from test_gpu_parity import kind_for

pytestmark = pytest.mark.gpu

WINDOW = {8: 1 << 27, 4: 1 << 28}


def _touched(idx):
    uniq = np.unique(idx)
    return uniq, np.searchsorted(uniq, idx).astype(np.uint64)


@pytest.mark.parametrize("dt,extra", [("u64", 4099), ("u32", 333), ("i64", 1 << 20)])
def test_shard_above_one_window_takes_tiled_path(world, orc, lam, dt, extra):
    k = world.team().kernels
    t = NP[dt]
    eb = np.dtype(t).itemsize
    win = WINDOW[eb]
    shard_len = win + extra
    rng = np.random.default_rng(4242 + eb)
    n = 1 << 21
    idx = rng.integers(0, shard_len, n).astype(np.uint64)
    idx[: n // 20] = rng.integers(win - 64, min(shard_len, win + 64), n // 20)   # around the window edge
    idx[n // 20: n // 10] = rng.integers(shard_len - 100, shard_len, n // 10 - n // 20)   # the last elements
    rng.shuffle(idx)
    uniq, pos = _touched(idx)
    d_uniq = torch.from_numpy(uniq.view(np.int64)).cuda()
    dt_obj = lam.dtype_of(dt)
    kind = kind_for(dt)
    shard = torch.zeros(shard_len * eb, dtype=torch.uint8, device="cuda")
    view = shard.view(dt_obj.torch)
    d_idx = torch.from_numpy(idx.view(np.int64)).cuda()
    old_strategy = k.strategy
    k.strategy = 0                                          # AUTO
    k.profile(True)
    try:
        for op in (ADD, FETCH_ADD, SWAP):
            vals = rng.integers(0, 1 << 20, n).astype(t)
            d_vals = torch.from_numpy(vals.view(np.uint8).copy()).cuda()
            before = view[d_uniq].cpu().numpy().view(t).copy()
            res = torch.zeros(n * eb, dtype=torch.uint8, device="cuda") if op != ADD else None
            k.profile_read(reset=True)
            k.apply_soa(shard, shard_len, kind, dt_obj, op, d_idx, 8, d_vals, 0, n, res, None)
            stages = k.profile_read(reset=True)
            assert k.errors() == 0
            assert stages["window"][1] >= 1, stages
            assert stages["tile_apply"][1] >= 2, stages        # one tile sweep per window
            assert stages["direct"][1] == 0, stages
            after = view[d_uniq].cpu().numpy().view(t)
            if op == ADD:
                ref = before.copy()
                L = orc.layout_new(uniq.size, 1, 0, 0)
                st, _, _ = orc.batch_op(L, [ref], kind, CODE[dt], t, op, pos, vals)
                assert st == 0 and np.array_equal(ref, after)
            else:
                got = res.cpu().numpy().view(t)
                st, bad = orc.check_linearizable(kind, CODE[dt], t, op, before, after, pos, vals, got, None)
                assert st == 0, (op, st, bad)
        # an out-of-bounds record raises OOB and is dropped; the rest still apply
        oob = idx[:70000].copy()
        oob[123] = shard_len
        before = view[d_uniq].cpu().numpy().view(t).copy()
        k.apply_soa(shard, shard_len, kind, dt_obj, ADD, torch.from_numpy(oob.view(np.int64)).cuda(), 8, None,
                    1, oob.size)
        from lamellar_runtime_amd.types import ERRBIT_OOB
        assert k.errors() & ERRBIT_OOB
        after = view[d_uniq].cpu().numpy().view(t)
        keep = np.delete(oob, 123)
        exp = before.copy()
        np.add.at(exp, np.searchsorted(uniq, keep), t(1))
        assert np.array_equal(after, exp)
    finally:
        k.profile(False)
        k.strategy = old_strategy
