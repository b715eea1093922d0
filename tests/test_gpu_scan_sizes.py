"""Counted partitions whose per-(tile, producer block) count scan holds more than 64K counters,
so the single-pass look-back scan (k_scan_lookback, lmr_scan.hip) runs rather than the one-block
scan every smaller test case takes: a one-shot two-level partition of 2^21 records over 8192 tiles
(32 producer blocks: 262144 counters, 64 look-back tiles), twice in a row on one context (the
scan's status words must be left zeroed for the next call).

fetch_add of ones is exact and checkable at this size without the oracle's serial replay: the
final count of every element equals its record count, and the olds returned for element e are
exactly 0 .. count(e) - 1 (one serial order per element). swap then checks the same scan with a
returning, non-combinable op: per element, the olds plus the final value are the initial value
and the swapped-in values, each once."""
import numpy as np
import pytest
import torch

from opgen import FETCH_ADD, SWAP
from test_gpu_parity import KIND_NATIVE

pytestmark = pytest.mark.gpu

TILE_ELEMS = {"u64": 8192, "u32": 16384}
TORCH = {"u64": torch.int64, "u32": torch.int32}


def _apply(k, lam, dt, shard, op, idx, vals):
    n = idx.numel()
    eb = 8 if dt == "u64" else 4
    res = torch.zeros(n * eb, dtype=torch.uint8, device="cuda")
    k.apply_soa(shard, shard.numel(), KIND_NATIVE, lam.dtype_of(dt), op, idx, 8, vals, 0, n, res, None, 0, 0)
    k.synchronize()
    k.check_errors()
    return res.view(TORCH[dt])


@pytest.mark.parametrize("dt", ["u64", "u32"])
def test_lookback_scan_counted_oneshot(world, lam, dt, monkeypatch):
    monkeypatch.setenv("LMR_STAGED", "0")                 # the one-shot counted partition
    k = world.team().kernels
    n = 1 << 21
    k.reserve(n)
    old_strategy = k.strategy
    k.strategy = 2                                        # tiled
    try:
        L = 8192 * TILE_ELEMS[dt]                         # 8192 tiles: two-level, 512 MiB
        g = torch.Generator(device="cuda")
        g.manual_seed(99)
        for rep in range(2):
            idx = torch.randint(0, L, (n,), dtype=torch.int64, device="cuda", generator=g)
            shard = torch.zeros(L, dtype=TORCH[dt], device="cuda")
            ones = torch.ones(n, dtype=TORCH[dt], device="cuda")
            olds = _apply(k, lam, dt, shard, FETCH_ADD, idx, ones).to(torch.int64)
            cnt = torch.bincount(idx, minlength=L)
            assert torch.equal(shard.to(torch.int64), cnt), f"final counts differ (rep {rep})"
            key = idx * (1 << 24) + olds                  # olds < 2^24 here
            s = torch.sort(key).values
            si, so = s >> 24, s & ((1 << 24) - 1)
            _, counts = torch.unique_consecutive(si, return_counts=True)
            starts = torch.repeat_interleave(torch.cumsum(counts, 0) - counts, counts)
            rank = torch.arange(n, device="cuda") - starts
            assert torch.equal(so, rank), f"fetch_add olds are not 0..count-1 per element (rep {rep})"
            del shard, ones, olds, key, s
        # swap: a returning op that does not combine. Every value is unique and below 2^31
        # (initial values 0..L-1, swapped-in values L..L+n-1), so per element the olds and the
        # final value must be exactly its initial value and the values swapped into it
        idx = torch.randint(0, L, (n,), dtype=torch.int64, device="cuda", generator=g)
        init = torch.arange(L, dtype=torch.int64, device="cuda")
        shard = init.to(TORCH[dt], copy=True)            # (a u64 shard must not alias init)
        vals = torch.arange(L, L + n, dtype=torch.int64, device="cuda")
        olds = _apply(k, lam, dt, shard, SWAP, idx, vals.to(TORCH[dt])).to(torch.int64)
        seen = torch.cat([olds, shard.to(torch.int64)])
        seen_at = torch.cat([idx, init])                  # the element each seen value came from
        want = torch.cat([init, vals])
        want_at = torch.cat([init, idx])                  # the element each value belongs to
        so, po = torch.sort(seen)
        wo, pw = torch.sort(want)
        assert torch.equal(so, wo), "swap olds and finals are not the values held"
        assert torch.equal(seen_at[po], want_at[pw]), "a swap old came from another element"
    finally:
        k.strategy = old_strategy
