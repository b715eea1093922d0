"""The CPU baselines bench.py reports (oracle/cpu_baseline.c) compute the right thing:
the threaded 1-PE apply and the 8-PE shared-memory exchange (C4) end in the oracle's
state. They are timed baselines, so only their results are checked here."""
import numpy as np
import pytest


@pytest.mark.parametrize("threads", [1, 4, 8])
def test_threaded_apply_matches_oracle(orc, threads):
    rng = np.random.default_rng(threads)
    el, n = 5000, 300000
    shard = rng.integers(0, 2**40, el, dtype=np.uint64)
    ref = shard.copy()
    gidx = rng.integers(0, el, n, dtype=np.uint64)
    vals = rng.integers(0, 2**40, n, dtype=np.uint64)
    st, t, _ = orc.cpu_baseline(3, np.uint64, 0, shard, gidx, vals, threads)
    assert st == 0 and t.n_buffers > 1
    np.add.at(ref, gidx.astype(np.int64), vals)
    assert np.array_equal(shard, ref)


@pytest.mark.parametrize("npes,tpe,dtype,code,op", [(8, 2, np.uint64, 3, 0), (3, 1, np.uint32, 2, 14),
                                                    (4, 4, np.int16, 5, 2)])
def test_multi_pe_exchange_matches_oracle(orc, npes, tpe, dtype, code, op):
    """C4 baseline: every PE's records reach their owner through the checksummed command
    queues and are applied once (add / xor / sub, Block layout with a ragged last PE)."""
    rng = np.random.default_rng(npes)
    alen, n = 100003, 120000
    L = orc.layout_new(alen, npes, 0, 0)
    shards = [np.zeros(orc.num_elems_pe(L, p), dtype=dtype) for p in range(npes)]
    g = [rng.integers(0, alen, n, dtype=np.uint64) for _ in range(npes)]
    v = [rng.integers(0, 1000, n).astype(dtype) for _ in range(npes)]
    st, t = orc.cpu_baseline_multi_pe(code, dtype, op, alen, shards, g, v, tpe)
    assert st == 0 and t.n_buffers >= npes
    sim = [np.zeros_like(s) for s in shards]
    for p in range(npes):
        orc.batch_op(L, sim, 1, code, dtype, op, g[p], v[p])
    for p in range(npes):
        assert np.array_equal(shards[p], sim[p]), p
