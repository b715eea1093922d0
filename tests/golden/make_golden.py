#!/usr/bin/env python3
"""Generate the committed golden fixtures in tests/golden/ (inputs + expected outputs).

The reference (Rust) cannot be built or run here and its tests are unseeded, so
these vectors come from the CPU oracle, itself pinned by the reference's own
known-answer tests (tests/test_oracle_known_answers.py). They freeze the
oracle's semantics per op and type so (1) regressions of the oracle show up on
CPU and (2) the GPU tests can check the device against data, not code.

Per element type: for every op available on AtomicArray<T>, a conflict-free
batch (each element targeted once: final state and per-record results are
order-independent, so bit-exact) plus colliding order-independent batches.
Layout tables for Block/Cyclic/sub-arrays at 3 PEs.
run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as orc  # noqa: E402
from opgen import (CAS, CAS_EPS, CODE, COMMUTATIVE_INT, DTYPE_NAMES, IS_FLOAT, NP, cas_operands,  # noqa: E402
                   ops_for, rand_elems, rand_vals)

SHARD, NREC = 400, 300


def kind_for(dt):
    return 2 if IS_FLOAT[dt] else 1


def make_dtype(dt):
    rng = np.random.default_rng(0x1A3E11A2 + CODE[dt])
    out = {}
    L = orc.layout_new(SHARD, 1, 0, 0)
    for op in ops_for(dt):
        shard0 = rand_elems(dt, SHARD, rng, op)
        idx = rng.permutation(SHARD)[:NREC].astype(np.uint64)
        vals = rand_vals(dt, NREC, rng, op)
        cur = eps = None
        if op in (CAS, CAS_EPS):
            cur, eps, shard0 = cas_operands(dt, shard0, vals, rng)
        final = shard0.copy()
        st, res, ok = orc.batch_op(L, [final], kind_for(dt), CODE[dt], NP[dt], op, idx, vals, cur, eps)
        assert st == 0
        p = f"op{op}_"
        out[p + "shard0"], out[p + "idx"], out[p + "vals"] = shard0, idx, vals
        out[p + "final"], out[p + "results"], out[p + "ok"] = final, res, ok
        out[p + "cur"] = np.array([cur if cur is not None else 0]).astype(NP[dt])
        out[p + "eps"] = np.array([eps if eps is not None else 0]).astype(NP[dt])
    if not IS_FLOAT[dt]:
        for op in sorted(COMMUTATIVE_INT):
            shard0 = rand_elems(dt, 64, rng, op)
            idx = rng.integers(0, 64, 1000).astype(np.uint64)
            vals = rand_vals(dt, idx.size, rng, op)
            final = shard0.copy()
            L64 = orc.layout_new(64, 1, 0, 0)
            st, _, _ = orc.batch_op(L64, [final], 1, CODE[dt], NP[dt], op, idx, vals)
            assert st == 0
            p = f"coll{op}_"
            out[p + "shard0"], out[p + "idx"], out[p + "vals"], out[p + "final"] = shard0, idx, vals, final
    np.savez_compressed(os.path.join(HERE, f"golden_{dt}.npz"), **out)


def make_layouts():
    out = {}
    for dist in (0, 1):
        for size, sub in ((1000, None), (1001, None), (2, None), (1000, (123, 877)), (50, (7, 8))):
            L = orc.layout_new(size, 3, 0, dist)
            if sub:
                L = orc.layout_sub(L, *sub)
            key = f"d{dist}_s{size}_" + (f"sub{sub[0]}_{sub[1]}" if sub else "full")
            tab = np.array([orc.pe_and_offset(L, i) or (2**64 - 1, 2**64 - 1) for i in range(L.size + 2)],
                           dtype=np.uint64)
            out[key + "_map"] = tab
            out[key + "_num_elems"] = np.array([orc.num_elems_pe(L, p) for p in range(3)], dtype=np.uint64)
            out[key + "_slice_start"] = np.array([orc.local_slice_start(L, p) for p in range(3)], dtype=np.uint64)
            out[key + "_index_size"] = np.array([orc.index_size(L)], dtype=np.uint64)
            out[key + "_layout"] = np.array(L.as_tuple(), dtype=np.uint64)
    np.savez_compressed(os.path.join(HERE, "golden_layouts.npz"), **out)


if __name__ == "__main__":
    for dt in DTYPE_NAMES:
        make_dtype(dt)
    make_layouts()
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))
