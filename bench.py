#!/usr/bin/env python3
"""Benchmark of the MI355X batched element-op path (BASELINE.json metric:
"batched array ops applied/sec (device-resident), 1/2/4/8 MI355X").

A step = one pass of the hot path over one batch of synthetic device-resident
input, every PE (one per GPU) issuing its own batch (weak scaling):
  c2 (default, N = 1): AtomicArray<u64>::batch_add(indices, vals), 2^28
      records, uniform-random global indices into a 2^26-element array; the
      local lamellae: no pack, no exchange.
  c4 (default, N > 1): the same batch per PE, indices uniform over the whole
      N * 2^26-element Block array: device pack by destination PE -> RCCL
      all-to-all(v) over xGMI -> device apply on every shard.
  c3: AtomicArray<f64>::batch_fetch_add, 2^26 records, Zipf(0.99) ranks over
      2^24 elements (ranks randomly permuted), vals = 1.0, olds returned.
  c5: AtomicArray<u32>, five batches per step (bit_and, bit_or, bit_xor, swap,
      compare_exchange), 2^30 / 8 records per PE split in equal fifths.
value = ops applied by all PEs / max-over-PEs wall time of the timed steps.

roofline: op-level, for the whole step: SURVEY 8(d)'s algorithmic bytes per op
(packed record + element read and write [+ returned value]) x ops per step / the
step time, against the 8.0 TB/s HBM3E peak; `traffic` is the HBM bytes per step
from the committed rocprofv3 PMC passes. Each kernel stage's own algorithmic bytes
over its average launch time (HIP events the library records on the launch
stream) are under apply_pipeline.stages. cpu_baseline: the reference-structured
threaded CPU apply (oracle/cpu_baseline.c, a restatement of the Rust path: the
reference itself cannot be built here) on a bounded sample, rank 0, N = 1, with
3 warm-up runs; extra lines for T = 4, C1 and the 8-PE shared-memory C4 shape.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c5]
       python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from _lamellar_bootstrap import load_package  # noqa: E402

HBM_PEAK = 8.0e12          # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "batched array ops applied/sec (device-resident), 1/2/4/8 MI355X"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default=None, choices=[None, "c2", "c3", "c4", "c5"])
    p.add_argument("--records-log2", type=int, default=None)
    p.add_argument("--elems-log2", type=int, default=None)
    p.add_argument("--strategy", default=os.environ.get("LAMELLAR_OP_STRATEGY", "auto"))
    p.add_argument("--cpu-threads", type=int, default=0, help="0: every core this process may run on")
    p.add_argument("--cpu-sample-log2", type=int, default=25)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--input-sets", type=int, default=0,
                   help="distinct input buffers rotated over the steps (0: one per step of a deferred "
                        "session, up to 16)")
    p.add_argument("--reserve-log2", type=int, default=30,
                   help="tiled-apply workspace (records, log2; 0: the step's records). The engine defers "
                        "large 1-PE batches into one staged session until the workspace is full, so a "
                        "2^30-record workspace (49 GB of the 288 GB of HBM) sweeps the shard once per four "
                        "C2 / sixteen C3 batches (2^29: two / eight; the C2 step then ran 3.16 or 3.37 ms "
                        "from box to box, 2^30 3.165-3.167, profiles/r5/ab_reserve/)")
    p.add_argument("--reserve-records", type=int, default=0,
                   help="tiled-apply workspace in records (overrides --reserve-log2 when set)")
    p.add_argument("--inputs", default="owned", choices=["owned", "borrowed"],
                   help="owned: each batch's input tensors are handed over with Owned(...) (the "
                        "reference's by-value Vec input; the bench never changes them), so consecutive "
                        "deferred batches are partitioned together; borrowed: plain tensors, each "
                        "batch partitioned at its spawn")
    p.add_argument("--no-other-configs", action="store_true",
                   help="default run only: skip the short C3 / C5 lines (other_configs)")
    p.add_argument("--e2e", action="store_true",
                   help="also time the host-buffer path: pinned host records -> H2D copy -> op")
    return p.parse_args()


def stage_bytes_per_op(stage, iw, vb, eb, n, shard_len, fetch, wide=False):
    """Algorithmic HBM bytes per op of each kernel stage (Kernels):
    the bytes a stage must read and write per record, shard traffic amortised.
    Returned values travel binned -> temp -> input order through stored u32 maps
    (qpos written by the coarse pass, rpos by the fine pass). fetch: the share of records
    whose op returns a value (C5: 2 of 5 batches); the un-partition counts only those.
    wide: the one-level staged partition (lmr_wide.hip: 8-byte elements, <= 2^24 of them, or
    1/2/4-byte elements, <= 2^26):
    the scatter writes u16 tile offsets and a u16 staging position per record, one gather
    brings the olds back."""
    pos = 4 * float(fetch)
    res = eb * float(fetch)
    if wide:
        return {"bin_count": iw,
                "bin_scatter": iw + vb + 2 + vb + 2 * float(fetch),
                "tile_apply": 2 + vb + res + 2.0 * eb * shard_len / max(n, 1),
                "unpartition": (2 + 2 * eb) if fetch else 0.0}.get(stage, 0.0)
    tile_elems = 65536 // max(eb, 4)
    two_level = (shard_len + tile_elems - 1) // tile_elems > 128
    return {
        "direct": iw + vb + 2 * eb + res,
        "bin_count": iw,
        "bin_scatter": iw + vb + 4 + vb + pos,          # coarse pass: record in, temp record (+ qpos) out
        "fine_scatter": 4 + vb + 2 + vb + pos,          # temp record in, tile-local record (+ rpos) out
        "tile_apply": 2 + vb + res + 2.0 * eb * shard_len / max(n, 1),
        "unpartition": (2 if two_level else 1) * (4 + 2 * eb) if fetch else 0.0,
        # count-free pack (nothing returned): record in, record out; the counted pack of
        # returning ops adds the count pass's index read and the u32 position out
        "pack": 8 + vb + iw + vb + 12 * float(fetch),
        "scatter_results": 4 + 2 * eb,
        "mvsi": vb + res,
        "window": 2 * iw + vb + 4 + vb + pos,           # count (idx) + scatter (idx, val in; u32 idx, val, pos out)
    }.get(stage, 0.0)


class Workload:
    """One BASELINE.json configuration: array + inputs + the step."""

    def __init__(self, lam, team, args):
        self.lam, self.team, self.args = lam, team, args
        self.k = team.kernels
        self.dev = self.k.device
        self.npes, self.me = team.num_pes(), team.my_pe()

    def gen(self):
        g = torch.Generator(device=self.dev)
        g.manual_seed(0x1A3E11A2 + self.me)
        return g

    t = 0          # steps issued (selects the input set)
    sets = None    # distinct input buffers, one per step of a deferred session

    def make_sets(self, nsets):
        """Distinct copies of the step's records (each a random permutation of them, so every step
        applies the same multiset and the verify invariants hold), rotated over consecutive steps:
        the batches one deferred session sweeps together read different buffers, as distinct
        batches of a real caller would, so none of them is served from a cache the previous
        batch's pass left warm."""
        g = torch.Generator(device=self.dev)
        g.manual_seed(0x5E75 + self.me)
        base = self.inputs()
        self.sets = [base]
        for _ in range(1, max(1, nsets)):
            cp = []
            for i, v in base:
                perm = torch.randperm(i.numel(), device=self.dev, generator=g)
                cp.append((i[perm].contiguous(), v[perm].contiguous()))
            self.sets.append(cp)

    def next_inputs(self):
        s = self.sets[self.t % len(self.sets)] if self.sets else self.inputs()
        self.t += 1
        if self.args.inputs == "owned":
            own = self.lam.Owned
            s = [(own(i), own(v)) for i, v in s]
        return s


class AddUniform(Workload):
    """C2 (N = 1) / C4 (N > 1): u64 batch_add, uniform indices."""
    dtype, fetch, eb, vb = "u64", False, 8, 8

    def setup(self):
        a = self.args
        self.n = 1 << (a.records_log2 or 28)
        self.elems = 1 << (a.elems_log2 or 26)
        glen = self.elems * self.npes
        self.arr = self.lam.AtomicArray(self.team, glen, self.lam.Distribution.Block, "u64")
        g = self.gen()
        self.idx = torch.randint(0, glen, (self.n,), dtype=torch.int64, device=self.dev, generator=g)
        self.vals = torch.randint(-2**63, 2**63 - 1, (self.n,), dtype=torch.int64, device=self.dev, generator=g)
        self.ops_per_step = self.n

    def inputs(self):
        return [(self.idx, self.vals)]

    def step(self):
        (i, v), = self.next_inputs()
        self.arr.batch_add(i, v).spawn()

    def verify(self, nsteps):
        # wrapping-sum invariant: sum(array) == steps * sum(vals), over all PEs (mod 2^64)
        s_arr = self.arr.local_data().sum(dtype=torch.int64)
        s_val = self.vals.sum(dtype=torch.int64) * nsteps
        return _allsum(self.npes, s_arr) == _allsum(self.npes, s_val)

    def describe(self):
        a = self.args
        if self.npes == 1 and os.environ.get("LAMELLAR_FORCE_EXCHANGE", "0") == "1":
            return ("C4 one-rank rehearsal: 2^%d batched u64 add records through the forced exchange "
                    "(lmr_batch_exchange over a 1-rank RCCL communicator), uniform-random indices into "
                    "a 2^%d-element AtomicArray<u64>" % (a.records_log2 or 28, a.elems_log2 or 26))
        if self.npes == 1:
            return ("C2: 2^%d batched u64 add records, uniform-random indices into a 2^%d-element "
                    "AtomicArray<u64>" % (a.records_log2 or 28, a.elems_log2 or 26))
        return ("C4: %d PEs all-to-all batched u64 add, 2^%d records per PE, Block array of %d x 2^%d "
                "elements, op buffers via RCCL all-to-all(v) over xGMI"
                % (self.npes, a.records_log2 or 28, self.npes, a.elems_log2 or 26))

    op_name = "batch_add (ArrayOpCmd::Add, MVMI)"
    survey_bpo = 4 + 8 + 16


class FetchAddZipf(Workload):
    """C3: f64 batch_fetch_add, Zipf(0.99) over 2^24 elements (contention)."""
    dtype, fetch, eb, vb = "f64", True, 8, 8

    def setup(self):
        a = self.args
        self.n = 1 << (a.records_log2 or 26)
        self.elems = 1 << (a.elems_log2 or 24)
        glen = self.elems * self.npes
        self.arr = self.lam.AtomicArray(self.team, glen, self.lam.Distribution.Block, "f64")
        g = self.gen()
        ranks = torch.arange(1, glen + 1, dtype=torch.float64, device=self.dev)
        cdf = torch.cumsum(ranks.pow(-0.99), 0)
        cdf /= cdf[-1].clone()
        u = torch.rand(self.n, dtype=torch.float64, device=self.dev, generator=g)
        r = torch.searchsorted(cdf, u).clamp_(max=glen - 1)
        g2 = torch.Generator(device=self.dev)
        g2.manual_seed(0xC3)                                   # same rank->index map on every PE
        perm = torch.randperm(glen, device=self.dev, generator=g2)
        self.idx = perm[r].contiguous()
        self.vals = torch.ones(self.n, dtype=torch.float64, device=self.dev)
        self.ops_per_step = self.n
        self.top_share = float((r == 0).float().mean())

    def inputs(self):
        return [(self.idx, self.vals)]

    def step(self):
        (i, v), = self.next_inputs()
        self.last = self.arr.batch_fetch_add(i, v).spawn()

    def verify(self, nsteps):
        # exact with vals = 1.0: element = steps * (records hitting it, all PEs)
        cnt = torch.bincount(self.idx, minlength=self.elems * self.npes).to(torch.float64) * nsteps
        if self.npes > 1:
            import torch.distributed as dist
            dist.all_reduce(cnt)
        L = self.arr.local_data()
        lo = self.me * self.elems
        return bool(torch.equal(L, cnt[lo:lo + L.numel()]))

    def describe(self):
        a = self.args
        return ("C3: f64 fetch_add, 2^%d records per PE, Zipf(0.99) ranks (randomly permuted) over "
                "2^%d elements per PE, vals = 1.0, olds returned in input order (top element %.1f%% of "
                "records)" % (a.records_log2 or 26, a.elems_log2 or 24, 100 * self.top_share))

    op_name = "batch_fetch_add (ArrayOpCmd::FetchAdd, MVMI)"
    survey_bpo = 4 + 8 + 16 + 8


class MixedU32(Workload):
    """C5: u32 and/or/xor/swap/compare_exchange in equal fifths, one batch each."""
    dtype, fetch, eb, vb = "u32", 0.4, 4, 4         # swap and compare_exchange return values

    def setup(self):
        a = self.args
        total = 1 << (a.records_log2 or 30)
        self.n = max(5, total // 8)                               # 2^30 total over 8 PEs
        self.elems = 1 << (a.elems_log2 or 26)
        glen = self.elems * self.npes
        self.arr = self.lam.AtomicArray(self.team, glen, self.lam.Distribution.Block, "u32")
        g = self.gen()
        m = self.n // 5
        self.parts = []
        for _ in range(5):
            i = torch.randint(0, glen, (m,), dtype=torch.int64, device=self.dev, generator=g)
            v = torch.randint(-2**31, 2**31 - 1, (m,), dtype=torch.int32, device=self.dev, generator=g)
            self.parts.append((i, v))
        self.ops_per_step = 5 * m

    def inputs(self):
        return list(self.parts)

    def step(self):
        a = self.arr
        (i0, v0), (i1, v1), (i2, v2), (i3, v3), (i4, v4) = self.next_inputs()
        a.batch_bit_and(i0, v0).spawn()
        a.batch_bit_or(i1, v1).spawn()
        a.batch_bit_xor(i2, v2).spawn()
        a.batch_swap(i3, v3).spawn()
        a.batch_compare_exchange(i4, 0, v4).spawn()

    def verify(self, nsteps):
        """One more step with every result captured, checked on a sample of elements
        (global index % 1021 == 0, about 1 in 1000): bit_and / bit_or / bit_xor final
        states against the oracle's serial replay, swap olds and compare_exchange
        Results against the linearisability checker (per element, one serial order of
        that element's records from every PE). Records of every PE that hit a sampled
        element are gathered on every PE."""
        from oracle import oracle as orc
        a, dev = self.arr, self.dev
        P = 1021
        lo = self.me * self.elems
        g_local = torch.arange(lo, lo + self.elems, device=dev)
        loc = torch.nonzero(g_local % P == 0).flatten()
        mine_g = (g_local[loc]).cpu().numpy().astype(np.uint64)
        ops = [(10, "batch_bit_and"), (12, "batch_bit_or"), (14, "batch_bit_xor"), (18, "batch_swap"),
               (21, "batch_compare_exchange")]
        per_batch = []
        for (op, fn), (i, v) in zip(ops, self.parts):
            before = a.local_data()[loc].cpu().numpy().view(np.uint32)
            h = getattr(a, fn)(i, 0, v) if op == 21 else getattr(a, fn)(i, v)
            r = h.block()
            after = a.local_data()[loc].cpu().numpy().view(np.uint32)
            sel = torch.nonzero(i % P == 0).flatten()
            rec_i = i[sel].cpu().numpy().astype(np.uint64)
            rec_v = v[sel].cpu().numpy().view(np.uint32)
            rec_r = rec_ok = None
            if op == 18:
                rec_r = r[sel].cpu().numpy().view(np.uint32)
            elif op == 21:
                rec_r = r.vals[sel].cpu().numpy().view(np.uint32)
                rec_ok = r.ok[sel].cpu().numpy()
            per_batch.append((mine_g, before, after, rec_i, rec_v, rec_r, rec_ok))
        parts = [per_batch]
        if self.npes > 1:
            import torch.distributed as dist
            parts = [None] * self.npes
            dist.all_gather_object(parts, per_batch)
        u32 = np.uint32
        for b, (op, fn) in enumerate(ops):
            g = np.concatenate([pp[b][0] for pp in parts])
            order = np.argsort(g)
            g = g[order]
            before = np.concatenate([pp[b][1] for pp in parts])[order]
            after = np.concatenate([pp[b][2] for pp in parts])[order]
            ri = np.concatenate([pp[b][3] for pp in parts])
            rv = np.concatenate([pp[b][4] for pp in parts])
            pos = np.searchsorted(g, ri).astype(np.uint64)           # compact element of each record
            if op in (10, 12, 14):
                ref = before.copy()
                L = orc.layout_new(g.size, 1, 0, 0)
                st, _, _ = orc.batch_op(L, [ref], 1, 2, u32, op, pos, rv)
                if st != 0 or not np.array_equal(ref, after):
                    return False
            else:
                rr = np.concatenate([pp[b][5] for pp in parts])
                ok = np.concatenate([pp[b][6] for pp in parts]).astype(np.uint8) if op == 21 else None
                st, _ = orc.check_linearizable(1, 2, u32, op, before, after, pos, rv, rr, ok,
                                               current=u32(0) if op == 21 else None)
                if st != 0:
                    return False
        return True

    def describe(self):
        a = self.args
        return ("C5: u32 bit_and/bit_or/bit_xor/swap/compare_exchange(current=0) in five equal batches, "
                "2^%d records in total over 8 PEs (2^%d per PE), 2^%d-element shard per PE"
                % (a.records_log2 or 30, (a.records_log2 or 30) - 3, a.elems_log2 or 26))

    op_name = "batch_bit_and/or/xor, batch_swap, batch_compare_exchange"
    survey_bpo = (16 + 16 + 16 + 20 + 24) / 5


def _allsum(npes, t):
    if npes > 1:
        import torch.distributed as dist
        dist.all_reduce(t)
    return int(t.item())


def cpu_threads():
    """Logical cores this process may use: the box's CPU share per GPU where the
    environment states it (OMP_NUM_THREADS, 16 on the GPU pool, which asks worker pools
    to stay within it), else the affinity mask. os.cpu_count() (the whole machine) is
    recorded beside it."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return n


def _timed(orc, reps, run, warm=3):
    for _ in range(warm):                                  # 3 full-size warm-up runs
        run(False)
    ts = sorted(run(False) for _ in range(reps))
    return ts[len(ts) // 2], ts


def cpu_baseline(args, cfg):
    """The reference-structured threaded CPU apply (oracle/cpu_baseline.c: op buffers
    of am_size_threshold = 100 kB packed by T/4 threads, applied by T threads with
    SeqCst atomics / CAS loops (NativeAtomic) or a lock per element (GenericAtomic,
    generic_atomic.rs:286-293)) on bounded samples of the workload, median of 10
    (BASELINE.md). The primary line uses every core this process may run on; extra
    lines: T = 4 (the reference's test setting, tests/add.rs:35), and C1 (configs[0],
    the add_test pattern on 1M u64 elements) batched and as per-element 1x1 ops."""
    from oracle import oracle as orc
    T = args.cpu_threads or cpu_threads()
    rng = np.random.default_rng(0x1A3E11A2)
    out = {}

    def one(dtype, npt, op, shard_len, gidx, vals, threads, reps, threshold=100000, results=False, cur=None,
            init=None):
        shard = np.zeros(shard_len, dtype=npt) if init is None else init

        def run(_warm):
            st, t, _ = orc.cpu_baseline(dtype, npt, op, shard, gidx, vals, threads, threshold, want_results=results,
                                        current=cur)
            assert st == 0
            return t.total_s
        med, ts = _timed(orc, reps, run)
        return gidx.size / med, med, ts

    if cfg in ("c2", "c4"):
        el = 1 << (args.elems_log2 or 26)
        n = 1 << args.cpu_sample_log2
        gidx = rng.integers(0, el, n, dtype=np.uint64)
        vals = rng.integers(0, 2**63, n, dtype=np.uint64)
        v, med, _ = one(3, np.uint64, 0, el, gidx, vals, T, 10)
        out["primary"] = {"value": v, "unit": "ops/s", "cores": T, "kind": "port",
                          "sample": f"C2 shape: 2^{args.cpu_sample_log2} u64 add records uniform over a "
                                    f"2^{args.elems_log2 or 26}-element shard, 100 kB op buffers packed by "
                                    f"{max(1, T // 4)} threads, applied with SeqCst atomics by {T} threads "
                                    f"(median of 10: {med * 1e3:.0f} ms; the box's CPU share; os.cpu_count() = "
                                    f"{os.cpu_count()})"}
        n4 = n >> 2
        v4, med4, _ = one(3, np.uint64, 0, el, gidx[:n4], vals[:n4], 4, 10)
        out["extra"] = [{"value": v4, "unit": "ops/s", "cores": 4, "kind": "port",
                         "sample": f"C2 shape, T = 4 (tests/add.rs:35), 2^{args.cpu_sample_log2 - 2} records, "
                                   f"median of 10 ({med4 * 1e3:.0f} ms)"}]
        # C1: add_test pattern, 1M-element u64 array, every element updated 50 times, batch_add(indices, 1)
        c1_el = 1000000
        c1_idx = np.tile(np.arange(c1_el, dtype=np.uint64), 8)
        rng.shuffle(c1_idx)
        v1, med1, _ = one(3, np.uint64, 0, c1_el, c1_idx, np.uint64(1), T, 5)
        out["extra"].append({"value": v1, "unit": "ops/s", "cores": T, "kind": "port",
                             "sample": f"C1 (configs[0]): batch_add(indices, 1) on a 1M-element u64 array, 8 "
                                       f"shuffled updates per element (8M ops), SVMI op buffers, median of 5 "
                                       f"({med1 * 1e3:.0f} ms)"})
        n11 = 1 << 18
        v11, med11, _ = one(3, np.uint64, 0, c1_el, c1_idx[:n11], np.uint64(1), T, 5, threshold=1)
        out["extra"].append({"value": v11, "unit": "ops/s", "cores": T, "kind": "port",
                             "sample": f"C1 as add_test issues it: per-element add(idx, 1), one 1-record op "
                                       f"buffer per op (2^18 ops; a lower bound on the reference's per-AM "
                                       f"cost), median of 5 ({med11 * 1e3:.0f} ms)"})
        # C4 (configs[3]): 8 PEs on one node exchanging op buffers through shared memory, the
        # shmem lamellae's command-queue protocol restated (oracle/cpu_baseline.c), T / 8 threads each
        P = 8
        tpe = max(1, T // P)
        n4p = 1 << max(16, args.cpu_sample_log2 - 4)
        alen = P * el
        L4 = orc.layout_new(alen, P, 0, 0)
        shards = [np.zeros(orc.num_elems_pe(L4, p), dtype=np.uint64) for p in range(P)]
        g4 = [rng.integers(0, alen, n4p, dtype=np.uint64) for _ in range(P)]
        v4s = [rng.integers(0, 2**63, n4p, dtype=np.uint64) for _ in range(P)]

        def run4(_warm):
            st, t = orc.cpu_baseline_multi_pe(3, np.uint64, 0, alen, shards, g4, v4s, tpe)
            assert st == 0
            return t.total_s
        med4p, _ = _timed(orc, 5, run4)
        out["extra"].append({"value": P * n4p / med4p, "unit": "ops/s", "cores": P * tpe, "kind": "port",
                             "sample": f"C4 (configs[3]) shape: {P} PEs x {tpe} threads, 2^{n4p.bit_length() - 1} "
                                       f"u64 add records per PE uniform over a {P} x 2^{args.elems_log2 or 26}-element "
                                       f"Block array, op buffers exchanged through shared memory with the shmem "
                                       f"lamellae's checksummed command queues (restated), median of 5 "
                                       f"({med4p * 1e3:.0f} ms)"})
    elif cfg == "c3":
        el = 1 << (args.elems_log2 or 24)
        n = 1 << 22
        ranks = np.arange(1, el + 1, dtype=np.float64)
        cdf = np.cumsum(ranks ** -0.99)
        cdf /= cdf[-1]
        gidx = rng.permutation(el)[np.minimum(np.searchsorted(cdf, rng.random(n)), el - 1)].astype(np.uint64)
        vals = np.ones(n, dtype=np.float64)
        v, med, _ = one(9, np.float64, 1, el, gidx, vals, T, 10, results=True)
        out["primary"] = {"value": v, "unit": "ops/s", "cores": T, "kind": "port",
                          "sample": f"C3 shape: 2^22 f64 fetch_add records, Zipf(0.99) over 2^"
                                    f"{args.elems_log2 or 24} elements, GenericAtomic per-element locks, olds "
                                    f"returned, {T} threads (median of 10: {med * 1e3:.0f} ms)"}
    elif cfg == "c5":
        el = 1 << (args.elems_log2 or 26)
        m = 1 << 21
        tot = 0.0
        for op in (10, 12, 14, 18, 21):
            gidx = rng.integers(0, el, m, dtype=np.uint64)
            vals = rng.integers(0, 2**32, m, dtype=np.uint64).astype(np.uint32)
            _, med, _ = one(2, np.uint32, op, el, gidx, vals, T, 10, results=op in (18, 21),
                            cur=np.uint32(0) if op == 21 else None)
            tot += med
        out["primary"] = {"value": 5 * m / tot, "unit": "ops/s", "cores": T, "kind": "port",
                          "sample": f"C5 shape: u32 bit_and/bit_or/bit_xor/swap/compare_exchange, 2^21 records "
                                    f"each uniform over 2^{args.elems_log2 or 26} elements, SeqCst atomics, "
                                    f"{T} threads (sum of per-op medians of 10: {tot * 1e3:.0f} ms)"}
    return out


def main():
    args = parse()
    lam = load_package()
    world = lam.LamellarWorldBuilder().with_strategy(
        {"auto": lam.Strategy.Auto, "direct": lam.Strategy.Direct, "tiled": lam.Strategy.Tiled}[args.strategy]
    ).build()
    team = world.team()
    k = team.kernels
    npes, me = world.num_pes(), world.my_pe()
    dev = k.device
    cfg = args.config or ("c2" if npes == 1 else "c4")
    W = {"c2": AddUniform, "c4": AddUniform, "c3": FetchAddZipf, "c5": MixedU32}[cfg](lam, team, args)
    W.setup()
    ws_records = W.n
    if args.reserve_records:
        ws_records = max(W.n, args.reserve_records)
    elif args.reserve_log2:
        ws_records = max(W.n, 1 << args.reserve_log2)
    k.max_ws_records = max(k.max_ws_records, ws_records)     # (the library caps it at lmr's max_rec_cap)
    k.reserve(ws_records)
    W.make_sets(input_sets(args, k.reserved, W.ops_per_step))
    world.barrier()

    for _ in range(args.warmup):
        W.step()
    world.wait_all()
    world.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        W.step()
    world.wait_all()              # every issued batch applied (deferred ones included)
    torch.cuda.synchronize(dev)
    world.barrier()
    t1 = time.perf_counter()
    # stage breakdown from a separate pass after the timed steps: the library's stage events
    # (timing events on the launch streams, one pair per stage) cost time of their own, so the
    # timed steps above run without them
    prof_steps = max(1, min(args.steps, 10))
    k.profile(True)
    k.profile_read(reset=True)
    for _ in range(prof_steps):
        W.step()
    world.wait_all()
    torch.cuda.synchronize(dev)
    stages = k.profile_read(reset=True)
    k.profile(False)
    world.wait_all()

    elapsed = t1 - t0
    if npes > 1:
        import torch.distributed as dist
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = npes * W.ops_per_step * args.steps / elapsed
    verified = None if args.no_verify else W.verify(args.warmup + args.steps + prof_steps)

    # ---- roofline: the whole op path against HBM ----
    # achieved = B_op (the survey's algorithmic bytes per op: packed record + element
    # read/write (+ returned value)) x ops per step / the step time; frac against the
    # 8.0 TB/s HBM3E spec. Per-stage figures (each kernel's own algorithmic bytes over
    # its HIP-event launch time) live in apply_pipeline.stages.
    per = {}
    for name, (ms, cnt, recs) in stages.items():
        if cnt:
            per[name] = (ms / cnt, cnt / prof_steps, recs / cnt)
    # index bytes per record the partition passes read: the caller's u64 global indices on
    # the local path, the exchange's packed local offsets (lmr_index_size) behind a pack
    iw = 8 if npes == 1 and "pack" not in per else W.arr.index_size()
    step_s = ms_per_step * 1e-3
    achieved = W.survey_bpo * W.ops_per_step / step_s
    traffic = None
    pmc = os.path.join(ROOT, "profiles", f"pmc_traffic_{cfg}.json")
    if os.path.exists(pmc) and per:
        tr = json.load(open(pmc))
        if "_per_record" in tr and all(st in tr["_per_record"] for st in per if st not in ("scan",)):
            # bytes per record x this run's records per launch x launches per step
            pr = tr["_per_record"]
            traffic = sum(pr.get(st, 0.0) * (per[st][2] or W.ops_per_step / per[st][1]) * per[st][1] for st in per)
            if "pack" in per and "_transport_per_record" in tr:
                # RCCL's copies (send-buffer read, receive-buffer write) of the records that leave
                # this PE: all of them in the one-rank rehearsal, (N - 1) / N of them at N PEs
                share = 1.0 if npes == 1 else (npes - 1) / npes
                traffic += tr["_transport_per_record"] * share * (per["pack"][2] or W.ops_per_step) * per["pack"][1]
        elif all(st in tr for st in per if st not in ("scan",)):
            traffic = sum(tr.get(st, 0.0) * per[st][1] for st in per)
            if "pack" in per and "_transport_per_pack" in tr:     # the exchange's RCCL copies
                traffic += tr["_transport_per_pack"] * per["pack"][1]
    dom = max(per, key=lambda st: per[st][0] * per[st][1]) if per else None
    # per stage: records per launch from the library's own count (a stage may run on a
    # subset of a step's batches, e.g. C5's counted stages)
    roof = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": achieved / HBM_PEAK, "traffic": traffic,
            "traffic_source": ("HBM bytes per step: committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes "
                               f"(profiles/pmc_traffic_{cfg}.json, FETCH_SIZE x2 per the gfx950 note) x launches "
                               "per step of this run" + ("" if "pack" not in per else
                                                         "; RCCL's copies x the share of records leaving this PE")
                               + "; not measured in this run") if traffic else None,
            "scope": "whole step (every kernel of the op path), SURVEY 8(d) bytes per op",
            "bytes_per_op": W.survey_bpo, "ops_per_step": W.ops_per_step, "dominant_kernel": dom}
    stage_rows = {}
    # the wide one-level staged path (no fine pass: 8-byte shards of <= 2^24 elements, smaller
    # elements up to 2^26)
    wide = (W.elems <= (1 << 24) if W.eb == 8 else W.elems <= (1 << 26)) and "fine_scatter" not in per \
        and "tile_apply" in per
    for st, (avg_ms, lps, rpl) in per.items():
        ops_per_launch = rpl if rpl else W.ops_per_step / lps
        bpo = stage_bytes_per_op(st, iw, W.vb, W.eb, ops_per_launch, W.elems, W.fetch, wide)
        row = {"ms_per_step": avg_ms * lps, "launches_per_step": lps, "avg_launch_ms": avg_ms,
               "records_per_launch": ops_per_launch, "bytes_per_op": bpo}
        if bpo:
            row["achieved_GBps"] = bpo * ops_per_launch / (avg_ms * 1e-3) / 1e9
            row["frac"] = row["achieved_GBps"] * 1e9 / HBM_PEAK
        stage_rows[st] = row
    apply_stages = [st for st in ("direct", "mvsi", "bin_count", "scan", "bin_scatter", "fine_scatter",
                                  "tile_apply", "unpartition", "pack", "scatter_results", "window") if st in per]
    apply_ms = sum(per[st][0] * per[st][1] for st in apply_stages)

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "ops/s",
        "n_gpus": npes,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": W.dtype,
        "data": "synthetic (seeded random indices and values, device-resident)",
        "config": {
            "workload": W.describe(),
            "records_per_pe": W.ops_per_step,
            "elems_per_pe": W.elems,
            "op": W.op_name,
            "strategy": args.strategy,
            "workspace_records": k.reserved,
            "input_sets": len(W.sets) if W.sets else 1,
            "inputs": args.inputs,
            "parallelism": f"{npes} PE(s), one per GPU",
        },
        "roofline": roof,
        "apply_pipeline": {"stages": stage_rows, "profiled_steps": prof_steps,
                           "device_ms_per_step": apply_ms,
                           "frac_of_device_time": (W.survey_bpo * W.ops_per_step / (apply_ms * 1e-3) / HBM_PEAK)
                           if apply_ms else None},
        "verified": verified,
        "cpu_baseline": None,
    }
    if args.e2e and cfg in ("c2", "c4"):
        out["e2e"] = e2e(lam, team, W, args)
    if args.config is None and npes == 1 and not args.no_other_configs:
        del W
        out["other_configs"] = other_configs(lam, world, team, args)
    if me == 0 and npes == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(args, cfg)
        out["cpu_baseline"] = cb.get("primary")
        if cb.get("extra"):
            out["cpu_baselines_extra"] = cb["extra"]
    if me == 0:
        print(json.dumps(out), flush=True)
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def input_sets(args, ws_records, ops_per_step):
    """Distinct input sets: one per step a deferred session can hold (up to 16), or --input-sets."""
    if args.input_sets:
        return args.input_sets
    return int(max(1, min(16, ws_records // max(1, ops_per_step))))


def other_configs(lam, world, team, args):
    """The default run (N = 1, C2) also times BASELINE.json's other single-GPU configurations
    (C3, C5) with the same clock, fewer steps and no profiling: short reported lines beside the
    headline, each verified against its checker after its timed steps. Two more C2 lines: plain
    (borrowed) input tensors, and one batch per sweep with no deferral at all (the latency of an
    isolated 2^28-record batch)."""
    from lamellar_runtime_amd import engine
    k = team.kernels
    dev = k.device
    res = {}
    lines = (("c3", FetchAddZipf, None), ("c5", MixedU32, None),
             ("c2_borrowed", AddUniform, "borrowed"), ("c2_one_batch", AddUniform, "nodefer"))
    for cfg, cls, mode in lines:
        saved = (args.inputs, engine._DEFER)
        try:
            if mode == "borrowed":
                args.inputs = "borrowed"
            elif mode == "nodefer":
                engine._DEFER = False                     # every batch applied at its spawn
            W = cls(lam, team, args)
            W.setup()
            k.reserve(W.n)
            W.make_sets(input_sets(args, k.reserved, W.ops_per_step) if mode != "nodefer" else 1)
            steps, warm = 10, 3
            for _ in range(warm):
                W.step()
            world.wait_all()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                W.step()
            world.wait_all()
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - t0
            ms = el / steps * 1e3
            desc = W.describe()
            if mode == "borrowed":
                desc += "; plain (borrowed) input tensors: each batch partitioned at its spawn, the shard sweep shared"
            elif mode == "nodefer":
                desc += "; no deferral (LAMELLAR_DEFER=0): each batch partitioned and applied at its spawn, one sweep per batch"
            res[cfg] = {"workload": desc, "ms_per_step": ms, "value": W.ops_per_step * steps / el,
                        "unit": "ops/s", "steps": steps, "warmup": warm, "dtype": W.dtype,
                        "roofline_frac": W.survey_bpo * W.ops_per_step / (ms * 1e-3) / HBM_PEAK,
                        "bytes_per_op": W.survey_bpo, "verified": W.verify(warm + steps)}
            del W
            torch.cuda.empty_cache()
        except Exception as e:  # a failing side line never costs the headline line
            res[cfg] = {"error": f"{type(e).__name__}: {e}"}
        finally:
            args.inputs, engine._DEFER = saved
    return res


def e2e(lam, team, W, args):
    """Records originate in host memory (the lamellae's buffers): PCIe-inclusive rates."""
    dev = W.dev
    idx_h = W.idx.cpu().pin_memory()
    vals_h = W.vals.cpu().pin_memory()
    idx_d, vals_d = torch.empty_like(W.idx), torch.empty_like(W.vals)
    fetch = lam.AtomicArray(team, W.elems * W.npes, lam.Distribution.Block, "u64")
    olds_h = torch.empty(W.n, dtype=torch.int64).pin_memory()
    team.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        idx_d.copy_(idx_h, non_blocking=True)
        vals_d.copy_(vals_h, non_blocking=True)
        W.arr.batch_add(idx_d, vals_d).spawn()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    for _ in range(args.steps):
        idx_d.copy_(idx_h, non_blocking=True)
        vals_d.copy_(vals_h, non_blocking=True)
        h = fetch.batch_fetch_add(idx_d, vals_d).spawn()
        olds_h.copy_(h._res.vals, non_blocking=True)
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    out = {"batch_add_ops_per_s": W.npes * W.n * args.steps / (t1 - t0),
           "batch_fetch_add_ops_per_s": W.npes * W.n * args.steps / (t2 - t1),
           "note": "pinned host idx+vals -> H2D -> device op (-> D2H olds for fetch_add), u64"}
    if W.npes == 1:
        out["wire"] = e2e_wire(lam, team, W, args)
    return out




def e2e_wire(lam, team, W, args):
    """The reference's own op-buffer bytes in host memory: IdxVal<u32,u64> records
    (16 B, repr(C)), applied by lmr_apply_mvmi_host (pieces uploaded / applied /
    results downloaded on three streams); fetch_add olds land in a pinned host array.
    At one PE a global index is the local offset."""
    from lamellar_runtime_amd import _capi
    from lamellar_runtime_amd.types import ArrayOpCmd
    k = team.kernels
    dt = lam.dtype_of("u64")
    iw = 4
    rb, vo = _capi.lib().lmr_record_bytes(iw, dt.code), _capi.lib().lmr_record_val_offset(iw, dt.code)
    assert (rb, vo) == (16, 8)
    # the op buffer and the olds in the library's pinned host heap (lmr_host_alloc: DMA'd in
    # place, as the reference's lamellae heap is mapped once for the world)
    rdt = np.dtype([("i", "<u4"), ("pad", "<u4"), ("v", "<u8")])
    buf = k.host_alloc(W.n * rdt.itemsize)
    olds = k.host_alloc(W.n * 8, np.uint64)
    rec = buf.view(rdt)
    rec["i"] = W.idx.cpu().numpy().astype(np.uint32)
    rec["v"] = W.vals.cpu().numpy().view(np.uint64)
    try:
        shard, slen = W.arr.local_shard(), W.arr.num_elems_local()
        kind = int(W.arr.kind)
        k.apply_mvmi_host(shard, slen, kind, dt, int(ArrayOpCmd.Add), buf, iw)      # warm
        t0 = time.perf_counter()
        for _ in range(args.steps):
            k.apply_mvmi_host(shard, slen, kind, dt, int(ArrayOpCmd.Add), buf, iw)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            k.apply_mvmi_host(shard, slen, kind, dt, int(ArrayOpCmd.FetchAdd), buf, iw, olds)
        t2 = time.perf_counter()
    finally:
        del rec
        k.host_free(buf)
        k.host_free(olds)
    return {"batch_add_ops_per_s": W.n * args.steps / (t1 - t0),
            "batch_fetch_add_ops_per_s": W.n * args.steps / (t2 - t1),
            "h2d_GBps": W.n * rb * args.steps / (t1 - t0) / 1e9,
            "note": "host IdxVal<u32,u64> op buffer (lmr_host_alloc) -> lmr_apply_mvmi_host; olds -> host"}


if __name__ == "__main__":
    main()
