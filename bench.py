#!/usr/bin/env python3
"""Benchmark of the MI355X batched element-op path (BASELINE.json metric:
"batched array ops applied/sec (device-resident), 1/2/4/8 MI355X").

A step = one `AtomicArray<u64>::batch_add(indices, vals)` over one batch of
synthetic device-resident input, every PE (one per GPU) issuing its own batch:
  N = 1 : C2 — 2^28 u64 add records, uniform-random global indices into a
          2^26-element array (the local lamellae: no pack, no exchange);
  N > 1 : C4 — the same batch per PE (weak scaling), indices uniform over the
          whole N * 2^26-element Block array: device pack by destination PE ->
          RCCL all-to-all(v) over xGMI -> device apply on every shard.
value = ops applied by all PEs / max-over-PEs wall time of the timed steps.

roofline: the dominant kernel's algorithmic HBM bytes per launch / its average
launch time (HIP events recorded by the library on the launch stream), against
the 8.0 TB/s HBM3E peak. cpu_baseline: the reference-structured threaded CPU
apply (oracle/cpu_baseline.c, a restatement of the Rust path: the reference
itself cannot be built here) on a bounded sample, rank 0, N = 1.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
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
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--records-log2", type=int, default=28)
    p.add_argument("--elems-log2", type=int, default=26)
    p.add_argument("--strategy", default=os.environ.get("LAMELLAR_OP_STRATEGY", "auto"))
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--cpu-sample-log2", type=int, default=24)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--e2e", action="store_true",
                   help="also time the host-buffer path: pinned host records -> H2D copy -> apply")
    return p.parse_args()


def stage_bytes_per_op(stage, iw, vb, eb, n, shard_len, fetch, two_level=True):
    """Algorithmic HBM bytes per op of each kernel stage."""
    pos = 4 if fetch else 0
    res = eb if fetch else 0
    if stage == "direct":
        return iw + vb + 2 * eb + res
    if stage == "bin_count":
        return iw
    if stage == "bin_scatter":      # coarse pass (two-level) or one-level scatter
        return iw + vb + (4 + vb + pos if two_level else 2 + vb + pos)
    if stage == "tile_apply":
        return 2 + vb + pos + res + 2.0 * eb * shard_len / max(n, 1)
    if stage == "pack":
        return 8 + 8 + vb + iw + vb + 4
    if stage == "fine_scatter":
        return 4 + vb + pos + 2 + vb + pos
    if stage == "scatter_results":
        return 4 + 2 * eb
    return 0.0


def cpu_baseline(args, elems_log2):
    """Reference-structured CPU apply on a bounded sample (C2 shape, same shard size)."""
    from oracle import oracle as orc
    n = 1 << args.cpu_sample_log2
    shard_len = 1 << elems_log2
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    rng = np.random.default_rng(0x1A3E11A2)
    gidx = rng.integers(0, shard_len, n, dtype=np.uint64)
    vals = rng.integers(0, 2**63, n, dtype=np.uint64)
    shard = np.zeros(shard_len, dtype=np.uint64)
    orc.cpu_baseline(3, np.uint64, 0, shard, gidx[:1 << 16], vals[:1 << 16], threads)  # warm
    best = None
    for _ in range(2):
        st, t, _ = orc.cpu_baseline(3, np.uint64, 0, shard, gidx, vals, threads)
        assert st == 0
        if best is None or t.total_s < best.total_s:
            best = t
    return {
        "value": n / best.total_s,
        "unit": "ops/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"2^{args.cpu_sample_log2} u64 add records, uniform over a 2^{elems_log2}-element "
                   f"shard, packed into 100 kB op buffers by {max(1, threads // 4)} threads and "
                   f"applied with SeqCst atomics by {threads} threads (best of 2; pack "
                   f"{best.pack_s * 1e3:.0f} ms + apply {best.apply_s * 1e3:.0f} ms)"),
    }


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
    n = 1 << args.records_log2
    elems_per_pe = 1 << args.elems_log2
    global_len = elems_per_pe * npes
    arr = lam.AtomicArray(team, global_len, lam.Distribution.Block, "u64")
    g = torch.Generator(device=dev)
    g.manual_seed(0x1A3E11A2 + me)
    idx = torch.randint(0, global_len, (n,), dtype=torch.int64, device=dev, generator=g)
    vals = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device=dev, generator=g)
    k.reserve(n)
    world.barrier()

    for _ in range(args.warmup):
        arr.batch_add(idx, vals).spawn()
    world.wait_all()
    k.profile(True)
    k.profile_read(reset=True)
    world.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        arr.batch_add(idx, vals).spawn()
    torch.cuda.synchronize(dev)
    world.barrier()
    t1 = time.perf_counter()
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
    value = npes * n * args.steps / elapsed

    verified = None
    if not args.no_verify:
        # wrapping-sum invariant: sum(array) == (W + K) * sum(vals) over all PEs (mod 2^64)
        s_arr = arr.local_data().sum(dtype=torch.int64)
        s_val = vals.sum(dtype=torch.int64) * (args.warmup + args.steps)
        if npes > 1:
            import torch.distributed as dist
            dist.all_reduce(s_arr)
            dist.all_reduce(s_val)
        verified = bool(int(s_arr.item()) == int(s_val.item()))

    # ---- roofline of the dominant kernel ----
    iw = 8 if npes == 1 else arr.index_size()
    recv_n = n  # uniform indices: each PE receives ~n records
    per = {}
    for name, (ms, cnt) in stages.items():
        if cnt:
            per[name] = (ms / cnt, cnt / args.steps)
    dom = max(per, key=lambda s: per[s][0] * per[s][1]) if per else None
    roof = None
    if dom:
        avg_ms, launches_per_step = per[dom]
        ops_per_launch = recv_n / launches_per_step if dom != "scan" else recv_n
        bpo = stage_bytes_per_op(dom, iw, 8, 8, ops_per_launch, elems_per_pe, False)
        achieved = bpo * ops_per_launch / (avg_ms * 1e-3)
        roof = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": achieved / HBM_PEAK, "traffic": None, "kernel": dom,
                "bytes_per_op": bpo, "avg_launch_ms": avg_ms}
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            try:
                tr = json.load(open(pmc)).get(dom)
                if tr:
                    roof["traffic"] = tr
            except Exception:
                pass
    apply_stages = [s for s in ("direct", "bin_count", "scan", "bin_scatter", "fine_scatter", "tile_apply")
                    if s in per]
    apply_ms = sum(per[s][0] * per[s][1] for s in apply_stages)
    survey_bpo = 4 + 8 + 16          # SURVEY.md §8(d) C2 B_op (u32 index, u64 value, element RMW)

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
        "dtype": "u64",
        "data": "synthetic (seeded uniform-random u64 indices and values, device-resident)",
        "config": {
            "workload": ("C2: 2^%d batched u64 add records, uniform-random indices into a 2^%d-element "
                         "AtomicArray<u64>" % (args.records_log2, args.elems_log2)) if npes == 1 else
                        ("C4: %d PEs all-to-all batched u64 add, 2^%d records per PE, Block array of "
                         "%d x 2^%d elements, op buffers via RCCL all-to-all(v) over xGMI"
                         % (npes, args.records_log2, npes, args.elems_log2)),
            "records_per_pe": n,
            "elems_per_pe": elems_per_pe,
            "op": "batch_add (ArrayOpCmd::Add, MVMI)",
            "strategy": args.strategy,
            "parallelism": f"{npes} PE(s), one per GPU",
        },
        "roofline": roof,
        "apply_pipeline": {"stages_ms_per_step": {s: per[s][0] * per[s][1] for s in per},
                           "apply_ms_per_step": apply_ms,
                           "survey_bytes_per_op": survey_bpo,
                           "survey_frac": (survey_bpo * n / (apply_ms * 1e-3) / HBM_PEAK) if apply_ms else None},
        "verified": verified,
        "cpu_baseline": None,
    }
    if args.e2e:
        # records originate in host memory (the lamellae's buffers): PCIe-inclusive rate
        idx_h = idx.cpu().pin_memory()
        vals_h = vals.cpu().pin_memory()
        idx_d, vals_d = torch.empty_like(idx), torch.empty_like(vals)
        fetch = lam.AtomicArray(team, global_len, lam.Distribution.Block, "u64")
        olds_h = torch.empty(n, dtype=torch.int64).pin_memory()
        world.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            idx_d.copy_(idx_h, non_blocking=True)
            vals_d.copy_(vals_h, non_blocking=True)
            arr.batch_add(idx_d, vals_d).spawn()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            idx_d.copy_(idx_h, non_blocking=True)
            vals_d.copy_(vals_h, non_blocking=True)
            h = fetch.batch_fetch_add(idx_d, vals_d)
            olds_h.copy_(h.spawn()._res.vals, non_blocking=True)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        out["e2e"] = {"batch_add_ops_per_s": npes * n * args.steps / (t1 - t0),
                      "batch_fetch_add_ops_per_s": npes * n * args.steps / (t2 - t1),
                      "note": "pinned host idx+vals -> H2D -> device op (-> D2H olds for fetch_add)"}
    if me == 0 and npes == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, args.elems_log2)
    if me == 0:
        print(json.dumps(out), flush=True)
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
