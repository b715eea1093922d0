#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes per kernel and per bench stage.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of
a wide coalesced stream -> doubled here; WRITE_SIZE is taken as reported.
Stage bytes are per stage invocation: the bytes of all the stage's kernels divided
by the launch count of the stage's anchor kernel (one launch per invocation).
usage: tools/pmc_summary.py <prof dir with pmc_fetch/ and pmc_write/> [out.json [records per invocation | bench log]]
With the records each stage invocation processed in the profiled run (e.g. 2^28 for a C3 session of
four 2^26-record batches), the json also holds "_per_record": bytes per record per stage, which
bench.py scales by its own records per launch (a session's batch count depends on the run).
Given instead the profiled bench command's log (its JSON line), each stage's records come from
the line: records per step x the steps the command ran, so sessions of mixed sizes are fine.
"""
import collections
import csv
import json
import os
import sys

# stage -> (anchor kernels: their launches summed count invocations; kernels whose bytes belong
# to the stage). Staged sessions: one bin_scatter / fine_scatter invocation per region, one
# tile_apply / unpartition invocation per tile sweep.
STAGES = {
    "bin_count": (("k_bin_count", "k_ccount", "k_ccount_stage", "k_wcount_stage"),
                  ("k_bin_count", "k_ccount", "k_ccount_stage", "k_wcount_stage", "k_wide_starts")),
    "bin_scatter": (("k_coarse_free", "k_coarse_scatter", "k_bin_scatter", "k_coarse_stage", "k_coarse_free_stage",
                     "k_wide_stage"),
                    ("k_coarse_free", "k_coarse_scatter", "k_coarse_offsets", "k_bin_scatter", "k_coarse_stage",
                     "k_coarse_free_stage", "k_wide_stage")),
    "fine_scatter": (("k_fine_free", "k_fine_scatter", "k_fine_piece", "k_fine_stage", "k_fine_bucket"),
                     ("k_fine_free", "k_fine_scatter", "k_fine_piece", "k_piece_count", "k_free_tile_totals",
                      "k_fine_stage", "k_fine_bucket")),
    "tile_apply": (("k_tile_owner",), ("k_tile_owner", "k_tile_delta", "k_tile_plan", "k_stage_plan", "k_bucket_plan")),
    "unpartition": (("k_tile_owner",), ("k_unpartition", "k_unpartition_multi", "k_unpart_rounds",
                                        "k_unpart_crounds", "k_unpart_wide")),
    "direct": (("k_apply_direct",), ("k_apply_direct",)),
    "pack": (("k_pack_count", "k_pack_stage", "k_pack_bucket"),
             ("k_pack_count", "k_pack_scatter", "k_pack_stage", "k_dest_offsets", "k_fill_counts", "k_pack_bucket",
              "k_bucket_hdr")),
    "scatter_results": (("k_scatter_results",), ("k_scatter_results",)),
}


def base_name(k):
    k = k.replace("(anonymous namespace)::", "")
    k = k.split("(")[0].split("<")[0]
    return k.replace("void ", "").replace("lmr::", "").strip()


def per_kernel(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)   # KB -> B
    return agg


def main():
    d = sys.argv[1]
    f = per_kernel(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"))
    w = per_kernel(os.path.join(d, "pmc_write", "run_counter_collection.csv"))
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for k in sorted(set(f) | set(w)):
        fb, wb = 2.0 * sum(f.get(k, [])), sum(w.get(k, []))
        n = max(len(f.get(k, [])), len(w.get(k, [])), 1)
        print(f"{k[:70]:70s} x{n:4d}  read {fb / n / 1e6:10.1f} MB  write {wb / n / 1e6:10.1f} MB  per launch")
        b = base_name(k)
        tot[b] += fb + wb
        cnt[b] += n
    out = {}
    for st, (anchors, ks) in STAGES.items():
        inv = sum(cnt.get(a, 0) for a in anchors)
        if st == "pack" and cnt.get("k_pack_count") and cnt.get("k_pack_stage"):
            inv = cnt["k_pack_count"]                      # counted pack: both kernels per invocation
        if inv:
            out[st] = sum(tot.get(x, 0.0) for x in ks) / inv
            print(f"stage {st:16s} {out[st] / 1e6:10.1f} MB per invocation")
    # the exchange's transport kernels (RCCL's copies) per pack invocation (one per chunk)
    rccl = sum(v for k, v in tot.items() if k.startswith("rccl") or k.startswith("ncclDevKernel"))
    if rccl and out.get("pack"):
        inv = sum(cnt.get(a, 0) for a in STAGES["pack"][0])
        if cnt.get("k_pack_count") and cnt.get("k_pack_stage"):
            inv = cnt["k_pack_count"]
        out["_transport_per_pack"] = rccl / inv
        print(f"transport (RCCL kernels)  {out['_transport_per_pack'] / 1e6:10.1f} MB per pack invocation")
    if len(sys.argv) > 3 and not sys.argv[3][0].isdigit():
        # the profiled bench command's own JSON line: its stage records per step (records per
        # launch x launches per step) x every step the command ran (warmup, timed, profiled) are
        # the records each stage processed, whatever the session sizes were
        line = next(json.loads(x) for x in open(sys.argv[3]) if x.startswith('{"metric'))
        steps = line["warmup"] + line["steps"] + line["apply_pipeline"]["profiled_steps"]
        rps = {st: r["records_per_launch"] * r["launches_per_step"] for st, r in line["apply_pipeline"]["stages"].items()}
        out["_per_record"] = {}
        for st, (anchors, _) in STAGES.items():
            inv = sum(cnt.get(a, 0) for a in anchors)
            if st == "pack" and cnt.get("k_pack_count") and cnt.get("k_pack_stage"):
                inv = cnt["k_pack_count"]
            if st in out and rps.get(st):
                out["_per_record"][st] = out[st] * inv / (steps * rps[st])
        for st, v in out["_per_record"].items():
            print(f"stage {st:16s} {v:10.2f} B per record")
        if "_transport_per_pack" in out and rps.get("pack"):
            inv = sum(cnt.get(a, 0) for a in STAGES["pack"][0])
            if cnt.get("k_pack_count") and cnt.get("k_pack_stage"):
                inv = cnt["k_pack_count"]
            out["_transport_per_record"] = out["_transport_per_pack"] * inv / (steps * rps["pack"])
            print(f"transport (RCCL kernels)  {out['_transport_per_record']:10.2f} B per record packed")
    elif len(sys.argv) > 3:
        recs = float(sys.argv[3])
        out["_per_record"] = {st: v / recs for st, v in out.items() if not st.startswith("_")}
        for st, v in out["_per_record"].items():
            print(f"stage {st:16s} {v:10.2f} B per record")
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
