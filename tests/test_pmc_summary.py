"""tools/pmc_summary.py: per-stage bytes from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (FETCH
doubled, KB -> B), per invocation and per record — from a fixed record count, or from the
profiled bench command's own JSON line (records per step x the steps the command ran)."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "pmc_summary.py")


def _counters(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Value"])
        w.writeheader()
        for name, kb in rows:
            w.writerow({"Kernel_Name": name, "Counter_Value": kb})


def _run(d, *extra):
    out = os.path.join(d, "out.json")
    subprocess.run([sys.executable, TOOL, d, out, *extra], check=True, stdout=subprocess.DEVNULL)
    return json.load(open(out))


def test_per_invocation_and_fixed_records(tmp_path):
    d = str(tmp_path)
    # two coarse launches (one invocation each), one fine launch; KB values
    _counters(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"),
              [("void lmr::k_coarse_free_stage<8>(...)", 100), ("void lmr::k_coarse_free_stage<8>(...)", 300),
               ("k_fine_free", 50)])
    _counters(os.path.join(d, "pmc_write", "run_counter_collection.csv"),
              [("void lmr::k_coarse_free_stage<8>(...)", 40), ("void lmr::k_coarse_free_stage<8>(...)", 60),
               ("k_fine_free", 25)])
    j = _run(d, "1024")
    kb = 1024.0
    assert j["bin_scatter"] == (2 * 400 + 100) * kb / 2          # FETCH x2 + WRITE, per invocation
    assert j["fine_scatter"] == (2 * 50 + 25) * kb / 1            # one k_fine_free invocation (anchor)
    assert j["_per_record"]["bin_scatter"] == j["bin_scatter"] / 1024


def test_per_record_from_the_bench_line(tmp_path):
    d = str(tmp_path)
    _counters(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"),
              [("k_coarse_free_stage", 10), ("k_coarse_free_stage", 30), ("k_coarse_free_stage", 20)])
    _counters(os.path.join(d, "pmc_write", "run_counter_collection.csv"),
              [("k_coarse_free_stage", 5), ("k_coarse_free_stage", 5), ("k_coarse_free_stage", 5)])
    line = {"metric": "m", "warmup": 2, "steps": 5,
            "apply_pipeline": {"profiled_steps": 5,
                               "stages": {"bin_scatter": {"records_per_launch": 3000.0, "launches_per_step": 0.5}}}}
    log = os.path.join(d, "bench.log")
    with open(log, "w") as f:
        f.write("noise\n" + json.dumps(line) + "\n")
    j = _run(d, log)
    total = (2 * 60 + 15) * 1024.0                                # every launch's bytes
    assert abs(j["_per_record"]["bin_scatter"] - total / (12 * 1500.0)) < 1e-9
