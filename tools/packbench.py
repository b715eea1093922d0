#!/usr/bin/env python3
"""Sender-side pack microbenchmark (lmr_pack_unordered) on one GPU: 2^26 records,
u64 values, uniform global indices into an npes x 2^26-element Block array, for
several PE counts -- the per-chunk pack of the C4 exchange without the exchange.
usage (GPU box): python tools/packbench.py [--log2 26] [--reps 10]"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from _lamellar_bootstrap import load_package  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2", type=int, default=26)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    lam = load_package()
    from lamellar_runtime_amd import _capi
    world = lam.LamellarWorldBuilder().build()
    k = world.team().kernels
    n = 1 << a.log2
    dt = lam.dtype_of("u64")
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    # npes = 512 over 2^29 elements: the key count of a pack by (destination PE, coarse
    # bucket) for 8 PEs x 64 coarse buckets of 2^20 u64 elements each
    for npes, elems in ((1, 1 << 26), (2, 2 << 26), (8, 8 << 26), (64, 8 << 26), (512, 8 << 26)):
        L = _capi.lmr_layout_t()
        _capi.lib().lmr_layout_new(ctypes.byref(L), elems, npes, 0, 0)
        iw = _capi.lib().lmr_index_size(ctypes.byref(L))
        gidx = torch.randint(0, elems, (n,), dtype=torch.int64, device="cuda", generator=g)
        vals = torch.randint(0, 1 << 62, (n,), dtype=torch.int64, device="cuda", generator=g)
        cap = (n + npes - 1) // npes
        cap += cap // 8 + 4096
        for _ in range(2):
            k.pack_regions(L, gidx, n, vals, dt, iw, cap)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            k.pack_regions(L, gidx, n, vals, dt, iw, cap)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        b = n * (8 + 8 + iw + 8)
        print(f"npes {npes} iw {iw} count-free: {ms:.3f} ms per 2^{a.log2}-record pack, "
              f"{b / ms / 1e9:.2f} TB/s on {b / n:.0f} B/record (read 16 + write)", flush=True)
        for want_pos in (False, True):
            for _ in range(2):
                k.pack(L, gidx, n, vals, dt, iw, stable=False, want_pos=want_pos)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                k.pack(L, gidx, n, vals, dt, iw, stable=False, want_pos=want_pos)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.reps * 1e3
            b = n * (8 + 8 + 8 + iw + 8 + (4 if want_pos else 0))
            print(f"npes {npes} iw {iw} pos {int(want_pos)}: {ms:.3f} ms per 2^{a.log2}-record pack, "
                  f"{b / ms / 1e9:.2f} TB/s on {b / n:.0f} B/record (count 8 + read 16 + write)", flush=True)


if __name__ == "__main__":
    main()
