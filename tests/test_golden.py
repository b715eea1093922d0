"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces every committed vector (regression pin).
GPU: the device reproduces them through the C ABI with no oracle at run time —
bit-exact state and results for the conflict-free batches, bit-exact final
state for the colliding order-independent integer batches.
"""
import os

import numpy as np
import pytest

from opgen import CODE, DTYPE_NAMES, IS_FLOAT, NP, bits_equal, ret_kind

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(dt):
    return dict(np.load(os.path.join(HERE, f"golden_{dt}.npz")))


def cases(g, prefix):
    ops = sorted({int(k[len(prefix):].split("_")[0]) for k in g if k.startswith(prefix)})
    return ops


def kind_for(dt):
    return 2 if IS_FLOAT[dt] else 1


@pytest.mark.parametrize("dt", DTYPE_NAMES)
def test_oracle_reproduces_golden(orc, dt):
    g = load(dt)
    for op in cases(g, "op"):
        p = f"op{op}_"
        s = g[p + "shard0"].copy()
        L = orc.layout_new(s.size, 1, 0, 0)
        cur = g[p + "cur"][0] if op in (21, 22) else None
        eps = g[p + "eps"][0] if op in (21, 22) else None
        st, res, ok = orc.batch_op(L, [s], kind_for(dt), CODE[dt], NP[dt], op, g[p + "idx"], g[p + "vals"], cur, eps)
        assert st == 0 and bits_equal(s, g[p + "final"]), (dt, op)
        if ret_kind(op):
            assert bits_equal(res, g[p + "results"]), (dt, op)
        if ret_kind(op) == 2:
            assert np.array_equal(ok, g[p + "ok"])
    for op in cases(g, "coll"):
        p = f"coll{op}_"
        s = g[p + "shard0"].copy()
        L = orc.layout_new(s.size, 1, 0, 0)
        assert orc.batch_op(L, [s], 1, CODE[dt], NP[dt], op, g[p + "idx"], g[p + "vals"])[0] == 0
        assert bits_equal(s, g[p + "final"])


def test_layout_tables_reproduce(orc, capi, lam):
    import ctypes
    from lamellar_runtime_amd import _capi
    g = dict(np.load(os.path.join(HERE, "golden_layouts.npz")))
    for key in sorted({k.rsplit("_", 1)[0] for k in g if k.endswith("_map")}):
        L = _capi.lmr_layout_t(*[int(x) for x in g[key + "_layout"]])
        for p in range(3):
            assert capi.lmr_num_elems_pe(ctypes.byref(L), p) == g[key + "_num_elems"][p]
            assert capi.lmr_local_slice_start(ctypes.byref(L), p) == g[key + "_slice_start"][p]
        assert capi.lmr_index_size(ctypes.byref(L)) == g[key + "_index_size"][0]
        for i, (pe, off) in enumerate(g[key + "_map"]):
            a, b = ctypes.c_uint64(), ctypes.c_uint64()
            okd = capi.lmr_pe_and_offset(ctypes.byref(L), i, ctypes.byref(a), ctypes.byref(b))
            assert (a.value, b.value) == (pe, off) if okd else pe == 2**64 - 1


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", [1, 2], ids=["direct", "tiled"])
@pytest.mark.parametrize("dt", DTYPE_NAMES)
def test_device_reproduces_golden(world, lam, dt, strategy):
    import torch
    k = world.team().kernels
    k.reserve(1 << 16)
    old = k.strategy
    k.strategy = strategy
    dto = lam.dtype_of(dt)
    eb = dto.bytes

    def dev(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()
    try:
        g = load(dt)
        for op in cases(g, "op"):
            p = f"op{op}_"
            n = g[p + "idx"].size
            shard = dev(g[p + "shard0"])
            res = torch.zeros(n * eb, dtype=torch.uint8, device="cuda")
            ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
            rk = ret_kind(op)
            cb = dto.to_bits(g[p + "cur"][0]) if op in (21, 22) else 0
            ebits = dto.to_bits(g[p + "eps"][0]) if op in (21, 22) else 0
            k.apply_soa(shard, g[p + "shard0"].size, kind_for(dt), dto, op, dev(g[p + "idx"]), 8,
                        dev(g[p + "vals"]), 0, n, res if rk else None, ok if rk == 2 else None, cb, ebits)
            k.synchronize()
            assert k.errors() == 0
            assert bits_equal(shard.cpu().numpy().view(NP[dt]), g[p + "final"]), (dt, op)
            if rk:
                assert bits_equal(res.cpu().numpy().view(NP[dt]), g[p + "results"]), (dt, op)
            if rk == 2:
                assert np.array_equal(ok.cpu().numpy(), g[p + "ok"]), (dt, op)
        for op in cases(g, "coll"):
            p = f"coll{op}_"
            shard = dev(g[p + "shard0"])
            k.apply_soa(shard, g[p + "shard0"].size, 1, dto, op, dev(g[p + "idx"]), 8, dev(g[p + "vals"]),
                        0, g[p + "idx"].size)
            k.synchronize()
            assert bits_equal(shard.cpu().numpy().view(NP[dt]), g[p + "final"]), (dt, op)
    finally:
        k.strategy = old
