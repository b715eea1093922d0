"""N > 1 exchange orchestration rehearsed on CPU: world_size 2, gloo backend.

The product exchange (engine._distributed: lmr_pack -> header all-to-all ->
all-to-all-v of indices/values -> apply -> reverse all-to-all-v -> result
scatter) runs unchanged; only the device kernels are replaced by the small
CPU test double below (no GPU here). Results are checked against the oracle
simulating both PEs.
"""
import ctypes
import os
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class CpuTestKernels:
    """Test double of DeviceKernels: same interface, numpy loops, a few ops."""

    is_device = False

    def __init__(self, device):
        from lamellar_runtime_amd import _capi
        self.device = torch.device("cpu")
        self.capi = _capi
        self.strategy = 0
        self.err = 0

    def empty(self, n, dt):
        return torch.zeros(max(int(n), 0), dtype=dt)

    def synchronize(self):
        pass

    def reserve(self, n):
        pass

    def errors(self, clear=True):
        e = self.err
        if clear:
            self.err = 0
        return e

    def check_errors(self):
        if self.errors():
            from lamellar_runtime_amd import LamellarError
            raise LamellarError(2, "test double error")

    def pack(self, layout, gidx, n, vals, dt, iw, stable=True, want_pos=True):
        g = gidx.numpy().view(np.uint64)[:n]
        pes, offs = np.zeros(n, np.int64), np.zeros(n, np.uint64)
        for j in range(n):
            pe, off = ctypes.c_uint64(), ctypes.c_uint64()
            assert self.capi.lib().lmr_pe_and_offset(ctypes.byref(layout), int(g[j]), ctypes.byref(pe),
                                                     ctypes.byref(off))
            pes[j], offs[j] = pe.value, off.value
        order = np.argsort(pes, kind="stable")
        it = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[iw]
        out_idx = torch.from_numpy(offs[order].astype(it).view(np.uint8).copy())
        out_vals = None
        if vals is not None:
            v = vals.numpy().view(dt.np)[:n]
            out_vals = torch.from_numpy(v[order].copy().view(np.uint8))
        out_pos = torch.from_numpy(order.astype(np.int32))
        counts = torch.from_numpy(np.bincount(pes, minlength=layout.num_pes).astype(np.int64))
        return out_idx, out_vals, out_pos, counts

    def _apply_one(self, a, i, op, v, cmp):
        old = a[i]
        if op in (0, 1):
            a[i] = old + v
        elif op == 18:
            a[i] = v
        elif op == 21:
            if old == cmp:
                a[i] = v
                return cmp, 1
            return old, 0
        elif op == 17:
            pass
        else:
            raise NotImplementedError(op)
        return old, 1

    def apply_soa(self, shard, shard_len, kind, dt, op, idx, iw, vals, scalar_bits, n, results=None,
                  ok=None, cmp_bits=0, eps_bits=0):
        a = shard.numpy().view(dt.np)
        it = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[iw]
        ii = idx.numpy().view(it)[:n]
        vv = vals.numpy().view(dt.np)[:n] if vals is not None else None
        sv = dt.from_bits(scalar_bits)
        cmp = dt.from_bits(cmp_bits)
        r = results.numpy().view(dt.np) if results is not None else None
        o = ok.numpy() if ok is not None else None
        with np.errstate(over="ignore"):
            for k in range(n):
                if ii[k] >= shard_len:
                    self.err |= 1
                    continue
                old, okk = self._apply_one(a, int(ii[k]), op, vv[k] if vv is not None else sv, cmp)
                if r is not None:
                    r[k] = old
                if o is not None:
                    o[k] = okk

    def stage_begin(self, shard, shard_len, kind, dt, op, cmp_bits=0, eps_bits=0, expect=0):
        self._stage = (shard, shard_len, kind, dt, op, cmp_bits, eps_bits)

    def stage_soa(self, idx, iw, vals, scalar_bits, n, results=None, ok=None):
        shard, shard_len, kind, dt, op, cb, eb = self._stage
        self.apply_soa(shard, shard_len, kind, dt, op, idx, iw, vals, scalar_bits, n, results, ok, cb, eb)

    def stage_finish(self):
        self._stage = None

    def apply_mvsi(self, shard, shard_len, kind, dt, op, vals, n, index, results=None, ok=None,
                   cmp_bits=0, eps_bits=0):
        idx = torch.from_numpy(np.full(n, index, dtype=np.uint64).view(np.uint8))
        self.apply_soa(shard, shard_len, kind, dt, op, idx, 8, vals, 0, n, results, ok, cmp_bits, eps_bits)

    def reduce(self, data, n, dt, op):
        a = data.numpy().view(dt.np)[:n]
        if n == 0:
            return False, 0
        with np.errstate(over="ignore"):
            acc = a[0]
            for x in a[1:]:
                if op == 0:
                    acc = (np.array([acc]) + np.array([x]))[0]
                elif op == 1:
                    acc = (np.array([acc]) * np.array([x]))[0]
                elif op == 2:
                    acc = acc if acc > x else x
                else:
                    acc = acc if acc < x else x
        u = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[dt.bytes]
        return True, int(np.array([acc], dtype=dt.np).view(u)[0])

    def scatter_results(self, res_in, pos, n, eb, res_out, ok_in=None, ok_out=None):
        u = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[eb]
        p = pos.numpy().view(np.int32)[:n]
        res_out.numpy().view(u)[p] = res_in.numpy().view(u)[:n]
        if ok_in is not None and ok_out is not None:
            ok_out.numpy()[p] = ok_in.numpy()[:n]


def _worker(rank, ws, port, outdir, dist_kind, chunk=None, ragged=False):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    if chunk:
        os.environ["LAMELLAR_EXCHANGE_CHUNK"] = str(chunk)
    from _lamellar_bootstrap import load_package
    lam = load_package()
    from test_dist_gloo import CpuTestKernels
    world = lam.LamellarWorldBuilder().with_kernels(CpuTestKernels).build()
    me = world.my_pe()
    rng = np.random.default_rng(100 + me)
    n_len = 1003
    arr = lam.AtomicArray(world.team(), n_len, dist_kind, "u64")
    res = {}
    # MVMI add with collisions
    nrec = 3000 if (me == 0 or not ragged) else 1234      # ragged: PEs with different chunk counts
    gi = rng.integers(0, n_len, nrec).astype(np.uint64)
    gv = rng.integers(0, 2**40, nrec).astype(np.uint64)
    arr.batch_add(gi, gv).block()
    world.barrier()
    res["after_add"] = arr.to_numpy()
    res["red"] = np.array([arr.sum().block(), arr.max().block(), arr.min().block(), arr.prod().block()],
                          dtype=np.uint64)
    # SVMI fetch_add (single value) -> olds come back in input order
    fi = rng.permutation(n_len)[:500].astype(np.uint64)
    olds = arr.batch_fetch_add(fi, 7).block()
    world.barrier()
    res["fetch_idx"], res["fetch_olds"] = fi, olds.numpy().view(np.uint64)
    res["after_fetch"] = arr.to_numpy()
    # MVSI: many values at one index
    arr.batch_add(5, np.arange(1, 11, dtype=np.uint64)).block()
    world.barrier()
    res["after_mvsi"] = arr.to_numpy()
    if ragged:
        # mixed shapes in one collective call: PE 0 MVSI, PE 1 MVMI
        if me == 0:
            arr.batch_add(7, np.arange(1, 5, dtype=np.uint64)).block()
        else:
            arr.batch_add(np.array([1, 2, 3], dtype=np.uint64), np.array([100, 200, 300], dtype=np.uint64)).block()
        world.barrier()
        res["after_mixed"] = arr.to_numpy()
    # compare_exchange on PE-owned indices: all succeed
    ci = np.arange(me, n_len, ws, dtype=np.uint64)
    cur = res["after_mvsi"][ci]
    r = arr.batch_compare_exchange(ci, 0, 1).block()  # current 0: only zero elements succeed
    vals, ok = r.numpy()
    res["cas_idx"], res["cas_vals"], res["cas_ok"], res["cas_cur"] = ci, vals, ok, cur
    world.barrier()
    res["gi"], res["gv"] = gi, gv
    np.savez(os.path.join(outdir, f"pe{rank}.npz"), **res)
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("dist_kind,chunk,ragged", [(0, None, False), (1, None, False), (0, 700, True),
                                                     (1, 256, True)],
                         ids=["Block", "Cyclic", "Block-chunked-ragged", "Cyclic-chunked-ragged"])
def test_two_pe_exchange_gloo(orc, dist_kind, chunk, ragged):
    """chunk: LAMELLAR_EXCHANGE_CHUNK (several pipelined chunks per batch); ragged:
    PEs with different batch lengths (different chunk counts) and a call where one
    PE passes an MVSI shape and the other an MVMI one."""
    ws = 2
    port = 29600 + dist_kind * 7 + (13 if ragged else 0) + (os.getpid() % 200)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(ws, port, d, dist_kind, chunk, ragged), nprocs=ws, join=True)
        pe = [dict(np.load(os.path.join(d, f"pe{r}.npz"))) for r in range(ws)]
    # oracle: both PEs' batch_add applied (order-independent wrapping add)
    from simworld import SimArray
    a = SimArray(orc, ws, 1003, dist_kind, "u64")
    for r in range(ws):
        assert a.op(0, pe[r]["gi"], pe[r]["gv"])[0] == 0
    exp = a.to_numpy()
    for r in range(ws):
        assert np.array_equal(pe[r]["after_add"], exp)
    with np.errstate(over="ignore"):
        prod = np.uint64(1)
        for x in exp:
            prod = prod * x
    for r in range(ws):     # wrapping sum / product, max, min of the whole array on every PE
        assert list(pe[r]["red"]) == [exp.sum(dtype=np.uint64), exp.max(), exp.min(), prod]
    # fetch_add of 7: final = exp + 7 * (#PEs that touched the index); olds linearizable
    cnt = np.zeros(1003, np.uint64)
    for r in range(ws):
        cnt[pe[r]["fetch_idx"].astype(np.int64)] += np.uint64(1)
    exp2 = exp + cnt * np.uint64(7)
    assert np.array_equal(pe[0]["after_fetch"], exp2)
    for r in range(ws):
        fi, olds = pe[r]["fetch_idx"].astype(np.int64), pe[r]["fetch_olds"]
        other = pe[1 - r]["fetch_idx"].astype(np.int64)
        both = np.isin(fi, other)
        assert np.all(olds[~both] == exp[fi[~both]])
        assert np.all((olds[both] == exp[fi[both]]) | (olds[both] == exp[fi[both]] + np.uint64(7)))
    # MVSI: both PEs add 1..10 at index 5
    exp3 = exp2.copy()
    exp3[5] += np.uint64(2 * 55)
    assert np.array_equal(pe[1]["after_mvsi"], exp3)
    # compare_exchange(current=0): ok exactly where the element was 0
    if ragged:
        exp4 = exp3.copy()
        exp4[7] += np.uint64(10)
        exp4[[1, 2, 3]] += np.array([100, 200, 300], dtype=np.uint64)
        for r in range(ws):
            assert np.array_equal(pe[r]["after_mixed"], exp4)
    for r in range(ws):
        assert np.array_equal(pe[r]["cas_ok"].astype(bool), pe[r]["cas_cur"] == 0)
