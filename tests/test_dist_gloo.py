"""N > 1 on CPU: world_size 2, gloo backend.

The product exchange is one C-ABI call (lmr_batch_exchange, device code). Here,
without a GPU, the parts of it that are host code run for real:
* the host-buffer transport (world.HostTransport) called through the
  lmr_transport_t function pointers exactly as the library calls them, over a
  2-rank gloo group, with ragged splits and every element unit;
* lmr_exchange_plan, the library's per-chunk host planning;
* the array API over 2 PEs (team transport selection, reductions, to_numpy)
  with a CPU test double of DeviceKernels whose batch_exchange is a one-chunk
  restatement of lmr_batch_exchange built on those two. Results are checked
  against the oracle simulating both PEs.
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

    def batch_exchange(self, transport, layout, shard, shard_len, kind, dt, op, gidx, h_index, i_len, vals,
                       h_val_bits, v_len, results=None, ok=None, cmp_bits=0, eps_bits=0, expect=0):
        """One-chunk restatement of lmr_batch_exchange over the real transport
        callbacks and the real lmr_exchange_plan."""
        lib = self.capi.lib()
        npes = layout.num_pes
        iw, eb = lib.lmr_index_size(ctypes.byref(layout)), dt.bytes
        n = 0 if (i_len == 0 or v_len == 0) else max(i_len, v_len)
        mvsi, scalar = i_len == 1 and v_len > 1, v_len == 1 and not (i_len == 1 and v_len > 1)
        t = transport.t
        hdr = np.zeros((npes, _capi_mod().XHDR_WORDS), np.int64)
        hdr[:, 1], hdr[:, 4] = -1, 1
        pos = None
        if mvsi:
            pe, off = ctypes.c_uint64(), ctypes.c_uint64()
            assert lib.lmr_pe_and_offset(ctypes.byref(layout), int(h_index), ctypes.byref(pe), ctypes.byref(off))
            hdr[pe.value, 0], hdr[pe.value, 1] = n, off.value
            s_idx, s_vals = np.zeros(8, np.uint8), vals.numpy().view(np.uint8).copy()
        else:
            g = gidx if i_len != 1 else torch.tensor([int(h_index)], dtype=torch.int64)
            si, sv, pos, counts = self.pack(layout, g, n, None if scalar else vals, dt, iw)
            hdr[:, 0] = counts.numpy()
            s_idx = np.concatenate([si.numpy(), np.zeros(8, np.uint8)])
            s_vals = np.concatenate([sv.numpy() if sv is not None else np.zeros(0, np.uint8), np.zeros(8, np.uint8)])
        if scalar:
            hdr[:, 2], hdr[:, 3] = 1, np.array([h_val_bits], np.uint64).view(np.int64)[0]
        rh = np.zeros_like(hdr)
        assert t.alltoall(t.self, hdr.ctypes.data, rh.ctypes.data, 8 * hdr.shape[1], None) == 0
        plan = [np.zeros(npes, np.uint64) for _ in range(8)]
        assert lib.lmr_exchange_plan(npes, iw, eb, hdr.ctypes.data, rh.ctypes.data, *[a.ctypes.data for a in plan]) == 1
        isb, iso, irb, iro, vsb, vso, vrb, vro = plan
        u64p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        r_idx = np.zeros(int(irb.sum()) + 8, np.uint8)
        r_vals = np.zeros(int(vrb.sum()) + 8, np.uint8)
        st = t.alltoallv(t.self, s_idx.ctypes.data, u64p(isb), u64p(iso), r_idx.ctypes.data, u64p(irb), u64p(iro),
                         iw, None)
        transport.raise_pending()
        assert st == 0
        assert t.alltoallv(t.self, s_vals.ctypes.data, u64p(vsb), u64p(vso), r_vals.ctypes.data, u64p(vrb),
                           u64p(vro), eb, None) == 0
        rcnt = np.maximum(rh[:, 0], 0)
        tot = int(rcnt.sum())
        r_res = torch.zeros(tot * eb, dtype=torch.uint8)
        r_ok = torch.zeros(tot, dtype=torch.uint8)
        io = vo = ro = 0
        for p in range(npes):
            c = int(rcnt[p])
            if c == 0:
                continue
            res_seg, ok_seg = r_res[ro * eb:(ro + c) * eb], r_ok[ro:ro + c]
            if rh[p, 1] >= 0:
                self.apply_mvsi(shard, shard_len, kind, dt, op, torch.from_numpy(r_vals[vo:vo + c * eb].copy()), c,
                                int(rh[p, 1]), res_seg, ok_seg, cmp_bits, eps_bits)
                vo += c * eb
            else:
                ii = torch.from_numpy(r_idx[io:io + c * iw].copy())
                if rh[p, 2]:
                    self.apply_soa(shard, shard_len, kind, dt, op, ii, iw, None,
                                   int(np.array([rh[p, 3]], np.int64).view(np.uint64)[0]), c, res_seg, ok_seg,
                                   cmp_bits, eps_bits)
                else:
                    self.apply_soa(shard, shard_len, kind, dt, op, ii, iw,
                                   torch.from_numpy(r_vals[vo:vo + c * eb].copy()), 0, c, res_seg, ok_seg,
                                   cmp_bits, eps_bits)
                    vo += c * eb
                io += c * iw
            ro += c
        if results is None and not self.capi.lib().lmr_op_ret_kind(op):
            return
        scnt = np.maximum(hdr[:, 0], 0).astype(np.uint64)
        sb, rb = rcnt.astype(np.uint64) * np.uint64(eb), scnt * np.uint64(eb)
        so, ro_ = np.concatenate([[0], np.cumsum(sb)[:-1]]).astype(np.uint64), \
            np.concatenate([[0], np.cumsum(rb)[:-1]]).astype(np.uint64)
        back = np.zeros(int(rb.sum()) + 8, np.uint8)
        src = np.concatenate([r_res.numpy(), np.zeros(8, np.uint8)])
        assert t.alltoallv(t.self, src.ctypes.data, u64p(sb), u64p(so), back.ctypes.data, u64p(rb), u64p(ro_),
                           eb, None) == 0
        okb = np.zeros(int(scnt.sum()) + 8, np.uint8)
        oks = np.concatenate([r_ok.numpy(), np.zeros(8, np.uint8)])
        sbo, rbo = rcnt.astype(np.uint64), scnt
        assert t.alltoallv(t.self, oks.ctypes.data, u64p(sbo), u64p(so // np.uint64(eb)), okb.ctypes.data,
                           u64p(rbo), u64p(ro_ // np.uint64(eb)), 1, None) == 0
        if n == 0 or results is None:
            return
        nb = torch.from_numpy(back[:n * eb].copy())
        nok = torch.from_numpy(okb[:n].copy())
        if mvsi:
            results.view(torch.uint8)[:n * eb] = nb
            if ok is not None:
                ok[:n] = nok
        else:
            self.scatter_results(nb, pos, n, eb, results, nok if ok is not None else None, ok)

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


def _worker(rank, ws, port, outdir, dist_kind, ragged=False):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
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
        # a fetch op where PE 1's batch is empty: it still takes part in the exchange
        ei = np.array([9, 10, 11], dtype=np.uint64) if me == 0 else np.zeros(0, np.uint64)
        eo = arr.batch_fetch_add(ei, 2).block()
        world.barrier()
        res["empty_olds"], res["after_empty"] = eo.numpy().view(np.uint64), arr.to_numpy()
    # compare_exchange on PE-owned indices: all succeed
    ci = np.arange(me, n_len, ws, dtype=np.uint64)
    cur = arr.to_numpy()[ci]
    r = arr.batch_compare_exchange(ci, 0, 1).block()  # current 0: only zero elements succeed
    vals, ok = r.numpy()
    res["cas_idx"], res["cas_vals"], res["cas_ok"], res["cas_cur"] = ci, vals, ok, cur
    world.barrier()
    res["gi"], res["gv"] = gi, gv
    np.savez(os.path.join(outdir, f"pe{rank}.npz"), **res)
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("dist_kind,ragged", [(0, False), (1, False), (0, True), (1, True)],
                         ids=["Block", "Cyclic", "Block-ragged", "Cyclic-ragged"])
def test_two_pe_exchange_gloo(orc, dist_kind, ragged):
    """ragged: PEs with different batch lengths, an empty batch on one PE, and a
    call where one PE passes an MVSI shape and the other an MVMI one."""
    ws = 2
    port = 29600 + dist_kind * 7 + (13 if ragged else 0) + (os.getpid() % 200)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(ws, port, d, dist_kind, ragged), nprocs=ws, join=True)
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
        assert np.array_equal(pe[0]["empty_olds"], exp4[[9, 10, 11]]) and pe[1]["empty_olds"].size == 0
        exp4[[9, 10, 11]] += np.uint64(2)
        for r in range(ws):
            assert np.array_equal(pe[r]["after_empty"], exp4)
    for r in range(ws):
        assert np.array_equal(pe[r]["cas_ok"].astype(bool), pe[r]["cas_cur"] == 0)


# ---------------------------------------------------------------- lmr_exchange_plan
def _capi_mod():
    from lamellar_runtime_amd import _capi
    return _capi


def _plan(_capi, npes, iw, eb, sh, rh):
    out = [np.zeros(npes, np.uint64) for _ in range(8)]
    sh, rh = np.asarray(sh, np.int64), np.asarray(rh, np.int64)
    pad = ((0, 0), (0, _capi_mod().XHDR_WORDS - sh.shape[1]))       # words past the chunk count: 0
    sh, rh = np.ascontiguousarray(np.pad(sh, pad)), np.ascontiguousarray(np.pad(rh, pad))
    k = _capi.lmr_exchange_plan(npes, iw, eb, sh.ctypes.data, rh.ctypes.data, *[a.ctypes.data for a in out])
    return k, out


def test_exchange_plan_array_values(capi):
    sh = np.array([[3, -1, 0, 0, 2], [0, -1, 0, 0, 2], [5, -1, 0, 0, 2]])
    rh = np.array([[4, -1, 0, 0, 1], [2, -1, 0, 0, 7], [0, -1, 0, 0, 3]])
    k, (isb, iso, irb, iro, vsb, vso, vrb, vro) = _plan(capi, 3, 4, 8, sh, rh)
    assert k == 7                                          # the largest chunk count any PE announced
    assert list(isb) == [12, 0, 20] and list(iso) == [0, 12, 12]
    assert list(irb) == [16, 8, 0] and list(iro) == [0, 16, 24]
    assert list(vsb) == [24, 0, 40] and list(vso) == [0, 24, 24]
    assert list(vrb) == [32, 16, 0] and list(vro) == [0, 32, 48]


def test_exchange_plan_mvsi_and_scalar(capi):
    """MVSI senders send values but no index (it travels in the header); scalar
    senders send indices but no values."""
    sh = np.array([[0, -1, 0, 0, 1], [6, 17, 0, 0, 1]])          # this PE: MVSI block of 6 for PE 1
    rh = np.array([[9, -1, 1, 42, 1], [6, 3, 0, 0, 1]])          # from PE 0: 9 scalar; from PE 1: MVSI
    k, (isb, iso, irb, iro, vsb, vso, vrb, vro) = _plan(capi, 2, 2, 4, sh, rh)
    assert k == 1
    assert list(isb) == [0, 0] and list(vsb) == [0, 24] and list(vso) == [0, 0]
    assert list(irb) == [18, 0] and list(vrb) == [0, 24] and list(vro) == [0, 0]


def test_exchange_plan_empty_and_negative_counts(capi):
    sh = np.zeros((4, 5), np.int64)
    sh[:, 1] = -1
    rh = sh.copy()
    rh[2, 0] = -5                                           # never trusted as a size
    k, out = _plan(capi, 4, 8, 8, sh, rh)
    assert k == 0 and all(int(a.sum()) == 0 for a in out)


# ---------------------------------------------------------------- host transport over gloo
def _transport_worker(rank, ws, port, outdir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from _lamellar_bootstrap import load_package
    lam = load_package()
    from lamellar_runtime_amd.world import HostTransport
    tp = HostTransport(ws, rank, dist.group.WORLD)
    t = tp.t
    assert (t.num_pes, t.my_pe, t.host_buffers) == (ws, rank, 1)
    out = {}
    # all-to-all: 40-byte rows (one exchange header row per PE)
    send = np.arange(ws * 5, dtype=np.int64) + 1000 * rank
    recv = np.zeros_like(send)
    assert t.alltoall(t.self, send.ctypes.data, recv.ctypes.data, 40, None) == 0
    out["a2a"] = recv
    u64p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    for unit in (1, 2, 4, 8):
        # PE r sends (r + 1) * (p + 2) elements to PE p; element = (src, dst, j) encoded
        cnt_s = np.array([(rank + 1) * (p + 2) for p in range(ws)], np.uint64)
        cnt_r = np.array([(p + 1) * (rank + 2) for p in range(ws)], np.uint64)
        sb, rb = cnt_s * np.uint64(unit), cnt_r * np.uint64(unit)
        so = np.concatenate([[0], np.cumsum(sb)[:-1]]).astype(np.uint64)
        ro = np.concatenate([[0], np.cumsum(rb)[:-1]]).astype(np.uint64)
        it = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[unit]
        sv = np.concatenate([(np.arange(int(cnt_s[p])) + 16 * rank + 4 * p) % 251 for p in range(ws)]).astype(it)
        rv = np.zeros(int(cnt_r.sum()), it)
        assert t.alltoallv(t.self, sv.ctypes.data, u64p(sb), u64p(so), rv.ctypes.data, u64p(rb), u64p(ro),
                           unit, None) == 0
        out[f"v{unit}"] = rv
    # a failing callback returns an error status (not LMR_OK) and keeps the exception
    bad = np.array([1, 0], np.uint64)
    st = t.alltoallv(t.self, send.ctypes.data, u64p(bad), u64p(bad), recv.ctypes.data, u64p(bad), u64p(bad), 1,
                     None)
    out["bad_status"] = np.array([st])
    try:
        tp.raise_pending()
        out["raised"] = np.array([0])
    except ValueError:
        out["raised"] = np.array([1])
    np.savez(os.path.join(outdir, f"t{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


def test_host_transport_callbacks_gloo():
    ws = 2
    port = 29650 + (os.getpid() % 200)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_transport_worker, args=(ws, port, d), nprocs=ws, join=True)
        pe = [dict(np.load(os.path.join(d, f"t{r}.npz"))) for r in range(ws)]
    for r in range(ws):
        exp = np.concatenate([np.arange(r * 5, r * 5 + 5) + 1000 * p for p in range(ws)])
        assert np.array_equal(pe[r]["a2a"], exp)
        for unit in (1, 2, 4, 8):
            exp = np.concatenate([(np.arange((p + 1) * (r + 2)) + 16 * p + 4 * r) % 251 for p in range(ws)])
            assert np.array_equal(pe[r][f"v{unit}"].astype(np.int64), exp)
        assert pe[r]["bad_status"][0] != 0 and pe[r]["raised"][0] == 1


def test_header_flag_constants_match_the_header(capi):
    """Every LMR_XHDR_* define of include/lamellar_gpu_ops.h has its mirror in _capi (same value)."""
    import re
    from lamellar_runtime_amd import _capi
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                            "lamellar_gpu_ops.h")).read()
    defs = dict(re.findall(r"#define LMR_XHDR_(\w+) (\d+)", hdr))
    assert {"WORDS", "SCALAR", "ORDERED", "FIXED", "DEVCOUNT", "OVERFLOW", "BUCKETS"} <= set(defs)
    for name, v in defs.items():
        assert getattr(_capi, "XHDR_" + name) == int(v), name
    flags = [int(v) for n, v in defs.items() if n != "WORDS"]
    assert all(f & (f - 1) == 0 for f in flags) and len(set(flags)) == len(flags)   # distinct single bits


def test_exchange_plan_flag_bits(capi):
    """The header's flags word: LMR_XHDR_SCALAR (1) means no values travel; LMR_XHDR_ORDERED (2)
    marks an in-order stream (one reference AM per destination) and changes no split."""
    from lamellar_runtime_amd import _capi
    assert (_capi.XHDR_SCALAR, _capi.XHDR_ORDERED) == (1, 2)
    sh = np.array([[4, -1, 2, 0, 1], [3, -1, 3, 9, 1]])          # ordered; ordered + scalar
    rh = np.array([[5, -1, 2, 0, 1], [6, -1, 3, 7, 1]])
    k, (isb, iso, irb, iro, vsb, vso, vrb, vro) = _plan(capi, 2, 4, 8, sh, rh)
    assert k == 1
    assert list(isb) == [16, 12] and list(irb) == [20, 24]       # every record's index travels
    assert list(vsb) == [32, 0] and list(vrb) == [40, 0]         # the scalar stream sends no values
