"""Host-buffer ingestion (lmr_apply_mvmi_host): the reference's IdxVal<I,T> op
buffer in host memory -> pieces uploaded / applied / results downloaded on
three streams. Checked against the oracle's apply of the same bytes
(bit-exact for integers), over several pieces (LMR_HOST_PIECE_RECORDS is set
small here so both the tiled (>= 2^16 records) and the direct last piece run),
with registered and pageable host buffers (pageable ones go through the
library's pinned bounce slots), and registered ranges unregistered and freed
right after use, their memory reused by the next allocations."""
import os

import numpy as np
import pytest
import torch

os.environ.setdefault("LMR_HOST_PIECE_RECORDS", "65536")

from opgen import CAS, CODE, FETCH_ADD, NP, ADD, XOR, bits_equal, cas_operands, rand_elems, rand_vals, ret_kind, to_aos

pytestmark = pytest.mark.gpu


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()


@pytest.mark.parametrize("dt,op,register", [("u64", ADD, True), ("u64", FETCH_ADD, True), ("u32", XOR, False),
                                            ("i64", FETCH_ADD, False), ("u32", CAS, True), ("f64", FETCH_ADD, True)])
def test_apply_mvmi_host_matches_oracle(world, orc, lam, dt, op, register):
    k = world.team().kernels
    rng = np.random.default_rng(31)
    shard_len = 300000
    n = 3 * 65536 + 1234                                  # 3 full pieces + a direct-path tail
    shard0 = rand_elems(dt, shard_len, rng, op)
    idx = rng.permutation(shard_len)[:n].astype(np.uint64)   # conflict-free: exact results
    vals = rand_vals(dt, n, rng, op)
    cur = eps = None
    if op == CAS:
        cur, eps, shard0 = cas_operands(dt, shard0, vals, rng)
    iw = 4
    rb, vo = orc.record_bytes(iw, CODE[dt]), orc.record_val_offset(iw, CODE[dt])
    buf = to_aos(idx, vals, iw, dt, rb, vo)
    kind = 2 if dt.startswith("f") else 1
    ref = shard0.copy()
    st_o, res_o, ok_o = orc.apply_mvmi(ref, kind, CODE[dt], NP[dt], op, buf, iw, cur, eps)
    assert st_o == 0
    dt_obj = lam.dtype_of(dt)
    d_shard = to_dev(shard0)
    rk = ret_kind(op)
    h_res = np.zeros(n, dtype=NP[dt]) if rk else None
    h_ok = np.zeros(n, dtype=np.uint8) if rk == 2 else None
    if register:
        k.host_register(buf)
        if h_res is not None:
            k.host_register(h_res)
    try:
        cb = dt_obj.to_bits(cur) if cur is not None else 0
        k.apply_mvmi_host(d_shard, shard_len, kind, dt_obj, op, buf, iw, h_res, h_ok, cb, 0)
    finally:
        if register:
            k.host_unregister(buf)
            if h_res is not None:
                k.host_unregister(h_res)
    assert k.errors() == 0
    got = d_shard.cpu().numpy().view(NP[dt])[:shard_len]
    assert bits_equal(got, ref)
    if rk:
        assert bits_equal(h_res, res_o)
    if rk == 2:
        assert np.array_equal(h_ok, ok_o)


def test_apply_mvmi_host_collisions_sum(world, orc, lam):
    """u64 add with heavy collisions over 5 pieces: final shard == oracle (wrapping sums commute)."""
    k = world.team().kernels
    rng = np.random.default_rng(32)
    shard_len, n = 5000, 5 * 65536
    idx = rng.integers(0, shard_len, n).astype(np.uint64)
    vals = rng.integers(0, 2**63, n).astype(np.uint64)
    rb, vo = orc.record_bytes(2, CODE["u64"]), orc.record_val_offset(2, CODE["u64"])
    buf = to_aos(idx, vals, 2, "u64", rb, vo)
    ref = np.zeros(shard_len, np.uint64)
    assert orc.apply_mvmi(ref, 1, CODE["u64"], np.uint64, ADD, buf, 2)[0] == 0
    d_shard = torch.zeros(shard_len, dtype=torch.int64, device="cuda")
    k.apply_mvmi_host(d_shard, shard_len, 1, lam.dtype_of("u64"), ADD, buf, 2)
    assert np.array_equal(d_shard.cpu().numpy().view(np.uint64), ref)


def test_registered_ranges_sharing_a_page(world, orc, lam):
    """Registered op buffers and result arrays that share a page (slices of one host arena), the
    pattern that preceded every host-path device fault: registration records the ranges and locks
    nothing (lmr_host_registered: no pinned pages), so records, results and compare_exchange's Ok
    flags all travel through the library's pinned bounce slots. The arena is freed afterwards and
    its memory reused by the next arena and by pageable host-to-device copies in between. Every
    round is bit-exact against the oracle."""
    k = world.team().kernels
    dt = "u32"
    shard_len, n = 300000, 2 * 65536 + 777
    rb, vo = orc.record_bytes(4, CODE[dt]), orc.record_val_offset(4, CODE[dt])
    for rnd in range(4):
        rng = np.random.default_rng(900 + rnd)
        shard0 = rand_elems(dt, shard_len, rng, CAS)
        idx = rng.permutation(shard_len)[:n].astype(np.uint64)
        vals = rand_vals(dt, n, rng, CAS)
        cur, _, shard0 = cas_operands(dt, shard0, vals, rng)
        recs = to_aos(idx, vals, 4, dt, rb, vo)
        # one arena: records, then results 16 bytes later (the two ranges share a page)
        arena = np.zeros(recs.nbytes + 16 + n * 4 + 64, np.uint8)
        buf = arena[:recs.nbytes]
        buf[:] = recs
        h_res = arena[recs.nbytes + 16:recs.nbytes + 16 + n * 4].view(np.uint32)
        h_ok = np.zeros(n, np.uint8)                        # pageable
        ref = shard0.copy()
        st_o, res_o, ok_o = orc.apply_mvmi(ref, 1, CODE[dt], NP[dt], CAS, recs, 4, cur, None)
        assert st_o == 0
        d_shard = to_dev(shard0)
        k.host_register(buf)
        k.host_register(h_res)
        try:
            assert k.host_registered(buf) == (0, 0, 1) and k.host_registered(h_res) == (0, 0, 1)
            k.apply_mvmi_host(d_shard, shard_len, 1, lam.dtype_of(dt), CAS, buf, 4, h_res, h_ok,
                              lam.dtype_of(dt).to_bits(cur), 0)
        finally:
            k.host_unregister(buf)
            left = k.host_registered(h_res)
            k.host_unregister(h_res)
        assert left == (0, 0, 1)
        assert k.host_registered(h_res) is None and k.host_registered(buf) is None
        assert k.errors() == 0
        assert bits_equal(d_shard.cpu().numpy().view(NP[dt])[:shard_len], ref)
        assert bits_equal(h_res.copy(), res_o)
        assert np.array_equal(h_ok, ok_o)
        del buf, h_res, arena
        # pageable copies of fresh allocations (the freed arena's memory is handed out again)
        for _ in range(3):
            x = rng.integers(0, 2**31, n, dtype=np.int64)
            assert np.array_equal(torch.from_numpy(x).cuda().cpu().numpy(), x)


def test_host_alloc_buffers_dma_in_place(world, orc, lam):
    """Short-lived pinned buffers from lmr_host_alloc: records and fetch results DMA'd in place
    without registration (u64 fetch_add, conflict-free, bit-exact), freed after each round."""
    k = world.team().kernels
    rng = np.random.default_rng(41)
    shard_len, n = 300000, 2 * 65536 + 99
    rb, vo = orc.record_bytes(4, CODE["u64"]), orc.record_val_offset(4, CODE["u64"])
    for _ in range(3):
        shard0 = rand_elems("u64", shard_len, rng, FETCH_ADD)
        idx = rng.permutation(shard_len)[:n].astype(np.uint64)
        vals = rand_vals("u64", n, rng, FETCH_ADD)
        recs = to_aos(idx, vals, 4, "u64", rb, vo)
        ref = shard0.copy()
        st_o, res_o, _ = orc.apply_mvmi(ref, 1, CODE["u64"], np.uint64, FETCH_ADD, recs, 4)
        assert st_o == 0
        buf = k.host_alloc(recs.nbytes)
        h_res = k.host_alloc(n * 8, np.uint64)
        try:
            buf[:] = recs
            d_shard = to_dev(shard0)
            k.apply_mvmi_host(d_shard, shard_len, 1, lam.dtype_of("u64"), FETCH_ADD, buf, 4, h_res)
            assert bits_equal(d_shard.cpu().numpy().view(np.uint64)[:shard_len], ref)
            assert bits_equal(h_res.copy(), res_o)
        finally:
            k.host_free(buf)
            k.host_free(h_res)


_HEAP = []


def _heap(k, nbytes=64 << 20):
    """One page-aligned host heap for the whole test process, registered once and never
    unregistered (the reference's lamellae heap lives from world init to shutdown)."""
    if not _HEAP:
        import mmap
        m = mmap.mmap(-1, nbytes)
        a = np.frombuffer(m, dtype=np.uint8)
        k.host_register_heap(a)
        _HEAP.extend([m, a])
    return _HEAP[1]


def test_heap_buffers_dma_in_place(world, orc, lam):
    """A lamellae-style heap registered once (lmr_host_register_heap: its whole inner pages
    page-locked for its lifetime): op buffers and fetch results placed at unaligned offsets inside
    it DMA their pinned pages in place and stage the partial end pages; results bit-exact against
    the oracle; a caller range inside the heap is refused (ranges never overlap)."""
    from lamellar_runtime_amd.kernels import LamellarError
    k = world.team().kernels
    heap = _heap(k)
    base = heap.ctypes.data
    info = k.host_registered(heap[100:200])
    assert info is not None and info[0] == base and info[1] == heap.nbytes and info[2] == 1
    with pytest.raises(LamellarError):
        k.host_register(heap[4096:8192])
    for dt, op in (("u64", FETCH_ADD), ("u32", CAS), ("f64", FETCH_ADD)):
        rng = np.random.default_rng(77 + CODE[dt])
        shard_len, n = 300000, 3 * 65536 + 1234
        shard0 = rand_elems(dt, shard_len, rng, op)
        idx = rng.permutation(shard_len)[:n].astype(np.uint64)
        vals = rand_vals(dt, n, rng, op)
        cur = eps = None
        if op == CAS:
            cur, eps, shard0 = cas_operands(dt, shard0, vals, rng)
        iw = 4
        rb, vo = orc.record_bytes(iw, CODE[dt]), orc.record_val_offset(iw, CODE[dt])
        recs = to_aos(idx, vals, iw, dt, rb, vo)
        buf = heap[1000:1000 + recs.nbytes]
        buf[:] = recs
        eb = np.dtype(NP[dt]).itemsize
        r0 = (1000 + recs.nbytes + 4095) // 4096 * 4096 + 24      # results start 24 B into a page
        h_res = heap[r0:r0 + n * eb].view(NP[dt])
        h_ok = heap[r0 + n * eb + 8:r0 + n * eb + 8 + n] if op == CAS else None
        ref = shard0.copy()
        kind = 2 if dt.startswith("f") else 1
        st_o, res_o, ok_o = orc.apply_mvmi(ref, kind, CODE[dt], NP[dt], op, recs, iw, cur, eps)
        assert st_o == 0
        d_shard = to_dev(shard0)
        dto = lam.dtype_of(dt)
        k.apply_mvmi_host(d_shard, shard_len, kind, dto, op, buf, iw, h_res, h_ok,
                          dto.to_bits(cur) if cur is not None else 0, 0)
        assert k.errors() == 0
        assert bits_equal(d_shard.cpu().numpy().view(NP[dt])[:shard_len], ref)
        assert bits_equal(h_res.copy(), res_o)
        if op == CAS:
            assert np.array_equal(h_ok, ok_o)


HEAP_SHUTDOWN_WORKER = r'''
import mmap, os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ["LMR_ROOT"])
from _lamellar_bootstrap import load_package
lam = load_package()
from lamellar_runtime_amd import _capi
world = lam.LamellarWorldBuilder().build()
k = world.team().kernels
lib = _capi.lib()
rng = np.random.default_rng(2026)
shard_len, n = 1 << 20, 3 * 65536 + 77
for rnd in range(3):
    m = mmap.mmap(-1, 32 << 20)                       # the lamellae heap of one world's lifetime
    heap = np.frombuffer(m, dtype=np.uint8)
    k.host_register_heap(heap)
    idx = rng.integers(0, shard_len, n).astype(np.uint32)
    vals = rng.integers(0, 2**40, n, dtype=np.uint64)
    rec = np.zeros(n, np.dtype([("i", "<u4"), ("pad", "<u4"), ("v", "<u8")]))
    rec["i"], rec["v"] = idx, vals
    buf = heap[4096 + 8 * rnd:4096 + 8 * rnd + rec.nbytes]
    buf[:] = rec.view(np.uint8)
    olds = heap[(8 << 20) + 16:(8 << 20) + 16 + 8 * n].view(np.uint64)
    shard = torch.zeros(shard_len, dtype=torch.int64, device=k.device)
    dt = lam.dtype_of("u64")
    k.apply_mvmi_host(shard, shard_len, 1, dt, int(lam.ArrayOpCmd.FetchAdd), buf, 4, olds)
    ref = np.zeros(shard_len, np.uint64)
    np.add.at(ref, idx.astype(np.int64), vals)
    assert np.array_equal(shard.cpu().numpy().view(np.uint64), ref)
    got = olds.copy()
    # shutdown: the heap unregistered (the library drains its host-stage copies first), dropped,
    # unmapped; then pageable copies of fresh memory, some of it at the heap's old addresses
    k.host_unregister_heap(heap)
    del buf, olds, heap
    m.close()
    for _ in range(3):
        x = rng.integers(0, 2**62, (4 << 20) // 8, dtype=np.int64)
        assert np.array_equal(torch.from_numpy(x).cuda().cpu().numpy(), x)
    torch.cuda.synchronize()
    assert k.errors() == 0
    # the olds per element chain from 0 (distinct partial sums)
    order = np.lexsort((got, idx))
    ii, gg = idx[order], got[order]
    first = np.r_[True, ii[1:] != ii[:-1]]
    assert np.all(gg[first] == 0)
print("heap shutdown ok", flush=True)
'''


def test_heap_shutdown_path():
    """The lamellae heap's whole life, three times in one process: lmr_host_register_heap over a
    fresh mapping, a fetch_add whose records and olds live in it (DMA'd in place), then
    lmr_host_unregister_heap (the library drains its host-stage copies first), unmap, and pageable
    copies of fresh memory. Runs in a process of its own: the fault rounds 3-5 saw followed an
    unlock of caller memory, and a repeat must not take the suite's process with it."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LMR_ROOT=root, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "-c", HEAP_SHUTDOWN_WORKER], env=env, timeout=170,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert p.returncode == 0 and "heap shutdown ok" in p.stdout, p.stdout[-4000:]
