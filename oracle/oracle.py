"""ctypes wrapper of liblamellar_oracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / the timed CPU baseline. See
lamellar_oracle.h for what it restates and how it is pinned.
"""
import ctypes
import os
from ctypes import POINTER, Structure, c_double, c_int, c_int64, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liblamellar_oracle.so")


class Layout(Structure):
    _fields_ = [("distribution", c_uint32), ("num_pes", c_uint32), ("my_pe", c_uint32),
                ("sub", c_uint32), ("orig_elem_per_pe", c_uint64),
                ("orig_remaining_elems", c_uint64), ("offset", c_uint64), ("size", c_uint64)]

    def as_tuple(self):
        return tuple(getattr(self, f) for f, _ in self._fields_)


class Am(Structure):
    _fields_ = [("pe", c_uint32), ("_pad", c_uint32), ("byte_off", c_uint64),
                ("nbytes", c_uint64), ("nrec", c_uint64), ("res_off", c_uint64)]


class CpuTimes(Structure):
    _fields_ = [("pack_s", c_double), ("apply_s", c_double), ("total_s", c_double),
                ("n_buffers", c_uint64)]


_lib = None


def build():
    import subprocess
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        l = ctypes.CDLL(LIB)
        L = POINTER(Layout)
        sig = {
            "orc_layout_new": (c_int, [L, c_uint64, c_uint32, c_uint32, c_uint32]),
            "orc_layout_sub": (c_int, [L, c_uint64, c_uint64, L]),
            "orc_pe_and_offset": (c_int, [L, c_uint64, POINTER(c_uint64), POINTER(c_uint64)]),
            "orc_num_elems_pe": (c_uint64, [L, c_uint64]),
            "orc_local_slice_start": (c_uint64, [L, c_uint64]),
            "orc_index_size": (c_uint32, [L]),
            "orc_record_bytes": (c_uint32, [c_uint32, c_uint32]),
            "orc_record_val_offset": (c_uint32, [c_uint32, c_uint32]),
            "orc_op_ret_kind": (c_uint32, [c_uint32]),
            "orc_op_supported": (c_int, [c_uint32, c_uint32, c_uint32]),
            "orc_apply_mvmi": (c_int, [c_void_p, c_uint64, c_uint32, c_uint32, c_uint32, c_void_p,
                                       c_void_p, c_void_p, c_uint64, c_uint32, c_void_p, c_void_p]),
            "orc_apply_svmi": (c_int, [c_void_p, c_uint64, c_uint32, c_uint32, c_uint32, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_uint64, c_uint32, c_void_p,
                                       c_void_p]),
            "orc_apply_mvsi": (c_int, [c_void_p, c_uint64, c_uint32, c_uint32, c_uint32, c_void_p,
                                       c_void_p, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p]),
            "orc_num_chunks": (c_uint64, [c_uint64, c_uint64]),
            "orc_pack_mvmi": (c_int64, [L, c_uint32, c_void_p, c_void_p, c_uint64, c_uint32, c_uint64,
                                        c_uint64, c_void_p, c_uint64, c_void_p, c_uint64, c_void_p,
                                        POINTER(c_int)]),
            "orc_pack_svmi": (c_int64, [L, c_void_p, c_uint64, c_uint32, c_uint64, c_uint64, c_void_p,
                                        c_uint64, c_void_p, c_uint64, c_void_p, POINTER(c_int)]),
            "orc_batch_op": (c_int, [L, c_void_p, c_uint32, c_uint32, c_uint32, c_void_p, c_void_p,
                                     c_void_p, c_uint64, c_void_p, c_uint64, c_void_p, c_void_p]),
            "orc_scatter_results": (None, [c_void_p, c_void_p, c_uint64, c_uint32, c_void_p]),
            "orc_reduce": (None, [c_uint32, c_uint32, c_void_p, c_uint64, c_void_p, c_void_p]),
            "orc_reduce_tree": (None, [c_uint32, c_uint32, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p]),
            "orc_elem_step": (c_int, [c_uint32, c_uint32, c_uint32, c_uint64, c_uint64, c_void_p, c_void_p,
                                      POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint8)]),
            "orc_check_linearizable": (c_int, [c_uint32, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p,
                                               c_void_p, c_uint64, c_void_p, c_uint64, c_void_p, c_uint64,
                                               c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]),
            "cpu_baseline_run": (c_int, [c_uint32, c_uint32, c_void_p, c_uint64, c_void_p, c_void_p,
                                         c_void_p, c_uint64, c_uint32, c_uint64, c_void_p, c_void_p,
                                         POINTER(CpuTimes)]),
            "cpu_baseline_multi_pe": (c_int, [c_uint32, c_uint32, c_uint32, c_uint32, c_uint64, c_void_p,
                                              c_void_p, c_void_p, c_uint64, c_uint64, POINTER(CpuTimes)]),
        }
        for k, (r, a) in sig.items():
            f = getattr(l, k)
            f.restype = r
            f.argtypes = a
        _lib = l
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(c_void_p)


def layout_new(size, num_pes, my_pe=0, dist=0):
    L = Layout()
    st = lib().orc_layout_new(ctypes.byref(L), size, num_pes, my_pe, dist)
    assert st == 0
    return L


def layout_sub(L, start, end):
    out = Layout()
    st = lib().orc_layout_sub(ctypes.byref(L), start, end, ctypes.byref(out))
    assert st == 0
    return out


def pe_and_offset(L, idx):
    pe, off = c_uint64(), c_uint64()
    ok = lib().orc_pe_and_offset(ctypes.byref(L), idx, ctypes.byref(pe), ctypes.byref(off))
    return (pe.value, off.value) if ok else None


def num_elems_pe(L, pe):
    return lib().orc_num_elems_pe(ctypes.byref(L), pe)


def local_slice_start(L, pe):
    return lib().orc_local_slice_start(ctypes.byref(L), pe)


def index_size(L):
    return lib().orc_index_size(ctypes.byref(L))


def record_bytes(iw, dtype_code):
    return lib().orc_record_bytes(iw, dtype_code)


def record_val_offset(iw, dtype_code):
    return lib().orc_record_val_offset(iw, dtype_code)


def _scalar_buf(value, np_dtype):
    if value is None:
        return None
    return np.array([value]).astype(np_dtype)


def batch_op(L, slices, kind, dtype_code, np_dtype, op, gidx, vals, current=None, eps=None,
             want_results=True):
    """Sequential reference semantics over every PE's slice (list of numpy arrays, modified in place).
    gidx: uint64 array (len 1 = single index); vals: array of np_dtype (len 1 = single value).
    Returns (status, results, ok)."""
    gidx = np.ascontiguousarray(np.asarray(gidx, dtype=np.uint64).reshape(-1))
    vals = np.ascontiguousarray(np.asarray(vals).astype(np_dtype).reshape(-1))
    n = max(gidx.size, vals.size)
    res = np.zeros(n, dtype=np_dtype) if want_results else None
    ok = np.zeros(n, dtype=np.uint8)
    ptrs = (c_void_p * len(slices))(*[s.ctypes.data for s in slices])
    c = _scalar_buf(current, np_dtype)
    e = _scalar_buf(eps, np_dtype)
    st = lib().orc_batch_op(ctypes.byref(L), ptrs, kind, dtype_code, op, _ptr(c), _ptr(e),
                            _ptr(gidx), gidx.size, _ptr(vals), vals.size, _ptr(res), _ptr(ok))
    return st, res, ok


def apply_mvmi(slice_, kind, dtype_code, np_dtype, op, idx_vals_bytes, iw, current=None, eps=None):
    rb = record_bytes(iw, dtype_code)
    n = idx_vals_bytes.size // rb
    res = np.zeros(n, dtype=np_dtype)
    ok = np.zeros(n, dtype=np.uint8)
    c, e = _scalar_buf(current, np_dtype), _scalar_buf(eps, np_dtype)
    st = lib().orc_apply_mvmi(slice_.ctypes.data, slice_.size, kind, dtype_code, op, _ptr(c), _ptr(e),
                              _ptr(idx_vals_bytes), idx_vals_bytes.size, iw, _ptr(res), _ptr(ok))
    return st, res, ok


def apply_svmi(slice_, kind, dtype_code, np_dtype, op, val, indices_bytes, iw, current=None, eps=None):
    n = indices_bytes.size // iw
    res = np.zeros(n, dtype=np_dtype)
    ok = np.zeros(n, dtype=np.uint8)
    v = np.array([val]).astype(np_dtype)
    c, e = _scalar_buf(current, np_dtype), _scalar_buf(eps, np_dtype)
    st = lib().orc_apply_svmi(slice_.ctypes.data, slice_.size, kind, dtype_code, op, _ptr(c), _ptr(e),
                              _ptr(v), _ptr(indices_bytes), indices_bytes.size, iw, _ptr(res), _ptr(ok))
    return st, res, ok


def apply_mvsi(slice_, kind, dtype_code, np_dtype, op, vals, index, current=None, eps=None):
    vals = np.ascontiguousarray(np.asarray(vals).astype(np_dtype))
    res = np.zeros(vals.size, dtype=np_dtype)
    ok = np.zeros(vals.size, dtype=np.uint8)
    c, e = _scalar_buf(current, np_dtype), _scalar_buf(eps, np_dtype)
    st = lib().orc_apply_mvsi(slice_.ctypes.data, slice_.size, kind, dtype_code, op, _ptr(c), _ptr(e),
                              _ptr(vals), vals.nbytes, index, _ptr(res), _ptr(ok))
    return st, res, ok


def pack(L, dtype_code, np_dtype, gidx, vals, iw, threshold=100000, threads=1):
    """Returns (status, list of (pe, record bytes ndarray, res_pos ndarray)). vals None -> SVMI."""
    gidx = np.ascontiguousarray(np.asarray(gidx, dtype=np.uint64))
    n = gidx.size
    rb = iw if vals is None else record_bytes(iw, dtype_code)
    max_ams = n + 1024 * (L.num_pes + 1) + 16
    ams = (Am * max_ams)()
    cap = n * rb + 64
    byts = np.zeros(cap, dtype=np.uint8)
    pos = np.zeros(max(n, 1), dtype=np.uint64)
    st = c_int(0)
    if vals is None:
        na = lib().orc_pack_svmi(ctypes.byref(L), _ptr(gidx), n, iw, threshold, threads, ams, max_ams,
                                 _ptr(byts), cap, _ptr(pos), ctypes.byref(st))
    else:
        v = np.ascontiguousarray(np.asarray(vals).astype(np_dtype))
        na = lib().orc_pack_mvmi(ctypes.byref(L), dtype_code, _ptr(gidx), _ptr(v), n, iw, threshold,
                                 threads, ams, max_ams, _ptr(byts), cap, _ptr(pos), ctypes.byref(st))
    out = []
    for i in range(max(na, 0)):
        a = ams[i]
        out.append((a.pe, byts[a.byte_off:a.byte_off + a.nbytes].copy(),
                    pos[a.res_off:a.res_off + a.nrec].copy()))
    return st.value, out


def cpu_baseline(dtype_code, np_dtype, op, shard, gidx, vals, threads, threshold=100000,
                 want_results=False, current=None):
    """Reference-structured threaded CPU apply (bench.py cpu_baseline leg)."""
    gidx = np.ascontiguousarray(gidx, dtype=np.uint64)
    n = gidx.size
    v = None
    sv = None
    if np.ndim(vals) == 0:
        sv = np.array([vals]).astype(np_dtype)
    else:
        v = np.ascontiguousarray(np.asarray(vals).astype(np_dtype))
    res = np.zeros(n, dtype=np_dtype) if want_results else None
    t = CpuTimes()
    c = _scalar_buf(current, np_dtype)
    st = lib().cpu_baseline_run(dtype_code, op, shard.ctypes.data, shard.size, _ptr(gidx), _ptr(v),
                                _ptr(sv), n, threads, threshold, _ptr(c), _ptr(res), ctypes.byref(t))
    return st, t, res


def cpu_baseline_multi_pe(dtype_code, np_dtype, op, array_len, shards, gidx, vals, threads_per_pe,
                          threshold=100000):
    """C4 CPU baseline (bench.py cpu_baseline leg): len(shards) PEs of threads_per_pe threads
    exchanging op buffers through shared memory (the shmem lamellae's protocol restated,
    cpu_baseline.c). shards[p] is updated in place; gidx[p] / vals[p] are PE p's records
    (equal counts)."""
    P = len(shards)
    n = int(gidx[0].size)
    gidx = [np.ascontiguousarray(g, dtype=np.uint64) for g in gidx]
    vals = [np.ascontiguousarray(np.asarray(v).astype(np_dtype)) for v in vals]
    assert all(g.size == n for g in gidx) and all(v.size == n for v in vals)
    arr_p = (ctypes.c_void_p * P)(*[s.ctypes.data for s in shards])
    arr_g = (ctypes.c_void_p * P)(*[g.ctypes.data for g in gidx])
    arr_v = (ctypes.c_void_p * P)(*[v.ctypes.data for v in vals])
    t = CpuTimes()
    st = lib().cpu_baseline_multi_pe(dtype_code, op, P, threads_per_pe, array_len, arr_p, arr_g, arr_v, n,
                                     threshold, ctypes.byref(t))
    return st, t


def check_linearizable(kind, dtype_code, np_dtype, op, init, final, idx, vals, rets=None, oks=None,
                       current=None, eps=None, max_nodes=1 << 22):
    """Per element: do the returned values / Ok flags and the final value come from
    some serial order of that element's records (linearize.c)? -> (status, element):
    status 0 = linearisable, 1 = not (element names one), 2 = undecided."""
    init = np.ascontiguousarray(np.asarray(init).astype(np_dtype))
    final = np.ascontiguousarray(np.asarray(final).astype(np_dtype))
    assert init.size == final.size
    idx = np.ascontiguousarray(np.asarray(idx, dtype=np.uint64).reshape(-1))
    vals = np.ascontiguousarray(np.asarray(vals).astype(np_dtype).reshape(-1))
    rets = None if rets is None else np.ascontiguousarray(np.asarray(rets).astype(np_dtype).reshape(-1))
    oks = None if oks is None else np.ascontiguousarray(np.asarray(oks, dtype=np.uint8).reshape(-1))
    c, e = _scalar_buf(current, np_dtype), _scalar_buf(eps, np_dtype)
    bad = c_uint64(0)
    st = lib().orc_check_linearizable(kind, dtype_code, op, _ptr(c), _ptr(e), _ptr(init), _ptr(final), init.size,
                                      _ptr(idx), idx.size, _ptr(vals), vals.size, _ptr(rets), _ptr(oks),
                                      max_nodes, ctypes.byref(bad))
    return st, bad.value


REDUCE_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3}


def reduce(dtype_code, np_dtype, op, data):
    """One PE's reduction step (array_reduce.rs:82-88): value or None."""
    a = np.ascontiguousarray(np.asarray(data, dtype=np_dtype))
    out = np.zeros(1, dtype=np_dtype)
    has = np.zeros(1, dtype=np.uint8)
    lib().orc_reduce(dtype_code, REDUCE_OPS[op], a.ctypes.data if a.size else None, a.size, out.ctypes.data,
                     has.ctypes.data)
    return out[0] if has[0] else None


def reduce_tree(dtype_code, np_dtype, op, per_pe):
    """Cross-PE tree (array_reduce.rs:90-107) over per-PE values (None = empty PE)."""
    n = len(per_pe)
    vals = np.array([0 if v is None else v for v in per_pe], dtype=np_dtype)
    has = np.array([v is not None for v in per_pe], dtype=np.uint8)
    out = np.zeros(1, dtype=np_dtype)
    oh = np.zeros(1, dtype=np.uint8)
    lib().orc_reduce_tree(dtype_code, REDUCE_OPS[op], vals.ctypes.data, has.ctypes.data, n, out.ctypes.data,
                          oh.ctypes.data)
    return out[0] if oh[0] else None
