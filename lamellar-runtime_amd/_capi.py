"""ctypes binding of liblamellar_gpu_ops.so (include/lamellar_gpu_ops.h).

This is the same binding a Rust maintainer would write with ``extern "C"``
(see INTEGRATION.md); Python uses it for the host-side mirror of the
reference's op-builder API, the tests and the benchmark.

There is no fallback: if the HIP library is missing or fails to load, importing
the package's device path raises :class:`LamellarLibraryError`.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_char_p, c_int, c_uint8, c_uint32,
                    c_uint64, c_void_p)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LAMELLAR_GPU_OPS_LIB",
                          os.path.join(_HERE, "liblamellar_gpu_ops.so"))


class LamellarLibraryError(RuntimeError):
    pass


class lmr_layout_t(Structure):
    """UnsafeArrayInner index-math fields (src/array/unsafe.rs:107-116)."""
    _fields_ = [
        ("distribution", c_uint32),
        ("num_pes", c_uint32),
        ("my_pe", c_uint32),
        ("sub", c_uint32),
        ("orig_elem_per_pe", c_uint64),
        ("orig_remaining_elems", c_uint64),
        ("offset", c_uint64),
        ("size", c_uint64),
    ]

    def as_tuple(self):
        return tuple(getattr(self, f) for f, _ in self._fields_)


class lmr_apply_desc_t(Structure):
    _fields_ = [
        ("shard", c_void_p),
        ("shard_len", c_uint64),
        ("kind", c_uint32),
        ("dtype", c_uint32),
        ("op", c_uint32),
        ("strategy", c_uint32),
        ("cmp_bits", c_uint64),
        ("eps_bits", c_uint64),
    ]


# lmr_transport_t callbacks (include/lamellar_gpu_ops.h, exchange section)
ALLTOALL_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p)
ALLTOALLV_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, POINTER(c_uint64), POINTER(c_uint64), c_void_p,
                                POINTER(c_uint64), POINTER(c_uint64), c_uint32, c_void_p)


class lmr_transport_t(Structure):
    """The exchange's all-to-all(v) provider: RCCL (lmr_transport_rccl_create) or
    a caller's callbacks (host_buffers = 1: the library stages through pinned host
    memory and the callbacks see host pointers)."""
    _fields_ = [
        ("num_pes", c_uint32),
        ("my_pe", c_uint32),
        ("host_buffers", c_uint32),
        ("flags", c_uint32),          # LMR_TRANSPORT_SPLIT_HEADERS = 1
        ("self", c_void_p),
        ("alltoall", ALLTOALL_FN),
        ("alltoallv", ALLTOALLV_FN),
    ]


XHDR_WORDS = 7     # LMR_XHDR_WORDS
XHDR_SCALAR, XHDR_ORDERED = 1, 2   # LMR_XHDR_SCALAR, LMR_XHDR_ORDERED (flags word of a header row)
# LMR_XHDR_FIXED, _DEVCOUNT, _OVERFLOW, _BUCKETS: fixed regions, device-count staging, a non-empty
# overflow list, regions laid out by owner bucket (sent whole)
XHDR_FIXED, XHDR_DEVCOUNT, XHDR_OVERFLOW, XHDR_BUCKETS = 4, 8, 16, 32


# ---- AM wire format (include/lamellar_gpu_ops.h, "AM wire format")
class lmr_net_darc_t(Structure):
    _fields_ = [("inner_addr", c_uint64), ("backend", c_uint32), ("reserved_", c_uint32),
                ("orig_world_pe", c_uint64), ("orig_team_pe", c_uint64)]


class lmr_am_view_t(Structure):
    _fields_ = [("shape", c_uint32), ("kind", c_uint32), ("dtype", c_uint32), ("op", c_uint32),
                ("cmp_bits", c_uint64), ("eps_bits", c_uint64),
                ("data", lmr_net_darc_t), ("lock", lmr_net_darc_t),
                ("native_type", c_uint32), ("distribution", c_uint32),
                ("orig_elem_per_pe", c_uint64), ("orig_remaining_elems", c_uint64), ("elem_size", c_uint64),
                ("offset", c_uint64), ("size", c_uint64),
                ("sub", c_uint32), ("index_size", c_uint32),
                ("val_bits", c_uint64), ("index", c_uint64),
                ("recs_offset", c_uint64), ("recs_bytes", c_uint64), ("body_bytes", c_uint64)]


class lmr_msg_entry_t(Structure):
    _fields_ = [("cmd", c_uint32), ("src", c_uint32), ("am_id", ctypes.c_int32),
                ("shape", c_uint32), ("kind", c_uint32), ("dtype", c_uint32),
                ("team_addr", c_uint64), ("req_id", c_uint64), ("req_sub_id", c_uint64),
                ("body_offset", c_uint64), ("body_bytes", c_uint64)]


class lmr_shard_t(Structure):
    _fields_ = [("shard", c_void_p), ("shard_len", c_uint64), ("strategy", c_uint32), ("reserved_", c_uint32)]


# (user, cmd, am_id, body, avail, *shape, *kind, *dtype, *body_bytes) -> 0 op AM / 1 other AM (sized)
AM_RESOLVER_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_uint32, ctypes.c_int32, c_void_p, c_uint64, POINTER(c_uint32),
                                  POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint64))
SHARD_RESOLVER_FN = ctypes.CFUNCTYPE(c_int, c_void_p, POINTER(lmr_am_view_t), POINTER(lmr_shard_t))

# name -> (restype, argtypes). Every symbol of include/lamellar_gpu_ops.h.
SIGNATURES = {
    "lmr_abi_version": (c_uint32, []),
    "lmr_status_string": (c_char_p, [c_int]),
    "lmr_ctx_create": (c_int, [c_int, POINTER(c_void_p)]),
    "lmr_ctx_destroy": (c_int, [c_void_p]),
    "lmr_ctx_reserve": (c_int, [c_void_p, c_uint64]),
    "lmr_ctx_error": (c_int, [c_void_p, c_void_p, POINTER(c_uint32), c_int]),
    "lmr_ctx_profile": (c_int, [c_void_p, c_int]),
    "lmr_ctx_profile_read": (c_int, [c_void_p, c_void_p, POINTER(ctypes.c_double), POINTER(c_uint64),
                                     POINTER(c_uint64), c_int]),
    "lmr_layout_new": (c_int, [POINTER(lmr_layout_t), c_uint64, c_uint32, c_uint32, c_uint32]),
    "lmr_layout_sub": (c_int, [POINTER(lmr_layout_t), c_uint64, c_uint64, POINTER(lmr_layout_t)]),
    "lmr_pe_and_offset": (c_int, [POINTER(lmr_layout_t), c_uint64, POINTER(c_uint64), POINTER(c_uint64)]),
    "lmr_num_elems_pe": (c_uint64, [POINTER(lmr_layout_t), c_uint32]),
    "lmr_local_slice_start": (c_uint64, [POINTER(lmr_layout_t), c_uint32]),
    "lmr_index_size": (c_uint32, [POINTER(lmr_layout_t)]),
    "lmr_record_bytes": (c_uint32, [c_uint32, c_uint32]),
    "lmr_record_val_offset": (c_uint32, [c_uint32, c_uint32]),
    "lmr_op_ret_kind": (c_uint32, [c_uint32]),
    "lmr_op_supported": (c_int, [c_uint32, c_uint32, c_uint32]),
    "lmr_pack": (c_int, [c_void_p, POINTER(lmr_layout_t), c_void_p, c_uint64, c_void_p, c_uint32,
                         c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "lmr_host_register": (c_int, [c_void_p, c_uint64]),
    "lmr_host_unregister": (c_int, [c_void_p]),
    "lmr_host_register_heap": (c_int, [c_void_p, c_uint64]),
    "lmr_host_unregister_heap": (c_int, [c_void_p]),
    "lmr_host_registered": (c_int, [c_void_p, c_uint64, POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint32)]),
    "lmr_host_alloc": (c_int, [c_uint64, POINTER(c_void_p)]),
    "lmr_host_free": (c_int, [c_void_p]),
    "lmr_apply_mvmi_host": (c_int, [c_void_p, POINTER(lmr_apply_desc_t), c_void_p, c_uint64, c_uint32,
                                    c_void_p, c_void_p, c_void_p]),
    "lmr_reduce": (c_int, [c_void_p, c_uint32, c_uint32, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p]),
    "lmr_pack_unordered": (c_int, [c_void_p, POINTER(lmr_layout_t), c_void_p, c_uint64, c_void_p, c_uint32,
                                   c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "lmr_pack_regions": (c_int, [c_void_p, POINTER(lmr_layout_t), c_void_p, c_uint64, c_void_p, c_uint32,
                                 c_uint32, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p]),
    "lmr_apply_mvmi": (c_int, [c_void_p, POINTER(lmr_apply_desc_t), c_void_p, c_uint64, c_uint32,
                               c_void_p, c_void_p, c_void_p]),
    "lmr_apply_svmi": (c_int, [c_void_p, POINTER(lmr_apply_desc_t), c_void_p, c_void_p, c_uint64,
                               c_uint32, c_void_p, c_void_p, c_void_p]),
    "lmr_apply_mvsi": (c_int, [c_void_p, POINTER(lmr_apply_desc_t), c_void_p, c_uint64, c_uint64,
                               c_void_p, c_void_p, c_void_p]),
    "lmr_apply_soa": (c_int, [c_void_p, POINTER(lmr_apply_desc_t), c_void_p, c_uint32, c_void_p,
                              c_void_p, c_uint64, c_void_p, c_void_p, c_void_p]),
    "lmr_scatter_results": (c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_void_p, c_void_p,
                                    c_void_p, c_void_p]),
    "lmr_stage_begin": (c_int, [c_void_p, POINTER(lmr_apply_desc_t)]),
    "lmr_stage_soa": (c_int, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_uint64, c_void_p,
                              c_void_p, c_void_p]),
    "lmr_stage_op": (c_int, [c_void_p, c_uint32, c_uint64, c_uint64, c_void_p]),
    "lmr_stage_flush": (c_int, [c_void_p, c_void_p]),
    "lmr_stage_finish": (c_int, [c_void_p, c_void_p]),
    "lmr_ctx_exchange_defer": (c_int, [c_void_p, c_int]),
    "lmr_exchange_flush": (c_int, [c_void_p, c_void_p]),
    "lmr_rccl_unique_id": (c_int, [c_void_p]),
    "lmr_transport_rccl_create": (c_int, [c_void_p, c_uint32, c_uint32, c_int, POINTER(c_void_p)]),
    "lmr_transport_rccl_destroy": (c_int, [c_void_p]),
    "lmr_transport_peer_create": (c_int, [c_void_p, ctypes.c_char_p, c_uint64, c_int, POINTER(c_void_p)]),
    "lmr_transport_peer_destroy": (c_int, [c_void_p]),
    "lmr_transport_peer_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    "lmr_batch_exchange": (c_int, [c_void_p, c_void_p, POINTER(lmr_layout_t), POINTER(lmr_apply_desc_t),
                                   c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_uint64, c_void_p,
                                   c_void_p, c_void_p]),
    "lmr_exchange_plan": (c_uint64, [c_uint32, c_uint32, c_uint32, c_void_p, c_void_p] + [c_void_p] * 8),
    "lmr_am_decode": (c_int, [c_void_p, c_uint64, c_uint32, c_uint32, c_uint32, POINTER(lmr_am_view_t)]),
    "lmr_am_encode": (c_int, [POINTER(lmr_am_view_t), c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]),
    "lmr_msg_parse": (c_int, [c_void_p, c_uint64, AM_RESOLVER_FN, c_void_p, POINTER(lmr_msg_entry_t), c_uint32,
                              POINTER(c_uint32)]),
    "lmr_reply_bytes": (c_uint64, [c_uint32, c_uint32, c_uint64]),
    "lmr_reply_encode": (c_int, [c_uint32, c_uint32, c_uint64, c_void_p, c_void_p, c_void_p, c_uint64]),
    "lmr_apply_msg": (c_int, [c_void_p, c_void_p, c_uint64, AM_RESOLVER_FN, SHARD_RESOLVER_FN, c_void_p, c_void_p,
                              c_uint64, POINTER(c_uint64), POINTER(c_uint64), c_uint32, POINTER(c_uint32),
                              c_void_p]),
}

STAGES = ["direct", "mvsi", "bin_count", "scan", "bin_scatter", "tile_apply", "pack",
          "scatter_results", "fine_scatter", "unpartition", "window", "ordered"]

_lib = None


def lib():
    """Load (once) and return the HIP library; raise loudly if unavailable."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LamellarLibraryError(
                f"liblamellar_gpu_ops.so not found at {LIB_PATH}; build it with "
                f"`python __graft_entry__.py build` (hipcc --offload-arch=gfx950)")
        try:
            l = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - environment specific
            raise LamellarLibraryError(f"failed to load {LIB_PATH}: {e}") from e
        side = "LAMELLAR_GPU_OPS_LIB" in os.environ      # an earlier build for a same-box A/B
        for name, (res, args) in SIGNATURES.items():
            if side and not hasattr(l, name):
                continue                                   # (entry points added since that build)
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def status_string(st: int) -> str:
    return lib().lmr_status_string(st).decode()
