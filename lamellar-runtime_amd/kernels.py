"""Device kernels of the batched element-op path, called through the C ABI.

`DeviceKernels` is the only product implementation: every method enqueues
gfx950 kernels of liblamellar_gpu_ops.so on torch's current HIP stream. There
is no CPU fallback; without a GPU the constructor raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import byref, c_uint32, c_uint64, c_void_p

import numpy as np
import torch

from . import _capi
from .types import (ERRBIT_DIVZERO, ERRBIT_OOB, ERRBIT_OVERFLOW, ERRBIT_TRANSPORT, ERRBIT_UNSUPPORTED,
                    LmrStatus, Strategy)


class LamellarError(RuntimeError):
    """Raised where the reference panics (OOB index, integer div by zero, ...)."""

    def __init__(self, status, msg=""):
        self.status = LmrStatus(status)
        super().__init__(f"{self.status.name}: {msg}")


def check(st: int, what: str = ""):
    if st != 0:
        raise LamellarError(st, f"{what}: {_capi.status_string(st)}")


def errbits_to_status(bits: int) -> int:
    if bits & ERRBIT_OOB:
        return LmrStatus.OOB
    if bits & ERRBIT_DIVZERO:
        return LmrStatus.DIVZERO
    if bits & ERRBIT_OVERFLOW:
        return LmrStatus.OVERFLOW
    if bits & ERRBIT_UNSUPPORTED:
        return LmrStatus.UNSUPPORTED
    if bits & ERRBIT_TRANSPORT:
        return LmrStatus.HIP
    return LmrStatus.OK


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class DeviceKernels:
    """Per-device context + the C-ABI calls, on torch's current stream."""

    is_device = True

    def __init__(self, device: torch.device, strategy: int = Strategy.Auto,
                 max_ws_records: int = 1 << 29):
        if device.type != "cuda" or not torch.cuda.is_available():
            raise LamellarError(LmrStatus.INVALID,
                                "the batched op path runs on a HIP device; no GPU is visible")
        self.device = device
        self.lib = _capi.lib()
        self.ctx = c_void_p()
        check(self.lib.lmr_ctx_create(device.index or 0, byref(self.ctx)), "lmr_ctx_create")
        self.strategy = int(strategy)
        # (LAMELLAR_MAX_WS_RECORDS raises or lowers the cap, e.g. for deeper deferred sessions)
        self.max_ws_records = int(os.environ.get("LAMELLAR_MAX_WS_RECORDS", max_ws_records))
        self.reserved = 0
        # the open deferred session of asynchronous batches (defer_soa): [shard key, (op, cmp, eps),
        # tensors its kernels still write or read]; applied by flush()
        self._deferred = None
        # record tensors of the open lmr_stage_* session, held until it is partitioned
        self._staged_refs = []
        # deferred exchange sessions (lmr_ctx_exchange_defer): a batch exchange of an op that
        # returns nothing leaves this PE's owner session open for the next such batch; flush()
        # applies it (LAMELLAR_EXCHANGE_DEFER=0: every exchange sweeps its own batch)
        self._xdeferred = None
        # a deferred session's owned batches are partitioned every this many batches (0: at the flush)
        self._partition_every = int(os.environ.get("LAMELLAR_DEFER_PARTITION_EVERY", "0"))
        if os.environ.get("LAMELLAR_EXCHANGE_DEFER", "1") != "0":
            check(self.lib.lmr_ctx_exchange_defer(self.ctx, 1), "lmr_ctx_exchange_defer")

    # ---------------------------------------------------------------- infra
    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def reserve(self, n: int):
        """Grow the tiled-apply workspace (allocation: call outside timed regions)."""
        n = min(int(n), self.max_ws_records)
        if n > self.reserved:
            self.flush()
            torch.cuda.synchronize(self.device)     # the workspace may be in use on any stream
            check(self.lib.lmr_ctx_reserve(self.ctx, n), "lmr_ctx_reserve")
            self.reserved = n

    def _maybe_reserve(self, n):
        if self.strategy != Strategy.Direct and n >= 65536 and self.reserved < min(n, self.max_ws_records):
            self.reserve(max(n, 1 << 20))

    def errors(self, clear=True) -> int:
        self.flush()
        bits = c_uint32(0)
        st = self.lib.lmr_ctx_error(self.ctx, self.stream(), byref(bits), 1 if clear else 0)
        if st == LmrStatus.HIP and not bits.value:
            # the stream or the error-word read failed: a runtime error, not a device error bit
            check(st, "lmr_ctx_error")
        return bits.value

    def check_errors(self):
        bits = self.errors(clear=True)
        if bits:
            st = errbits_to_status(bits)
            raise LamellarError(st, f"device error bits 0x{bits:x}")

    def profile(self, enable=True):
        """Record HIP events around every kernel stage (lmr_ctx_profile)."""
        check(self.lib.lmr_ctx_profile(self.ctx, 1 if enable else 0), "lmr_ctx_profile")

    def profile_read(self, reset=True):
        """{stage: (total_ms, launches, records)} accumulated since the last reset."""
        self.flush()
        n = len(_capi.STAGES)
        ms = (ctypes.c_double * n)()
        cnt = (c_uint64 * n)()
        rec = (c_uint64 * n)()
        check(self.lib.lmr_ctx_profile_read(self.ctx, self.stream(), ms, cnt, rec, 1 if reset else 0),
              "lmr_ctx_profile_read")
        return {name: (ms[i], cnt[i], rec[i]) for i, name in enumerate(_capi.STAGES)}

    def synchronize(self):
        self.flush()
        torch.cuda.current_stream(self.device).synchronize()

    # ---------------------------------------------------------------- deferred batches
    # The op-builder API's batches are asynchronous (the reference applies batches in
    # flight together in no particular order). Consecutive batches on one shard are staged
    # into one mixed session (lmr_stage_begin / lmr_stage_op / lmr_stage_soa) and applied
    # together, in issue order per element, by flush(): one shard sweep for many batches.
    # flush() runs before anything else touches the device state this context manages
    # (every other call here, synchronize, error reads, the arrays' local data).
    def defer_soa(self, shard, shard_len, kind, dt, op, idx, iw, vals, scalar_bits, n,
                  results=None, ok=None, cmp_bits=0, eps_bits=0, borrowed=False):
        """Stage n records for a later flush(); their results / Ok flags are valid after it.
        borrowed: idx / vals are the caller's own buffers, which it may change after this call
        returns -- the records are partitioned now (lmr_stage_flush, stream-ordered), so only
        the shard sweep waits for the flush."""
        key = (shard.data_ptr(), int(shard_len), int(kind), int(dt.code))
        if (self._deferred is not None and self._deferred[0] != key) or self._xdeferred is not None:
            self.flush()                      # (an open exchange session holds the context's session)
        if self.strategy != Strategy.Direct and n >= 65536 and self.reserved < min(n, self.max_ws_records):
            self.flush()                      # the workspace grows only with nothing staged
            self._maybe_reserve(n)
        opk = (int(op), int(cmp_bits), int(eps_bits))
        if self._deferred is None:
            d = self._desc(shard, shard_len, kind, dt, op, cmp_bits, eps_bits)
            check(self.lib.lmr_stage_begin(self.ctx, byref(d)), "lmr_stage_begin")
            self._deferred = [key, opk, []]
        elif self._deferred[1] != opk:
            check(self.lib.lmr_stage_op(self.ctx, opk[0], c_uint64(opk[1]), c_uint64(opk[2]), self.stream()),
                  "lmr_stage_op")
            self._deferred[1] = opk
        self._deferred[2].append((shard, idx, vals, results, ok))
        sv = c_uint64(int(scalar_bits) & 0xFFFFFFFFFFFFFFFF)
        st = self.lib.lmr_stage_soa(self.ctx, _p(idx), int(iw), _p(vals),
                                    None if vals is not None else ctypes.cast(byref(sv), c_void_p),
                                    int(n), _p(results), _p(ok), self.stream())
        if st:
            self._deferred = None
            self.lib.lmr_stage_finish(self.ctx, self.stream())
            check(st, "lmr_stage_soa")
        if borrowed or (self._partition_every and len(self._deferred[2]) % self._partition_every == 0):
            # borrowed inputs are partitioned now; owned ones every few batches, so the device
            # starts on a long session while the host stages its later batches
            check(self.lib.lmr_stage_flush(self.ctx, self.stream()), "lmr_stage_flush")

    def flush(self):
        """Apply the deferred batches (one sweep) on this stream."""
        self._flush_local()
        if self._xdeferred is not None:
            held = self._xdeferred
            self._xdeferred = None
            check(self.lib.lmr_exchange_flush(self.ctx, self.stream()), "lmr_exchange_flush")
            del held                          # released once the sweep is enqueued (stream-ordered reuse)

    def _flush_local(self):
        d = self._deferred
        if d is None:
            return
        self._deferred = None
        # the tensors in d[2] are released after the finish is enqueued: the caching allocator
        # reuses their memory only for work ordered after it on this stream
        check(self.lib.lmr_stage_finish(self.ctx, self.stream()), "lmr_stage_finish")

    def empty(self, n, torch_dtype):
        return torch.empty(max(int(n), 0), dtype=torch_dtype, device=self.device)

    def to_device(self, t):
        return t.to(self.device, non_blocking=False)

    # ---------------------------------------------------------------- ops
    def _desc(self, shard, shard_len, kind, dt, op, cmp_bits=0, eps_bits=0):
        d = _capi.lmr_apply_desc_t()
        d.shard = shard.data_ptr()
        d.shard_len = int(shard_len)
        d.kind = int(kind)
        d.dtype = int(dt.code)
        d.op = int(op)
        d.strategy = self.strategy
        d.cmp_bits = int(cmp_bits)
        d.eps_bits = int(eps_bits)
        return d

    def apply_soa(self, shard, shard_len, kind, dt, op, idx, iw, vals, scalar_bits, n,
                  results=None, ok=None, cmp_bits=0, eps_bits=0):
        """Apply n records (idx: iw-byte local offsets; vals tensor or scalar bits)."""
        self.flush()
        self._maybe_reserve(n)
        d = self._desc(shard, shard_len, kind, dt, op, cmp_bits, eps_bits)
        sv = c_uint64(int(scalar_bits) & 0xFFFFFFFFFFFFFFFF)
        st = self.lib.lmr_apply_soa(self.ctx, byref(d), _p(idx), int(iw), _p(vals),
                                    None if vals is not None else ctypes.cast(byref(sv), c_void_p),
                                    int(n), _p(results), _p(ok), self.stream())
        check(st, "lmr_apply_soa")

    # ---- staged apply (lmr_stage_*): the owner side of the multi-PE exchange
    def stage_begin(self, shard, shard_len, kind, dt, op, cmp_bits=0, eps_bits=0, expect=0):
        """Open a staged session for one op on one shard. `expect`: records the
        session will likely stage; the workspace grows to hold them now, before
        anything is staged (lmr_ctx_reserve is refused while records are staged)."""
        self.flush()
        if expect:
            self._maybe_reserve(int(expect))
        d = self._desc(shard, shard_len, kind, dt, op, cmp_bits, eps_bits)
        check(self.lib.lmr_stage_begin(self.ctx, byref(d)), "lmr_stage_begin")

    def stage_soa(self, idx, iw, vals, scalar_bits, n, results=None, ok=None):
        """Stage n records (lmr_apply_soa's arguments) into the session; their
        results / Ok flags are valid once stage_finish has run on this stream. The
        records are partitioned at the next stage_flush / stage_finish: the tensors are
        held until then."""
        self._staged_refs.append((idx, vals))
        sv = c_uint64(int(scalar_bits) & 0xFFFFFFFFFFFFFFFF)
        st = self.lib.lmr_stage_soa(self.ctx, _p(idx), int(iw), _p(vals),
                                    None if vals is not None else ctypes.cast(byref(sv), c_void_p),
                                    int(n), _p(results), _p(ok), self.stream())
        check(st, "lmr_stage_soa")

    def stage_op(self, op, cmp_bits=0, eps_bits=0):
        """Later stage_soa calls stage under `op` (a mixed session: op phases applied in
        staging order per element, lmr_stage_op)."""
        check(self.lib.lmr_stage_op(self.ctx, int(op), c_uint64(int(cmp_bits) & 0xFFFFFFFFFFFFFFFF),
                                    c_uint64(int(eps_bits) & 0xFFFFFFFFFFFFFFFF), self.stream()), "lmr_stage_op")

    def stage_flush(self):
        """Partition the staged records now (lmr_stage_flush)."""
        check(self.lib.lmr_stage_flush(self.ctx, self.stream()), "lmr_stage_flush")
        self._staged_refs = []

    def stage_finish(self):
        """Apply every staged record in one sweep of the shard and close the session."""
        check(self.lib.lmr_stage_finish(self.ctx, self.stream()), "lmr_stage_finish")
        self._staged_refs = []

    def apply_mvmi(self, shard, shard_len, kind, dt, op, idx_vals_bytes, nbytes, iw,
                   results=None, ok=None, cmp_bits=0, eps_bits=0):
        """Apply a reference wire-format op buffer (packed IdxVal<I,T> records)."""
        self.flush()
        self._maybe_reserve(nbytes // max(1, self.lib.lmr_record_bytes(iw, dt.code)))
        d = self._desc(shard, shard_len, kind, dt, op, cmp_bits, eps_bits)
        st = self.lib.lmr_apply_mvmi(self.ctx, byref(d), _p(idx_vals_bytes), int(nbytes), int(iw),
                                     _p(results), _p(ok), self.stream())
        check(st, "lmr_apply_mvmi")

    def apply_mvmi_host(self, shard, shard_len, kind, dt, op, h_records, iw, h_results=None, h_ok=None,
                        cmp_bits=0, eps_bits=0):
        """Apply a host-resident op buffer (numpy uint8 IdxVal<I,T> bytes); fetch results / Ok
        flags land in the host numpy arrays h_results / h_ok (lmr_apply_mvmi_host). Synchronous:
        returns when the host results are valid."""
        self.flush()
        d = self._desc(shard, shard_len, kind, dt, op, cmp_bits, eps_bits)
        st = self.lib.lmr_apply_mvmi_host(self.ctx, byref(d), h_records.ctypes.data, int(h_records.nbytes),
                                          int(iw), None if h_results is None else h_results.ctypes.data,
                                          None if h_ok is None else h_ok.ctypes.data, self.stream())
        check(st, "lmr_apply_mvmi_host")
        torch.cuda.current_stream(self.device).synchronize()

    def host_register(self, arr):
        """Record a host numpy buffer as an op / result buffer (lmr_host_register); zero-copy
        DMA needs host_alloc memory."""
        check(self.lib.lmr_host_register(arr.ctypes.data, int(arr.nbytes)), "lmr_host_register")

    def host_register_heap(self, arr):
        """Page-lock a host heap for its lifetime (lmr_host_register_heap): buffers inside it DMA in
        place. Unregister only at shutdown."""
        check(self.lib.lmr_host_register_heap(arr.ctypes.data, int(arr.nbytes)), "lmr_host_register_heap")

    def host_unregister_heap(self, arr):
        check(self.lib.lmr_host_unregister_heap(arr.ctypes.data), "lmr_host_unregister_heap")

    def host_unregister(self, arr):
        check(self.lib.lmr_host_unregister(arr.ctypes.data), "lmr_host_unregister")

    def host_registered(self, arr):
        """(0, 0, 1) when a registered range holds the buffer (the library locks no caller memory:
        its copies are staged through the bounce slots), else None (lmr_host_registered)."""
        base, nb, refs = c_uint64(0), c_uint64(0), c_uint32(0)
        st = self.lib.lmr_host_registered(arr.ctypes.data, int(arr.nbytes), byref(base), byref(nb), byref(refs))
        return (base.value, nb.value, refs.value) if st == 0 else None

    def host_alloc(self, nbytes, dtype=np.uint8):
        """A pinned host buffer (lmr_host_alloc) as a numpy array; release with host_free."""
        p = ctypes.c_void_p()
        check(self.lib.lmr_host_alloc(int(nbytes), byref(p)), "lmr_host_alloc")
        raw = (ctypes.c_uint8 * int(nbytes)).from_address(p.value)
        return np.frombuffer(raw, dtype=np.uint8).view(dtype)

    def host_free(self, arr):
        check(self.lib.lmr_host_free(arr.ctypes.data), "lmr_host_free")

    def apply_svmi(self, shard, shard_len, kind, dt, op, scalar_bits, indices, n, iw,
                   results=None, ok=None, cmp_bits=0, eps_bits=0):
        self.flush()
        self._maybe_reserve(n)
        d = self._desc(shard, shard_len, kind, dt, op, cmp_bits, eps_bits)
        sv = c_uint64(int(scalar_bits) & 0xFFFFFFFFFFFFFFFF)
        st = self.lib.lmr_apply_svmi(self.ctx, byref(d), ctypes.cast(byref(sv), c_void_p), _p(indices),
                                     int(n), int(iw), _p(results), _p(ok), self.stream())
        check(st, "lmr_apply_svmi")

    def apply_mvsi(self, shard, shard_len, kind, dt, op, vals, n, index, results=None, ok=None,
                   cmp_bits=0, eps_bits=0):
        self.flush()
        d = self._desc(shard, shard_len, kind, dt, op, cmp_bits, eps_bits)
        st = self.lib.lmr_apply_mvsi(self.ctx, byref(d), _p(vals), int(n), int(index), _p(results),
                                     _p(ok), self.stream())
        check(st, "lmr_apply_mvsi")

    def pack(self, layout, gidx, n, vals, dt, iw, stable=True, want_pos=True):
        """Partition by destination PE -> (idx, vals, pos, counts[int64 device]).
        stable=False: lmr_pack_unordered (no order inside a PE's range)."""
        self.flush()
        npes = layout.num_pes
        out_idx = self.empty(n * iw, torch.uint8)
        out_vals = self.empty(n * dt.bytes, torch.uint8) if vals is not None else None
        out_pos = self.empty(n, torch.int32) if want_pos else None
        counts = self.empty(npes, torch.int64)
        offsets = self.empty(npes + 1, torch.int64)
        fn = self.lib.lmr_pack if stable else self.lib.lmr_pack_unordered
        st = fn(self.ctx, byref(layout), _p(gidx), int(n), _p(vals), int(dt.code), int(iw),
                _p(out_idx), _p(out_vals), _p(out_pos), _p(counts), _p(offsets), self.stream())
        check(st, "lmr_pack" if stable else "lmr_pack_unordered")
        return out_idx, out_vals, out_pos, counts

    def pack_regions(self, layout, gidx, n, vals, dt, iw, cap):
        """lmr_pack_regions: count-free pack into fixed regions of `cap` records per PE
        -> (idx, vals, counts[int64 device]); a count above cap: that region overflowed."""
        self.flush()
        npes = layout.num_pes
        out_idx = self.empty(npes * cap * iw, torch.uint8)
        out_vals = self.empty(npes * cap * dt.bytes, torch.uint8) if vals is not None else None
        fill = self.empty(npes, torch.int32)
        counts = self.empty(npes, torch.int64)
        st = self.lib.lmr_pack_regions(self.ctx, byref(layout), _p(gidx), int(n), _p(vals), int(dt.code), int(iw),
                                       _p(out_idx), _p(out_vals), int(cap), _p(fill), _p(counts), self.stream())
        check(st, "lmr_pack_regions")
        return out_idx, out_vals, counts

    def reduce(self, data, n, dt, op):
        """lmr_reduce over n elements -> (has, value bits) (one 9-byte readback)."""
        self.flush()
        out = self.empty(2, torch.int64)
        has = out[1:].view(torch.uint8)[:1]
        st = self.lib.lmr_reduce(self.ctx, int(dt.code), int(op), _p(data), int(n), _p(out), _p(has),
                                 self.stream())
        check(st, "lmr_reduce")
        h = out.cpu()
        return bool(h[1].item() & 0xFF), int(h[0].item()) & 0xFFFFFFFFFFFFFFFF

    def batch_exchange(self, transport, layout, shard, shard_len, kind, dt, op, gidx, h_index, i_len, vals,
                       h_val_bits, v_len, results=None, ok=None, cmp_bits=0, eps_bits=0, expect=0):
        """lmr_batch_exchange: one batched op over every PE (collective). gidx: i_len
        global indices (device) unless i_len == 1 (h_index); vals: v_len elements
        (device) unless v_len == 1 (h_val_bits). `expect`: records this PE will likely
        receive; the workspace grows to hold them before the call. An op that returns nothing
        may leave its owner session open (deferred, applied by flush() or by the next exchange
        of another op); the next exchange of the same op on the same shard adds to it."""
        self._flush_local()
        key = (shard.data_ptr(), int(shard_len), int(kind), int(dt.code), int(op), int(cmp_bits), int(eps_bits))
        if self._xdeferred is not None and (self._xdeferred[0] != key or results is not None or ok is not None):
            self.flush()
        if expect:
            self._maybe_reserve(int(expect))
        d = self._desc(shard, shard_len, kind, dt, op, cmp_bits, eps_bits)
        hv = c_uint64(int(h_val_bits) & 0xFFFFFFFFFFFFFFFF)
        st = self.lib.lmr_batch_exchange(self.ctx, transport.ptr, byref(layout), byref(d), _p(gidx),
                                         int(h_index) & 0xFFFFFFFFFFFFFFFF, int(i_len), _p(vals),
                                         ctypes.cast(byref(hv), c_void_p), int(v_len), _p(results), _p(ok),
                                         self.stream())
        transport.raise_pending()
        if st != 0:
            self._xdeferred = None                # a failed exchange drops the open session
        check(st, "lmr_batch_exchange")
        # (the library keeps the session open only for a count-free owner session; flushing a
        # session it closed itself is a no-op)
        # the open session holds the shard: an array dropped before the flush keeps its memory until
        # the sweep has run, so no new array can take its address (and its key) meanwhile
        self._xdeferred = (key, shard) if results is None and ok is None else None

    def apply_msg(self, msg: bytes, resolve, shard_of, max_entries=1 << 16):
        """lmr_apply_msg over one lamellae message (single AM or batched) in host memory.
        resolve(am_id) -> (shape, kind, dtype code) of a registered op AM, the serialized
        body size (int) of another AM (a ReturnAm, a user AM: left to the runtime), or None
        (unknown: the message is refused); shard_of(view) -> (device tensor, shard_len,
        strategy) for a decoded AM, or None to skip it. Returns {entry index: reply bytes}
        for the returning AMs."""
        self.flush()
        errs = []

        def res_cb(_user, _cmd, am_id, _body, _avail, shape, kind, dtype, body_bytes):
            try:
                r = resolve(int(am_id))
            except Exception as e:  # noqa: BLE001 - reported after the C call
                errs.append(e)
                return 2
            if r is None:
                return 2
            if isinstance(r, int):
                body_bytes[0] = r
                return 1
            shape[0], kind[0], dtype[0] = (int(x) for x in r)
            return 0

        keep = []

        def shard_cb(_user, view, out):
            try:
                r = shard_of(view.contents)
            except Exception as e:  # noqa: BLE001
                errs.append(e)
                return 1
            if r is None:
                return 1
            t, slen, strategy = r
            keep.append(t)
            out[0].shard = t.data_ptr()
            out[0].shard_len = int(slen)
            out[0].strategy = int(strategy)
            return 0

        rfn, sfn = _capi.AM_RESOLVER_FN(res_cb), _capi.SHARD_RESOLVER_FN(shard_cb)
        raw = (ctypes.c_uint8 * max(len(msg), 1)).from_buffer_copy(msg if msg else b"\0")
        cap = 16 * len(msg) + 4096
        replies = (ctypes.c_uint8 * cap)()
        offs = (c_uint64 * max_entries)()
        lens = (c_uint64 * max_entries)()
        n = c_uint32()
        st = self.lib.lmr_apply_msg(self.ctx, raw, len(msg), rfn, sfn, None, replies, cap, offs, lens, max_entries,
                                    byref(n), self.stream())
        if errs:
            raise errs[0]
        check(st, "lmr_apply_msg")
        return {e: bytes(replies[int(offs[e]):int(offs[e]) + int(lens[e])]) for e in range(n.value) if lens[e]}

    def scatter_results(self, res_in, pos, n, eb, res_out, ok_in=None, ok_out=None):
        self.flush()
        st = self.lib.lmr_scatter_results(_p(res_in), _p(pos), int(n), int(eb), _p(res_out),
                                          _p(ok_in), _p(ok_out), self.stream())
        check(st, "lmr_scatter_results")
