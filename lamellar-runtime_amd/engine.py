"""Host orchestration of one batched element op (the body of the reference's
UnsafeArray::initiate_batch_op / initiate_batch_fetch_op_2 /
initiate_batch_result_op_2, src/array/unsafe/operations.rs:290-477).

1 PE (local lamellae): the reference never serialises (every AM takes the
`dst == src` shortcut, active_messaging/registered_active_message.rs:150-154),
so the records go straight to the apply kernel: at one PE a global index *is*
the local offset (Block, Cyclic and sub-arrays alike), bounds-checked on the
device.

N PEs (one per GPU): a collective step replaces the shmem lamellae:
  lmr_pack_unordered (device, grouped by destination PE, IndexSize-narrowed offsets)
  -> header all-to-all (per destination: count, MVSI index, scalar value)
  -> all-to-all-v of indices and values (RCCL over xGMI)
  -> apply of every received segment (device)
  -> [fetch / result ops] reverse all-to-all-v of results + lmr_scatter_results
     back into input order (operations/handle.rs:315-317).
The step is cut into chunks and software-pipelined over a pack stream, the
RCCL stream and an apply stream (_distributed).
Every PE must issue the same sequence of batch calls (a PE with nothing to
send passes an empty batch): the exchange is collective where the reference's
AMs are one-sided.
"""
from __future__ import annotations

import contextlib
import numbers
import os

import numpy as np
import torch

from .kernels import LamellarError
from .types import RET_KIND, BatchReturnType, DType, LmrStatus, op_supported


# Route 1-PE batches through the exchange step too (rehearses the RCCL calls of
# the multi-GPU path on a one-GPU box); off by default.
_FORCE_EXCHANGE = os.environ.get("LAMELLAR_FORCE_EXCHANGE", "0") == "1"


class BatchResult:
    """Results of a fetch / result batch: values (and Ok flags) in input order."""

    def __init__(self, vals, ok, dt: DType, ret):
        self.vals = vals     # torch tensor (storage dtype) or None
        self.ok = ok         # torch uint8 tensor (Result ops) or None
        self.dt = dt
        self.ret = ret

    def numpy(self):
        v = self.vals.cpu().numpy().view(self.dt.np) if self.vals is not None else None
        if self.ret == BatchReturnType.Result:
            return v, self.ok.cpu().numpy().astype(bool)
        return v

    def __len__(self):
        return 0 if self.vals is None else int(self.vals.numel())


def _is_scalar(x):
    return isinstance(x, (numbers.Number, np.generic)) or (isinstance(x, np.ndarray) and x.ndim == 0)


def index_input(k, x):
    """OpInput<usize>: scalar -> (True, int, 1); sequence -> (False, int64 tensor, len)."""
    if _is_scalar(x):
        return True, int(x), 1
    if isinstance(x, torch.Tensor):
        t = x.reshape(-1)
        if t.dtype != torch.int64:
            t = t.to(torch.int64)
        t = t.to(k.device) if t.device != k.device else t
        return False, t.contiguous(), int(t.numel())
    a = np.asarray(x)
    if a.size == 0:
        return False, k.empty(0, torch.int64), 0
    a = a.reshape(-1)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    else:
        a = a.astype(np.int64)
    return False, torch.from_numpy(np.ascontiguousarray(a)).to(k.device), int(a.size)


def value_input(k, dt: DType, x):
    """OpInput<T>: scalar -> (True, bits, 1); sequence -> (False, storage tensor, len)."""
    if _is_scalar(x):
        return True, dt.to_bits(x), 1
    if isinstance(x, torch.Tensor):
        t = x.reshape(-1)
        if t.dtype != dt.torch:
            if t.element_size() == dt.bytes and not t.is_floating_point() and not dt.is_float:
                t = t.view(dt.torch)          # same-width integer: reinterpret the bits
            else:
                t = _np_to_storage(t.cpu().numpy(), dt)
        t = t.to(k.device) if t.device != k.device else t
        return False, t.contiguous(), int(t.numel())
    a = np.asarray(x).reshape(-1)
    if a.size == 0:
        return False, k.empty(0, dt.torch), 0
    return False, _np_to_storage(a, dt).to(k.device), int(a.size)


_STORAGE_NP = {1: np.int8, 2: np.int16, 4: np.int32, 8: np.int64}


def _np_to_storage(a: np.ndarray, dt: DType) -> torch.Tensor:
    v = np.ascontiguousarray(a.astype(dt.np))
    if dt.is_float:
        return torch.from_numpy(v)
    if dt.torch_name == "uint8":
        return torch.from_numpy(v.view(np.uint8))
    return torch.from_numpy(v.view(_STORAGE_NP[dt.bytes]))


def run_batch(arr, op, index, val, current=None, eps=None) -> BatchResult:
    """Apply `op` for every (index, value) pair; returns results in input order."""
    team = arr.team
    k = team.kernels
    dt = arr.dtype
    if not op_supported(arr.kind, dt, op):
        raise LamellarError(LmrStatus.UNSUPPORTED, f"{op!r} on {type(arr).__name__}<{dt.name}>")
    ret = RET_KIND[op]
    cmp_bits = dt.to_bits(current) if current is not None else 0
    eps_bits = dt.to_bits(eps) if eps is not None else 0
    i_scalar, idx, i_len = index_input(k, index)
    v_scalar, vals, v_len = value_input(k, dt, val)
    if i_len == 0 or v_len == 0:                        # "no vals no indices" :345-347
        return BatchResult(k.empty(0, dt.torch) if ret else None,
                           k.empty(0, torch.uint8) if ret == BatchReturnType.Result else None, dt, ret)
    if i_len > 1 and v_len > 1 and i_len != v_len:
        raise LamellarError(LmrStatus.LENGTH, f"{i_len} indices vs {v_len} values")
    n = max(i_len, v_len)
    results = k.empty(n, dt.torch) if ret != BatchReturnType.None_ else None
    ok = k.empty(n, torch.uint8) if ret == BatchReturnType.Result else None
    mvsi = (i_len == 1 and v_len > 1)
    if team.num_pes() == 1 and not _FORCE_EXCHANGE:
        _local(arr, k, dt, op, i_scalar, idx, v_scalar, vals, n, mvsi, results, ok, cmp_bits, eps_bits)
    else:
        _distributed(arr, k, dt, op, ret, i_scalar, idx, v_scalar, vals, n, mvsi, results, ok,
                     cmp_bits, eps_bits)
    return BatchResult(results, ok, dt, ret)


def _host_map(arr, g):
    from . import _capi
    import ctypes
    pe, off = ctypes.c_uint64(0), ctypes.c_uint64(0)
    okm = _capi.lib().lmr_pe_and_offset(ctypes.byref(arr.layout), int(g) & 0xFFFFFFFFFFFFFFFF,
                                        ctypes.byref(pe), ctypes.byref(off))
    if not okm:
        raise LamellarError(LmrStatus.OOB, f"Index: {g} out of bounds for array of len: {arr.len()}")
    return pe.value, off.value


def _local(arr, k, dt, op, i_scalar, idx, v_scalar, vals, n, mvsi, results, ok, cmp_bits, eps_bits):
    shard, slen = arr.local_shard(), arr.num_elems_local()
    if mvsi:
        _, off = _host_map(arr, idx)
        k.apply_mvsi(shard, slen, arr.kind, dt, op, vals, n, off, results, ok, cmp_bits, eps_bits)
        return
    if i_scalar:
        idx = torch.tensor([idx], dtype=torch.int64, device=k.device)
    k.apply_soa(shard, slen, arr.kind, dt, op, idx, 8, None if v_scalar else vals,
                vals if v_scalar else 0, n, results, ok, cmp_bits, eps_bits)


def _exchange_chunk() -> int:
    """Records per exchange chunk (LAMELLAR_EXCHANGE_CHUNK, default 2^26), at most
    2^27 so one chunk's value bytes stay below 2^31 per peer."""
    return min(1 << 27, max(1, int(os.environ.get("LAMELLAR_EXCHANGE_CHUNK", str(1 << 26)))))


class _Streams:
    """Pack/exchange and apply streams of one batch on a device (no-ops on CPU)."""

    def __init__(self, k):
        self.dev = getattr(k, "is_device", True) and k.device.type == "cuda"
        if self.dev:
            self.main = torch.cuda.current_stream(k.device)
            self.pack = torch.cuda.Stream(k.device)
            self.apply = torch.cuda.Stream(k.device)
            self.pack.wait_stream(self.main)
            self.apply.wait_stream(self.main)

    def on(self, which):
        if not self.dev:
            return contextlib.nullcontext()
        return torch.cuda.stream(getattr(self, which))

    def used_on(self, which, *tensors):
        """Tell the caching allocator that `tensors` are read/written on stream `which`."""
        if self.dev:
            st = getattr(self, which)
            for t in tensors:
                if t is not None and t.is_cuda:
                    t.record_stream(st)

    def join(self):
        if self.dev:
            self.main.wait_stream(self.pack)
            self.main.wait_stream(self.apply)


def _distributed(arr, k, dt, op, ret, i_scalar, idx, v_scalar, vals, n, mvsi, results, ok,
                 cmp_bits, eps_bits):
    """Chunked, software-pipelined exchange.

    The batch is cut into chunks of LAMELLAR_EXCHANGE_CHUNK records. Per chunk j:
    pack (pack stream) -> header all-to-all (counts, MVSI index, scalar value)
    -> async all-to-all-v of indices and values (RCCL stream) -> the apply
    stream waits for the exchange and applies every source's records in one
    call. Chunk j's exchange overlaps chunk j+1's pack and chunk j-1's apply;
    returned values of chunk j travel back (async) after chunk j+1's exchange
    has been issued, then lmr_scatter_results puts them in input order.

    Owner side: every chunk's received records are partitioned into shard tiles
    on arrival (lmr_stage_soa) and all chunks are applied in one sweep of the
    shard after the last one (lmr_stage_finish), so the shard is read and
    written once per batch, not once per chunk. Returned values of every chunk
    travel back after that sweep.

    Collective: every PE issues the same sequence. PEs agree on the chunk count
    through the first header (column 4 = the sender's chunk count); a PE past
    its own last chunk sends empty chunks.
    """
    team = arr.team
    npes = team.num_pes()
    iw = arr.index_size()
    eb = dt.bytes
    returning = ret != BatchReturnType.None_
    st = _Streams(k)
    chunk = _exchange_chunk()
    if mvsi:
        my_k = 1
        mvsi_pe, mvsi_off = _host_map(arr, idx)
    else:
        if i_scalar:
            idx = torch.tensor([idx], dtype=torch.int64, device=k.device)
        m = int(idx.numel())
        my_k = max(1, -(-m // chunk))
    sbits = (vals & 0xFFFFFFFFFFFFFFFF) if (v_scalar and not mvsi) else 0
    shard, slen = arr.local_shard(), arr.num_elems_local()
    empty_u8 = k.empty(0, torch.uint8)
    # the owner expects about as many records as it sends (uniform streams); more
    # than the workspace holds only costs an extra shard sweep
    with st.on("apply"):
        k.stage_begin(shard, slen, arr.kind, dt, op, cmp_bits, eps_bits,
                      expect=0 if mvsi else (m + m // 8 + (1 << 16)))

    def pack_chunk(j):
        """-> (send_idx, send_vals, pos, counts (device or host), lo, hi)"""
        if mvsi:
            if j > 0:
                return empty_u8, empty_u8, None, torch.zeros(npes, dtype=torch.int64), 0, 0
            c = torch.zeros(npes, dtype=torch.int64)
            c[mvsi_pe] = n
            sv = vals.view(torch.uint8) if vals.dtype != torch.uint8 else vals
            return empty_u8, sv, None, c, 0, n
        lo, hi = min(m, j * chunk), min(m, (j + 1) * chunk)
        with st.on("pack"):
            si, sv, pos, counts = k.pack(arr.layout, idx[lo:hi], hi - lo,
                                         None if v_scalar else vals[lo:hi], dt, iw,
                                         stable=False, want_pos=returning)
        return si, (sv if sv is not None else empty_u8), pos, counts, lo, hi

    def send_back(p):
        """Reverse exchange of a chunk's returned values + scatter into input order."""
        r_res, r_ok, recv_counts, send_counts, pos, lo, hi = p
        with st.on("apply"):
            back, wb = team.alltoallv_async(r_res, [c * eb for c in recv_counts],
                                            [c * eb for c in send_counts], eb)
            back_ok, wo = (team.alltoallv_async(r_ok, recv_counts, send_counts)
                           if r_ok is not None else (None, None))
            wb.wait()
            if wo is not None:
                wo.wait()
            st.used_on("apply", back, back_ok, pos)
            nsent = int(sum(send_counts))
            if mvsi:
                results.view(torch.uint8)[:nsent * eb].copy_(back[:nsent * eb])
                if ok is not None:
                    ok[:nsent].copy_(back_ok[:nsent])
            elif nsent:
                k.scatter_results(back, pos, nsent, eb, results[lo:hi], back_ok,
                                  ok[lo:hi] if ok is not None else None)

    nchunks = my_k
    nxt = pack_chunk(0)
    pending = []
    j = 0
    while j < nchunks:
        send_idx, send_vals, pos, counts, lo, hi = nxt
        with st.on("pack"):
            send_counts = counts.cpu() if counts.is_cuda else counts      # waits for this pack only
        header = torch.zeros(npes, 5, dtype=torch.int64)
        header[:, 0] = send_counts
        header[:, 1] = -1
        if mvsi and j == 0:
            header[mvsi_pe, 1] = mvsi_off
        if v_scalar and not mvsi:
            header[:, 2] = 1
            header[:, 3] = torch.tensor(np.array([sbits], dtype=np.uint64).view(np.int64))
        header[:, 4] = my_k
        with st.on("pack"):
            rh = team.alltoall_header(header)
        if j == 0:
            nchunks = int(rh[:, 4].max())
        send_counts = header[:, 0].tolist()
        recv_counts = rh[:, 0].tolist()
        idx_ss = [c * iw if header[p, 1] < 0 else 0 for p, c in enumerate(send_counts)]
        idx_rs = [c * iw if rh[p, 1] < 0 else 0 for p, c in enumerate(recv_counts)]
        val_ss = [0 if header[p, 2] else c * eb for p, c in enumerate(send_counts)]
        val_rs = [0 if rh[p, 2] else c * eb for p, c in enumerate(recv_counts)]
        with st.on("pack"):
            r_idx, w_i = team.alltoallv_async(send_idx, idx_ss, idx_rs, iw)
            r_vals, w_v = team.alltoallv_async(send_vals, val_ss, val_rs, eb)
        # next chunk's pack runs while this chunk is on the wire
        nxt = pack_chunk(j + 1) if j + 1 < nchunks else None
        total = int(sum(recv_counts))
        with st.on("apply"):
            w_i.wait()
            w_v.wait()
            st.used_on("apply", r_idx, r_vals)
            r_res = k.empty(total * eb, torch.uint8) if returning else None
            r_ok = k.empty(total, torch.uint8) if ret == BatchReturnType.Result else None
            _apply_received(k, arr, dt, op, shard, slen, rh, recv_counts, iw, eb, r_idx, r_vals,
                            r_res, r_ok, cmp_bits, eps_bits)
        if returning:
            pending.append((r_res, r_ok, recv_counts, send_counts, pos, lo, hi))
        j += 1
    with st.on("apply"):
        k.stage_finish()
    for p in pending:
        send_back(p)
    st.join()


def _apply_received(k, arr, dt, op, shard, slen, rh, recv_counts, iw, eb, r_idx, r_vals, r_res, r_ok,
                    cmp_bits, eps_bits):
    """Stage one chunk's received records into the open session: consecutive
    sources with the same value form (array values / the same scalar) go in one
    call; MVSI sources are applied at once, one by one (their block is applied
    as one atomic unit)."""
    npes = len(recv_counts)
    io = vo = ro = 0
    s = 0
    while s < npes:
        c = int(recv_counts[s])
        if c == 0:
            s += 1
            continue
        if rh[s, 1] >= 0:
            k.apply_mvsi(shard, slen, arr.kind, dt, op, r_vals[vo:vo + c * eb], c, int(rh[s, 1]),
                         r_res[ro * eb:(ro + c) * eb] if r_res is not None else None,
                         r_ok[ro:ro + c] if r_ok is not None else None, cmp_bits, eps_bits)
            vo += c * eb
            ro += c
            s += 1
            continue
        scalar, bits = int(rh[s, 2]), int(rh[s, 3])
        e, cnt = s, 0
        while e < npes and (int(recv_counts[e]) == 0 or
                            (rh[e, 1] < 0 and int(rh[e, 2]) == scalar and (not scalar or int(rh[e, 3]) == bits))):
            cnt += int(recv_counts[e])
            e += 1
        seg_idx = r_idx[io:io + cnt * iw]
        seg_res = r_res[ro * eb:(ro + cnt) * eb] if r_res is not None else None
        seg_ok = r_ok[ro:ro + cnt] if r_ok is not None else None
        if scalar:
            ubits = int(np.array([bits], dtype=np.int64).view(np.uint64)[0])
            k.stage_soa(seg_idx, iw, None, ubits, cnt, seg_res, seg_ok)
        else:
            k.stage_soa(seg_idx, iw, r_vals[vo:vo + cnt * eb], 0, cnt, seg_res, seg_ok)
            vo += cnt * eb
        io += cnt * iw
        ro += cnt
        s = e
