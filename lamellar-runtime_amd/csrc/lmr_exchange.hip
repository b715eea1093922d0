// lmr_exchange.hip — the multi-PE exchange of one batched op behind the C ABI
// (lmr_batch_exchange), its transports (RCCL over xGMI; host-buffer callbacks),
// and the host planning it shares with the tests (lmr_exchange_plan).
//
// Replaces, for num_pes > 1, the trip of the reference's op AMs over a lamellae:
// the pack loops put records into per-destination buffers
// (src/array/unsafe/operations.rs:663-811), each full buffer becomes an AM sent with
// Shmem::send_to_pes_async (src/lamellae/shmem_lamellae.rs:168-186 ->
// command_queues.rs:725-807), the owner's recv_data loop (:1395-1531) hands it to
// exec_am (registered_active_message.rs:443-497), and fetch results come back as
// AM data (:307-359) into the handle's reorder (operations/handle.rs:315-317).
// Here, per chunk of the batch:
//   pack stream : pack by owner PE (count-free regions / lmr_pack_unordered; the stable
//                 lmr_pack for a batch that is one reference AM per destination) and the
//                 chunk's header rows (count, MVSI local index, flags, scalar bits, chunk
//                 count); chunk j+1's pack runs while the host waits for chunk j's headers
//   exchange    : header all-to-all -> [host reads the rows: RCCL's all-to-all-v takes
//                 host counts] -> all-to-all-v of local indices and values
//   apply stream: waits for the chunk's exchange, stages every source's records
//                 (lmr_stage_soa; MVSI sources lmr_apply_mvsi) -> after the last
//                 chunk one shard sweep (lmr_stage_finish) -> reverse all-to-all-v of
//                 each chunk's results -> lmr_scatter_results into input order.
// Chunk j's exchange overlaps chunk j-1's staging on the apply stream; receive
// buffers are double-buffered between the two streams.
// Ops whose records commute (add / sub / mul / and / or / xor, nothing returned) pack bucketed
// regions instead (lmr_bucket.hip): per owner, slices by owner bucket, sent whole, binned by the
// owner without a coarse pass; over the peer transport the pack writes them into the owners' HBM.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include <dlfcn.h>
#include <mutex>
#include <rccl/rccl.h>
#include "../../include/lamellar_gpu_ops.h"
#include "lmr_internal.hpp"
#include "lmr_device.hpp"

namespace lmr {

hipError_t xstate_drain(const XState* x);

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    // grow-only: a larger request first waits for the exchange's internal streams (the old
    // buffer may be in use there; the library uses these buffers on no other stream)
    hipError_t need(size_t bytes, const lmr::XState* owner) {
        if (bytes <= cap) return hipSuccess;
        if (p) {
            hipError_t e = xstate_drain(owner);
            if (e != hipSuccess) return e;
            (void)hipFree(p);
            p = nullptr;
            cap = 0;
        }
        size_t c = std::max<size_t>(bytes, 4096);
        c = c + c / 8;
        hipError_t e = hipMalloc(&p, c);
        if (e != hipSuccess) { p = nullptr; return e; }
        cap = c;
        return hipSuccess;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
    template <typename T> T* as() const { return reinterpret_cast<T*>(p); }
};

struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t need(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t c = std::max<size_t>(bytes, 4096);
        hipError_t e = hipHostMalloc(&p, c, hipHostMallocDefault);
        if (e != hipSuccess) { p = nullptr; return e; }
        cap = c;
        return hipSuccess;
    }
    void release() { if (p) (void)hipHostFree(p); p = nullptr; cap = 0; }
};

}  // namespace

// Exchange state of a context: internal streams, events, grow-only buffers.
// Streams: sp packs, sx runs every forward collective, sa stages and applies. Send buffers,
// header rows and receive buffers are double-buffered by chunk parity, so chunk j+1's pack
// runs while the host waits for chunk j's header rows, and chunk j+1's all-to-all-v
// overlaps chunk j's staging.
struct XState {
    hipStream_t sp = nullptr, sx = nullptr, sa = nullptr;
    hipStream_t sh = nullptr;            // header exchanges of split-header transports
    // the peer push's device-side waits, each on a high-priority stream of its own (so a wave
    // polling the mailbox holds no hardware queue the pack or the staging runs on); the pack and
    // apply streams wait for them through events
    hipStream_t sw_free = nullptr, sw_pub = nullptr;
    hipEvent_t ev_free_ok[2] = {nullptr, nullptr}, ev_pub_ok[2] = {nullptr, nullptr}, ev_marked[2] = {nullptr, nullptr};
    hipEvent_t ev_begin = nullptr, ev_pack_done = nullptr, ev_apply_done = nullptr, ev_x_done = nullptr,
               ev_h_done = nullptr;
    hipEvent_t ev_hdr[2] = {nullptr, nullptr}, ev_x[2] = {nullptr, nullptr};
    hipEvent_t ev_recv_free[2] = {nullptr, nullptr}, ev_send_free[2] = {nullptr, nullptr},
               ev_packed[2] = {nullptr, nullptr};
    bool recv_used[2] = {false, false}, send_used[2] = {false, false};
    DevBuf counts, offsets, one_idx, fill;
    DevBuf hdr_send[2], hdr_recv[2], send_idx[2], send_vals[2];
    DevBuf recv_idx[2], recv_vals[2];
    std::vector<DevBuf> pos, res, rok;   // per chunk (returning ops)
    DevBuf ovf_idx, ovf_vals, ovf_count;  // count-free pack: records past their region (global index, value)
    // the peer push's bucketed mode (lmr_bucket.hip): the sender's (owner, bucket) fill counters and
    // per-owner totals, the owner's session of fixed tile regions and its tile fills
    DevBuf bfill, btot, tfill;
    BucketSession bs;
    bool tfill_zero = false;             // tfill is zero as the apply stream will see it
    DevBuf back, back_ok;
    HostBuf h_hdr;                       // per chunk parity: [send rows | recv rows] int64
    HostBuf h_send, h_recv;              // host-buffer transports
    // waits for the three internal streams (not the whole device: other work may share it)
    hipError_t drain() const {
        hipError_t e = hipSuccess, r;
        for (hipStream_t s : {sp, sx, sa, sh, sw_free, sw_pub})
            if (s && (r = hipStreamSynchronize(s)) != hipSuccess && e == hipSuccess) e = r;
        return e;
    }
};

hipError_t xstate_drain(const XState* x) { return x->drain(); }

void xstate_free(XState* x) {
    if (!x) return;
    (void)x->drain();
    for (DevBuf* b : {&x->hdr_send[0], &x->hdr_send[1], &x->hdr_recv[0], &x->hdr_recv[1], &x->counts, &x->offsets,
                      &x->one_idx, &x->fill, &x->send_idx[0], &x->send_idx[1], &x->send_vals[0], &x->send_vals[1],
                      &x->recv_idx[0], &x->recv_idx[1], &x->recv_vals[0], &x->recv_vals[1], &x->back, &x->back_ok,
                      &x->ovf_idx, &x->ovf_vals, &x->ovf_count, &x->bfill, &x->btot, &x->tfill})
        b->release();
    for (auto* v : {&x->pos, &x->res, &x->rok})
        for (DevBuf& b : *v) b.release();
    x->h_hdr.release();
    x->h_send.release();
    x->h_recv.release();
    for (hipEvent_t e : {x->ev_begin, x->ev_pack_done, x->ev_apply_done, x->ev_x_done, x->ev_h_done, x->ev_hdr[0],
                         x->ev_hdr[1],
                         x->ev_x[0], x->ev_x[1], x->ev_recv_free[0], x->ev_recv_free[1], x->ev_send_free[0],
                         x->ev_send_free[1], x->ev_packed[0], x->ev_packed[1], x->ev_free_ok[0], x->ev_free_ok[1],
                         x->ev_pub_ok[0], x->ev_pub_ok[1], x->ev_marked[0], x->ev_marked[1]})
        if (e) (void)hipEventDestroy(e);
    if (x->sw_free) (void)hipStreamDestroy(x->sw_free);
    if (x->sw_pub) (void)hipStreamDestroy(x->sw_pub);
    if (x->sp) (void)hipStreamDestroy(x->sp);
    if (x->sx) (void)hipStreamDestroy(x->sx);
    if (x->sa) (void)hipStreamDestroy(x->sa);
    if (x->sh) (void)hipStreamDestroy(x->sh);
    delete x;
}

static hipError_t xstate_init(XState* x) {
    if (x->sp) return hipSuccess;
    hipError_t e = hipStreamCreateWithFlags(&x->sp, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&x->sx, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&x->sa, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&x->sh, hipStreamNonBlocking);
    for (hipEvent_t* ev : {&x->ev_begin, &x->ev_pack_done, &x->ev_apply_done, &x->ev_x_done, &x->ev_h_done,
                           &x->ev_hdr[0],
                           &x->ev_hdr[1], &x->ev_x[0], &x->ev_x[1], &x->ev_recv_free[0], &x->ev_recv_free[1],
                           &x->ev_send_free[0], &x->ev_send_free[1], &x->ev_packed[0], &x->ev_packed[1],
                           &x->ev_free_ok[0], &x->ev_free_ok[1], &x->ev_pub_ok[0], &x->ev_pub_ok[1], &x->ev_marked[0],
                           &x->ev_marked[1]})
        if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    return e;
}

// the peer push's wait streams, made on the first pushed batch only (a context that never
// pushes holds no extra hardware queue)
static hipError_t xstate_wait_streams(XState* x) {
    if (x->sw_pub) return hipSuccess;
    int lo_prio = 0, hi_prio = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio);
    if (e == hipSuccess && !x->sw_free) e = hipStreamCreateWithPriority(&x->sw_free, hipStreamNonBlocking, hi_prio);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&x->sw_pub, hipStreamNonBlocking, hi_prio);
    return e;
}

// per-PE header rows of one chunk: [count, MVSI local index or -1, flags (LMR_XHDR_*), scalar
// bits, chunk count, packed records of the batch, chunk size]
// ovf (may be null): the sender's overflow count so far; > 0 sets LMR_XHDR_OVERFLOW in every row
__global__ void k_xhdr(const uint64_t* counts, uint32_t npes, int64_t mvsi_pe, int64_t mvsi_off, int64_t mvsi_n,
                       int64_t flags, uint64_t sbits, int64_t my_k, int64_t m, int64_t chunk, int64_t* hdr,
                       const uint32_t* ovf) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npes) return;
    int64_t* r = hdr + uint64_t(p) * LMR_XHDR_WORDS;
    const bool mv = mvsi_pe >= 0 && int64_t(p) == mvsi_pe;
    r[0] = mvsi_pe >= 0 ? (mv ? mvsi_n : 0) : (counts ? int64_t(counts[p]) : 0);
    r[1] = mv ? mvsi_off : -1;
    r[2] = flags | ((ovf && *ovf) ? int64_t(LMR_XHDR_OVERFLOW) : int64_t(0));
    r[3] = int64_t(sbits);
    r[4] = my_k;
    r[5] = m;
    r[6] = chunk;
}

// batch start: the count-free pack's fill counters (and the bucketed pack's), and the overflow count
// (one launch instead of a memset per chunk; the packs leave their fill counters zero after each chunk)
__global__ void k_xbegin(uint32_t* fill, uint32_t nfill, uint32_t* bfill, uint32_t nbfill, uint32_t* ovf) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nfill) fill[i] = 0;
    if (i < nbfill) bfill[i] = 0;
    if (i < 2) ovf[i] = 0;
}

// the bucketed session's one tile sweep (nothing when none is open)
hipError_t bucket_sweep(lmr_ctx* ctx, XState* x, hipStream_t s) {
    if (!x->bs.open) return hipSuccess;
    TiledWs w = carve_tiled_ws(ctx->ws, ctx->rec_cap);
    w.side = SideLane{ctx->side, ctx->side_fork, ctx->side_join};
    const hipError_t e = launch_bucket_sweep(x->bs, w, s);   // (its plan kernel zeroes the tile fills)
    x->tfill_zero = e == hipSuccess;
    return e;
}

}  // namespace lmr

using namespace lmr;

namespace {

inline lmr_status_t hs(hipError_t e) { return e == hipSuccess ? LMR_OK : LMR_E_HIP; }

// LMR_XDEBUG=1: the exchange names the line of a failing HIP step on stderr (diagnostics only)
lmr_status_t xfail(int line) {
    static const bool dbg = getenv("LMR_XDEBUG") != nullptr;
    if (dbg) fprintf(stderr, "[lmr_exchange] HIP failure at lmr_exchange.hip:%d (%s)\n", line,
                     hipGetErrorString(hipGetLastError()));
    return LMR_E_HIP;
}

// Transport calls; host-buffer transports get pinned staging around the callback.
lmr_status_t tp_alltoall(const lmr_transport_t* tp, XState* x, const void* send, void* recv, uint64_t bytes,
                         hipStream_t s) {
    if (!tp->host_buffers) return tp->alltoall(tp->self, send, recv, bytes, reinterpret_cast<lmr_stream_t>(s));
    const size_t tot = size_t(bytes) * tp->num_pes;
    if (x->h_send.need(tot) != hipSuccess || x->h_recv.need(tot) != hipSuccess) return LMR_E_HIP;
    if (hipMemcpyAsync(x->h_send.p, send, tot, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return LMR_E_HIP;
    lmr_status_t st = tp->alltoall(tp->self, x->h_send.p, x->h_recv.p, bytes, reinterpret_cast<lmr_stream_t>(s));
    if (st != LMR_OK) return st;
    // (the staging is shared with calls on the other internal streams: nothing may still read it)
    if (hipMemcpyAsync(recv, x->h_recv.p, tot, hipMemcpyHostToDevice, s) != hipSuccess) return LMR_E_HIP;
    return hs(hipStreamSynchronize(s));
}

lmr_status_t tp_alltoallv(const lmr_transport_t* tp, XState* x, const void* send, const uint64_t* sb,
                          const uint64_t* so, void* recv, const uint64_t* rb, const uint64_t* ro, uint32_t unit,
                          hipStream_t s) {
    if (!tp->host_buffers)
        return tp->alltoallv(tp->self, send, sb, so, recv, rb, ro, unit, reinterpret_cast<lmr_stream_t>(s));
    // segments are packed back to back in the host staging on both sides (a count-free pack
    // leaves the send segments in fixed regions; a PE's own records leave a gap in the receive
    // layout): the callbacks see prefix offsets
    std::vector<uint64_t> cso(tp->num_pes), cro(tp->num_pes);
    uint64_t st_end = 0, rt_end = 0;
    bool rcontig = true;
    for (uint32_t p = 0; p < tp->num_pes; p++) {
        cso[p] = st_end;
        st_end += sb[p];
        cro[p] = rt_end;
        rcontig = rcontig && (rb[p] == 0 || ro[p] == rt_end);
        rt_end += rb[p];
    }
    if (x->h_send.need(st_end + 8) != hipSuccess || x->h_recv.need(rt_end + 8) != hipSuccess) return LMR_E_HIP;
    for (uint32_t p = 0; p < tp->num_pes; p++)
        if (sb[p] && hipMemcpyAsync(static_cast<uint8_t*>(x->h_send.p) + cso[p], static_cast<const uint8_t*>(send) + so[p],
                                    sb[p], hipMemcpyDeviceToHost, s) != hipSuccess)
            return LMR_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return LMR_E_HIP;
    lmr_status_t st = tp->alltoallv(tp->self, x->h_send.p, sb, cso.data(), x->h_recv.p, rb, cro.data(), unit,
                                    reinterpret_cast<lmr_stream_t>(s));
    if (st != LMR_OK) return st;
    if (rcontig) {
        if (rt_end && hipMemcpyAsync(static_cast<uint8_t*>(recv) + cro[0], x->h_recv.p, rt_end, hipMemcpyHostToDevice,
                                     s) != hipSuccess)
            return LMR_E_HIP;
    } else {
        for (uint32_t p = 0; p < tp->num_pes; p++)
            if (rb[p] && hipMemcpyAsync(static_cast<uint8_t*>(recv) + ro[p], static_cast<uint8_t*>(x->h_recv.p) + cro[p],
                                        rb[p], hipMemcpyHostToDevice, s) != hipSuccess)
                return LMR_E_HIP;
    }
    // (the staging is shared with calls on the other internal streams: nothing may still read it)
    return hs(hipStreamSynchronize(s));
}

// ---- the RCCL transport: grouped ncclSend / ncclRecv on the caller's stream.
// RCCL is bound at run time: a process that already loaded librccl (torch does) keeps
// that one copy, so the library and torch.distributed never hold two RCCL runtimes.
struct RcclApi {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclCommAbort) comm_abort = nullptr;
    decltype(&ncclCommSplit) comm_split = nullptr;   // optional: a header communicator
    bool ok = false;
};

const RcclApi& rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
        if (!h) return;
        api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
        api.comm_init_rank = reinterpret_cast<decltype(api.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
        api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        api.group_start = reinterpret_cast<decltype(api.group_start)>(dlsym(h, "ncclGroupStart"));
        api.group_end = reinterpret_cast<decltype(api.group_end)>(dlsym(h, "ncclGroupEnd"));
        api.send = reinterpret_cast<decltype(api.send)>(dlsym(h, "ncclSend"));
        api.recv = reinterpret_cast<decltype(api.recv)>(dlsym(h, "ncclRecv"));
        api.comm_abort = reinterpret_cast<decltype(api.comm_abort)>(dlsym(h, "ncclCommAbort"));
        api.comm_split = reinterpret_cast<decltype(api.comm_split)>(dlsym(h, "ncclCommSplit"));
        // ncclCommAbort is required: after a failed call it is the only way to end queued peer
        // send / recv kernels, so an RCCL without it is not used (the caller gets LMR_E_UNSUPPORTED)
        api.ok = api.get_unique_id && api.comm_init_rank && api.comm_destroy && api.group_start &&
                 api.group_end && api.send && api.recv && api.comm_abort;
    });
    return api;
}

struct RcclTransport {
    lmr_transport_t tp;
    ncclComm_t comm = nullptr;
    ncclComm_t hcomm = nullptr;   // header rows (split off comm): their own stream, no false
                                  // dependency on the previous chunk's records
    int device = 0;
};

ncclDataType_t nccl_type(uint32_t unit) {
    switch (unit) {
    case 8: return ncclUint64;
    case 4: return ncclUint32;
    default: return ncclUint8;
    }
}

// A failed ncclSend / ncclRecv inside the group still ends the group (RCCL requires the
// ncclGroupEnd), and the call reports the first failure.
lmr_status_t rccl_alltoall(void* self, const void* send, void* recv, uint64_t bytes, lmr_stream_t stream) {
    RcclTransport* t = static_cast<RcclTransport*>(self);
    if (!t->comm) return LMR_E_HIP;                  // aborted after an earlier failure
    ncclComm_t comm = t->hcomm ? t->hcomm : t->comm;
    const uint32_t unit = (bytes % 8 == 0) ? 8 : (bytes % 4 == 0 ? 4 : 1);
    const size_t cnt = size_t(bytes / unit);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const RcclApi& R = rccl();
    if (R.group_start() != ncclSuccess) return LMR_E_HIP;
    bool ok = true;
    for (uint32_t p = 0; p < t->tp.num_pes && ok; p++) {
        ok = R.send(static_cast<const uint8_t*>(send) + uint64_t(p) * bytes, cnt, nccl_type(unit), int(p), comm, s) ==
                 ncclSuccess &&
             R.recv(static_cast<uint8_t*>(recv) + uint64_t(p) * bytes, cnt, nccl_type(unit), int(p), comm, s) ==
                 ncclSuccess;
    }
    return (R.group_end() == ncclSuccess && ok) ? LMR_OK : LMR_E_HIP;
}

lmr_status_t rccl_alltoallv(void* self, const void* send, const uint64_t* sb, const uint64_t* so, void* recv,
                            const uint64_t* rb, const uint64_t* ro, uint32_t unit, lmr_stream_t stream) {
    RcclTransport* t = static_cast<RcclTransport*>(self);
    if (!t->comm) return LMR_E_HIP;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const ncclDataType_t ty = nccl_type(unit == 2 ? 1 : unit);
    const uint32_t u = (unit == 8 || unit == 4) ? unit : 1;
    const RcclApi& R = rccl();
    if (R.group_start() != ncclSuccess) return LMR_E_HIP;
    bool ok = true;
    for (uint32_t p = 0; p < t->tp.num_pes && ok; p++) {
        if (sb[p]) ok = R.send(static_cast<const uint8_t*>(send) + so[p], size_t(sb[p] / u), ty, int(p), t->comm, s) ==
                        ncclSuccess;
        if (ok && rb[p]) ok = R.recv(static_cast<uint8_t*>(recv) + ro[p], size_t(rb[p] / u), ty, int(p), t->comm, s) ==
                              ncclSuccess;
    }
    return (R.group_end() == ncclSuccess && ok) ? LMR_OK : LMR_E_HIP;
}

// After a transport failure the peers may never post their halves of the queued send / recv
// pairs, so waiting for the device could block forever: an RCCL transport aborts its
// communicator first (ncclCommAbort ends the queued RCCL kernels; the transport then refuses
// every later call and the job must make a new one). A host-buffer transport's failure leaves
// only local copies on the device.
void transport_abort(const lmr_transport_t* tp) {
    if (!tp || tp->alltoall != rccl_alltoall) return;
    RcclTransport* t = static_cast<RcclTransport*>(tp->self);
    if (t->hcomm) rccl().comm_abort(t->hcomm);
    if (t->comm) rccl().comm_abort(t->comm);
    t->comm = t->hcomm = nullptr;
}

bool valid_layout(const lmr_layout_t* L) {
    return L && L->num_pes > 0 && L->my_pe < L->num_pes && L->distribution <= 1 && L->orig_elem_per_pe > 0;
}

// the peer push's bucketed mode (on by default; LAMELLAR_EXCHANGE_BUCKETS=0 turns it off -- a PE
// that turns it off makes every PE's handshake fall back to the plain push). One-rank peer
// rehearsal (C4): 5.30-5.37 ms plain push, 4.52 ms bucketed (profiles/r6/c4_buckets/)
bool bucket_mode_enabled() {
    const char* e = getenv("LAMELLAR_EXCHANGE_BUCKETS");
    return !(e && e[0] == '0');
}

bool free_pack_enabled() {
    const char* e = getenv("LAMELLAR_FREE_PACK");
    return !(e && e[0] == '0');
}

// A PE's records for itself skip the transport (dst == src bypasses RCCL): staged
// straight from the send buffer, results copied back on the device. LAMELLAR_EXCHANGE_SELF=
// transport sends them through the transport like any other (a 1-PE rehearsal always does, so
// it makes the RCCL calls of the multi-GPU run).
bool self_bypass_enabled() {
    const char* e = getenv("LAMELLAR_EXCHANGE_SELF");
    return !(e && e[0] == 't');
}

// fixed-region mode (LAMELLAR_EXCHANGE_FIXED=0 turns it off; every PE must set it alike): whole
// fixed regions on the wire, device-side counts at the owner, no host read of later chunks' rows
bool fixed_mode_enabled() {
    const char* e = getenv("LAMELLAR_EXCHANGE_FIXED");
    return !(e && e[0] == '0');
}

uint64_t exchange_chunk() {
    const char* e = getenv("LAMELLAR_EXCHANGE_CHUNK");
    uint64_t c = (e && *e) ? strtoull(e, nullptr, 10) : (uint64_t(1) << 26);
    if (c < 1) c = 1;
    if (c > (uint64_t(1) << 27)) c = uint64_t(1) << 27;
    return c;
}

// elements of one all-to-all-v element unit that divide every split of a buffer of
// `w`-byte items (splits are item multiples)
uint32_t unit_for(uint32_t w) { return (w % 8 == 0) ? 8 : (w % 4 == 0 ? 4 : 1); }

}  // namespace

uint64_t lmr::exchange_chunk_records() { return exchange_chunk(); }

extern "C" {

uint64_t lmr_exchange_plan(uint32_t npes, uint32_t iw, uint32_t eb, const int64_t* sh, const int64_t* rh,
                           uint64_t* idx_sb, uint64_t* idx_so, uint64_t* idx_rb, uint64_t* idx_ro,
                           uint64_t* val_sb, uint64_t* val_so, uint64_t* val_rb, uint64_t* val_ro) {
    uint64_t k = 0, a = 0, b = 0, c = 0, d = 0;
    for (uint32_t p = 0; p < npes; p++) {
        const int64_t* s = sh + uint64_t(p) * LMR_XHDR_WORDS;
        const int64_t* r = rh + uint64_t(p) * LMR_XHDR_WORDS;
        const uint64_t sc = uint64_t(s[0] > 0 ? s[0] : 0), rc = uint64_t(r[0] > 0 ? r[0] : 0);
        idx_sb[p] = s[1] < 0 ? sc * iw : 0;            // MVSI senders name their index in the header
        idx_rb[p] = r[1] < 0 ? rc * iw : 0;
        val_sb[p] = (s[2] & LMR_XHDR_SCALAR) ? 0 : sc * eb;   // one scalar value travels in the header
        val_rb[p] = (r[2] & LMR_XHDR_SCALAR) ? 0 : rc * eb;
        idx_so[p] = a; a += idx_sb[p];
        idx_ro[p] = b; b += idx_rb[p];
        val_so[p] = c; c += val_sb[p];
        val_ro[p] = d; d += val_rb[p];
        if (r[4] > 0 && uint64_t(r[4]) > k) k = uint64_t(r[4]);
    }
    return k;
}

lmr_status_t lmr_rccl_unique_id(uint8_t id[128]) {
    if (!id) return LMR_E_INVALID;
    if (!rccl().ok) return LMR_E_UNSUPPORTED;
    ncclUniqueId u;
    if (rccl().get_unique_id(&u) != ncclSuccess) return LMR_E_HIP;
    static_assert(sizeof(u) == 128, "ncclUniqueId is 128 bytes");
    memcpy(id, &u, 128);
    return LMR_OK;
}

lmr_status_t lmr_transport_rccl_create(const uint8_t id[128], uint32_t num_pes, uint32_t my_pe, int device,
                                       lmr_transport_t** out) {
    if (!id || !out || num_pes == 0 || my_pe >= num_pes) return LMR_E_INVALID;
    *out = nullptr;
    if (!rccl().ok) return LMR_E_UNSUPPORTED;
    if (hipSetDevice(device) != hipSuccess) return LMR_E_HIP;
    RcclTransport* t = new RcclTransport();
    ncclUniqueId u;
    memcpy(&u, id, 128);
    if (rccl().comm_init_rank(&t->comm, int(num_pes), u, int(my_pe)) != ncclSuccess) {
        delete t;
        return LMR_E_HIP;
    }
    t->device = device;
    // the header communicator (collective like the init; without ncclCommSplit, if the split
    // fails, or with LMR_SPLIT_HEADERS=0 -- which every rank must set alike -- headers share the
    // data communicator and its stream). The two communicators' collectives run on two streams
    // and may start in a different order on different ranks; that cannot deadlock as long as
    // both RCCL kernels are co-resident on every GPU (each takes a few CUs of 256: a header
    // all-to-all is one channel), which is what the split assumes.
    static const bool split = [] { const char* v = getenv("LMR_SPLIT_HEADERS"); return !(v && v[0] == '0'); }();
    if (split && rccl().comm_split && rccl().comm_split(t->comm, 0, int(my_pe), &t->hcomm, nullptr) != ncclSuccess)
        t->hcomm = nullptr;
    t->tp.num_pes = num_pes;
    t->tp.my_pe = my_pe;
    t->tp.host_buffers = 0;
    t->tp.flags = t->hcomm ? LMR_TRANSPORT_SPLIT_HEADERS : 0u;
    t->tp.self = t;
    t->tp.alltoall = rccl_alltoall;
    t->tp.alltoallv = rccl_alltoallv;
    *out = &t->tp;
    return LMR_OK;
}

lmr_status_t lmr_transport_rccl_destroy(lmr_transport_t* tp) {
    if (!tp || tp->alltoall != rccl_alltoall) return LMR_E_INVALID;
    RcclTransport* t = static_cast<RcclTransport*>(tp->self);
    (void)hipSetDevice(t->device);
    (void)hipDeviceSynchronize();
    if (t->hcomm) rccl().comm_destroy(t->hcomm);
    if (t->comm) rccl().comm_destroy(t->comm);       // (an aborted communicator is already gone)
    delete t;
    return LMR_OK;
}

lmr_status_t lmr_batch_exchange(lmr_ctx_t* ctx, const lmr_transport_t* tp, const lmr_layout_t* layout,
                                const lmr_apply_desc_t* desc, const uint64_t* d_gidx, uint64_t h_index,
                                uint64_t i_len, const void* d_vals, const void* h_val, uint64_t v_len,
                                void* d_results, uint8_t* d_ok, lmr_stream_t stream) {
    if (!ctx || !tp || !valid_layout(layout) || !desc || tp->num_pes != layout->num_pes ||
        tp->my_pe != layout->my_pe || layout->num_pes > uint32_t(kMaxPackPes))
        return LMR_E_INVALID;
    if (desc->dtype >= LMR_NUM_DTYPES || desc->op >= LMR_NUM_OPS || desc->strategy > LMR_STRATEGY_ORDERED)
        return LMR_E_INVALID;
    if (!lmr_op_supported(desc->kind, desc->dtype, desc->op)) return LMR_E_UNSUPPORTED;
    if (i_len > 1 && v_len > 1 && i_len != v_len) return LMR_E_LENGTH;
    if ((i_len > 1 && !d_gidx) || (v_len > 1 && !d_vals) || (v_len == 1 && !h_val)) return LMR_E_INVALID;
    const uint32_t npes = layout->num_pes;
    const uint32_t eb = uint32_t(dtype_bytes(int(desc->dtype)));
    const uint32_t iw = lmr_index_size(layout);
    const uint32_t rk = lmr_op_ret_kind(desc->op);
    // every PE of a returning op sends results back, even one whose own batch is empty
    const bool returning = rk != LMR_RET_NONE;
    const bool want_ok = rk == LMR_RET_RESULT;
    const uint64_t n = (i_len == 0 || v_len == 0) ? 0 : std::max(i_len, v_len);
    if (n > 0 && ((returning && !d_results) || (want_ok && !d_ok))) return LMR_E_INVALID;
    const bool mvsi = i_len == 1 && v_len > 1;
    const bool scalar = v_len == 1 && !mvsi;
    uint64_t sbits = 0;
    if (scalar) memcpy(&sbits, h_val, eb);
    // A batch that is one reference AM per destination keeps its input order per owner: in the
    // reference a batch below 1000 records is one OpInput chunk (src/array/operations.rs:462-469),
    // so its pack appends each destination's records in input order into one buffer
    // (unsafe/operations.rs:709-758) and the owner's AM applies them sequentially
    // (impl/src/array_ops.rs:203-250; own records through the local shortcut,
    // registered_active_message.rs:150-154). Such a sender packs stably and flags its header
    // rows; the owner applies each flagged source's stream in order (LMR_STRATEGY_ORDERED).
    // LMR_STRATEGY_ORDERED asks for the same at any size.
    const bool ordered = !mvsi && n > 0 &&
                         (desc->strategy == LMR_STRATEGY_ORDERED ||
                          (desc->strategy == LMR_STRATEGY_AUTO && n < kOrderedAuto));
    (void)hipSetDevice(ctx->device);
    if (!ctx->xch) ctx->xch = new XState();
    XState* x = ctx->xch;
    if (xstate_init(x) != hipSuccess) return xfail(__LINE__);
    hipStream_t s0 = reinterpret_cast<hipStream_t>(stream);
    // --- shape on the sender side
    int64_t mvsi_pe = -1, mvsi_off = 0;
    const uint64_t* gidx = d_gidx;
    const uint64_t m = mvsi ? 0 : n;                   // records that go through the pack
    if (mvsi) {
        uint64_t pe = 0, off = 0;
        if (!lmr_pe_and_offset(layout, h_index, &pe, &off)) return LMR_E_OOB;   // unsafe/operations.rs:611-613
        mvsi_pe = int64_t(pe);
        mvsi_off = int64_t(off);
    } else if (n > 0 && i_len == 1) {                  // one index (1 x 1): a one-record batch
        if (x->one_idx.need(8, x) != hipSuccess) return xfail(__LINE__);
        if (hipMemcpyAsync(x->one_idx.p, &h_index, 8, hipMemcpyHostToDevice, s0) != hipSuccess) return xfail(__LINE__);
        gidx = x->one_idx.as<uint64_t>();
    }
    const uint64_t chunk = exchange_chunk();
    const uint64_t my_k = mvsi ? 1 : std::max<uint64_t>(1, (m + chunk - 1) / chunk);
    // --- buffers that do not depend on the chunk
    const size_t rows = size_t(npes) * LMR_XHDR_WORDS;
    for (int b = 0; b < 2; b++)
        if (x->hdr_send[b].need(rows * 8, x) != hipSuccess || x->hdr_recv[b].need(rows * 8, x) != hipSuccess)
            return xfail(__LINE__);
    if (x->counts.need(size_t(npes) * 8, x) != hipSuccess || x->offsets.need(size_t(npes + 1) * 8, x) != hipSuccess ||
        x->h_hdr.need(4 * rows * 8) != hipSuccess)
        return xfail(__LINE__);
    const uint64_t cmax = std::min<uint64_t>(m, chunk);
    // nothing returned: the count-free pack (fixed per-destination regions, no count pass);
    // records past a destination's region go to an overflow list, exchanged after the last chunk
    const bool free_pack = !returning && !ordered && !mvsi && npes <= 512 && free_pack_enabled();
    const uint32_t me = layout->my_pe;
    const bool bypass = npes > 1 && self_bypass_enabled();
    auto region_cap = [&](uint64_t c) -> uint64_t {
        const uint64_t q = (c + npes - 1) / npes;
        return q + q / 8 + 4096;
    };
    // a sender's region capacity for its chunk j (records m, chunk size ch): 0 past its last chunk
    auto cap_of = [&](uint64_t mm, uint64_t ch, uint64_t j) -> uint64_t {
        if (ch == 0 || j * ch >= mm) return 0;
        return region_cap(std::min(ch, mm - j * ch));
    };
    const uint64_t send_recs = free_pack ? std::max<uint64_t>(cmax, uint64_t(npes) * region_cap(cmax)) : cmax;
    if (free_pack && (send_recs > 0xFFFFFFFFull || x->fill.need(size_t(npes) * 4 + 8, x) != hipSuccess))
        return xfail(__LINE__);
    if (free_pack && (x->ovf_idx.need(m * 8 + 16, x) != hipSuccess ||
                      x->ovf_vals.need((scalar ? 0 : m * eb) + 16, x) != hipSuccess ||
                      x->ovf_count.need(16, x) != hipSuccess))
        return xfail(__LINE__);
    for (int b = 0; b < 2; b++)
        if (x->send_idx[b].need(send_recs * iw + 8, x) != hipSuccess ||
            x->send_vals[b].need(send_recs * eb + 8, x) != hipSuccess)
            return xfail(__LINE__);
    // --- the internal streams start after everything already on the caller's stream
    if (hipEventRecord(x->ev_begin, s0) != hipSuccess || hipStreamWaitEvent(x->sp, x->ev_begin, 0) != hipSuccess ||
        hipStreamWaitEvent(x->sx, x->ev_begin, 0) != hipSuccess || hipStreamWaitEvent(x->sa, x->ev_begin, 0) != hipSuccess ||
        hipStreamWaitEvent(x->sh, x->ev_begin, 0) != hipSuccess)
        return xfail(__LINE__);
    // header rows on their own stream when the transport allows it (LMR_TRANSPORT_SPLIT_HEADERS;
    // host-buffer transports are host-ordered): chunk j+1's header exchange is posted before
    // chunk j's all-to-all-v and waits only for chunk j+1's pack, so the host's per-chunk read
    // of the counts overlaps the previous chunk's records in flight
    const bool split = tp->host_buffers || (tp->flags & LMR_TRANSPORT_SPLIT_HEADERS);
    hipStream_t const shd = split ? x->sh : x->sx;
    x->recv_used[0] = x->recv_used[1] = false;
    x->send_used[0] = x->send_used[1] = false;
    // a deferred exchange session left open by an earlier call: this batch adds to it when it is
    // the same op on the same shard and stages count-free; otherwise it is applied first
    lmr_status_t st = LMR_OK;
    bool cont = false;
    const bool was_open = ctx->xdefer_open && (stage_session_open(ctx) || x->bs.open);
    ctx->xdefer_open = false;                   // (the staged-session calls refuse while it is set)
    if (was_open) {
        cont = !returning && !ordered && stage_session_free(ctx) && stage_session_of(ctx, *desc);
        if (!cont) {
            if (bucket_sweep(ctx, x, x->sa) != hipSuccess) return xfail(__LINE__);
            if (stage_session_open(ctx) && (st = lmr_stage_finish(ctx, reinterpret_cast<lmr_stream_t>(x->sa))) != LMR_OK)
                return st;
        }
    }
    if (!cont && (st = lmr_stage_begin(ctx, desc)) != LMR_OK) return st;
    // fixed-region mode: a FIXED sender's regions go whole to DEVCOUNT receivers (their count-free
    // session stages each region with its record count read on the device from the header rows),
    // so when every PE is both the host reads no header after chunk 0
    const bool devcount = fixed_mode_enabled() && !returning && !ordered && stage_session_free(ctx);
    const int64_t my_flags = (scalar ? LMR_XHDR_SCALAR : 0) | (ordered ? LMR_XHDR_ORDERED : 0) |
                             (free_pack ? LMR_XHDR_FIXED : 0) | (devcount ? LMR_XHDR_DEVCOUNT : 0);
    // the peer push's bucketed mode, as far as this PE can take it: the layout's buckets fit the
    // pack's keys, a bucket slice of the receive region holds this PE's chunk with headroom, and the
    // workspace holds the owner's tile regions
    PeerTransport* peer = peer_of(tp);
    uint32_t bC = 0, bcap = 0;
    int bshift = 0;
    bool my_bucket = false;
    if (peer && free_pack && devcount && bucket_mode_enabled() && ctx->ws && ctx->rec_cap > 0 && npes <= kBucketMaxSrc &&
        desc->shard_len > 0 && bucket_geometry(*layout, int(desc->dtype), bC, bshift)) {
        bcap = bucket_slice_cap(peer_region_records(peer), bC, eb);
        const uint64_t per = (cmax + uint64_t(npes) * bC - 1) / (uint64_t(npes) * bC);
        const int ts = tile_shift(int(desc->dtype));
        const uint64_t my_tiles = (desc->shard_len + (uint64_t(1) << ts) - 1) >> ts;
        my_bucket = bcap > 0 && uint64_t(bcap) >= per + per / 16 + 256 &&
                    my_tiles <= (uint64_t(bC) << bucket_tpb_log2());
    }
    if (my_bucket && (x->bfill.need(size_t(npes) * bC * 4 + 8, x) != hipSuccess ||
                      x->btot.need(size_t(npes) * 4 + 8, x) != hipSuccess))
        return xfail(__LINE__);
    if (my_bucket && !x->tfill.p) {
        if (x->tfill.need(size_t(kMaxTiles) * 4 + 8, x) != hipSuccess) return xfail(__LINE__);
        x->tfill_zero = false;
    }
    // a failed exchange closes the session (its staged records are dropped) so the context
    // stays usable; the work already enqueued on the internal streams drains first (after a
    // transport failure the transport is aborted first: peers may never post their halves)
    struct SessionGuard {
        lmr_ctx_t* c;
        const lmr_transport_t* t;
        bool armed = true;
        bool tp_failed = false;
        ~SessionGuard() {
            if (!armed) return;
            if (tp_failed) transport_abort(t);
            (void)c->xch->drain();
            stage_abort(c->stage);
            c->xch->bs.open = false;               // (its tile fills are zeroed before the next session)
            c->xch->bs.staged = 0;
            c->xch->tfill_zero = false;
        }
    } guard{ctx, tp};
    struct ChunkRec {
        std::vector<uint64_t> send_cnt, recv_cnt;
        uint64_t lo, hi, total;
    };
    std::vector<ChunkRec> chunks;
    std::vector<uint64_t> isb(npes), iso(npes), irb(npes), iro(npes), vsb(npes), vso(npes), vrb(npes), vro(npes);
    auto h_send_rows = [&](int b) { return static_cast<const int64_t*>(x->h_hdr.p) + size_t(b) * 2 * rows; };
    auto h_recv_rows = [&](int b) { return h_send_rows(b) + rows; };
    auto chunk_lo = [&](uint64_t j) { return std::min(m, j * chunk); };
    auto chunk_hi = [&](uint64_t j) { return std::min(m, (j + 1) * chunk); };
    // ---- local part of chunk j (pack stream): pack by destination PE into send buffer j&1
    // and write the chunk's header rows. No collective here, so chunk j+1's pack is enqueued
    // before the host waits for chunk j's header exchange and runs while it waits.
    auto counted_pack = [&](uint64_t j) -> lmr_status_t {
        const int b = int(j & 1);
        const uint64_t lo = chunk_lo(j), cnt = chunk_hi(j) - lo;
        const uint8_t* v = scalar ? nullptr : static_cast<const uint8_t*>(d_vals) + lo * eb;
        uint32_t* pos = returning ? x->pos[j].as<uint32_t>() : nullptr;
        return (ordered ? lmr_pack : lmr_pack_unordered)(
            ctx, layout, gidx + lo, cnt, v, desc->dtype, iw, x->send_idx[b].p, scalar ? nullptr : x->send_vals[b].p, pos,
            x->counts.as<uint64_t>(), x->offsets.as<uint64_t>(), reinterpret_cast<lmr_stream_t>(x->sp));
    };
    // send buffer b and its header rows: chunk j-2's all-to-all-v (and, for own records staged
    // from the send buffer or counted from the header rows, chunk j-2's staging) are done with them
    auto wait_send_slot = [&](int b) -> lmr_status_t {
        if (x->send_used[b] && hipStreamWaitEvent(x->sp, x->ev_send_free[b], 0) != hipSuccess) return xfail(__LINE__);
        if (x->recv_used[b] && hipStreamWaitEvent(x->sp, x->ev_recv_free[b], 0) != hipSuccess) return xfail(__LINE__);
        return LMR_OK;
    };
    // the collective exchange's bucketed regions (rb): the push's layout -- per owner a header of
    // slice counts, then C slices of bucket offsets -- in the send buffer, sent whole by the
    // transport, binned by the owner without a coarse pass. Decided from inputs every PE has alike
    // (the environment, the layout, the op), so every FIXED sender packs them or none does.
    bool rb = false;
    uint32_t rC = 0;
    int rshift = 0;
    // slice capacity of a sender's chunk j (records m, chunk size ch): 0 past its last chunk
    auto rcb_of = [&](uint64_t mm, uint64_t ch, uint64_t j) -> uint32_t {
        if (ch == 0 || j * ch >= mm || rC == 0) return 0;
        const uint64_t c = std::min(ch, mm - j * ch);
        const uint64_t per = (c + uint64_t(npes) * rC - 1) / (uint64_t(npes) * rC);
        // 1/16 + 256 records of headroom (the regions travel whole: headroom is wire bytes); a
        // uniform stream's slices hold ~2^17-2^20 records, whose spread is far below that, and
        // what a skewed one puts past a slice takes the overflow round
        return uint32_t(per + per / 16 + 256);
    };
    auto pack_chunk = [&](uint64_t j) -> lmr_status_t {
        const uint64_t lo = chunk_lo(j), cnt = chunk_hi(j) - lo;
        const int b = int(j & 1);
        const bool packed = !mvsi && j < my_k && cnt > 0;
        lmr_status_t e = wait_send_slot(b);
        if (e != LMR_OK) return e;
        if (returning && x->pos.size() <= j) x->pos.resize(j + 1);
        if (packed) {
            if (returning && x->pos[j].need(cnt * 4 + 8, x) != hipSuccess) return xfail(__LINE__);
            if (rb) {
                // fixed regions laid out by owner bucket, back to back in send buffer b (sent whole)
                PackArgs pa;
                pa.layout = *layout;
                pa.gidx = gidx + lo;
                pa.vals = scalar ? nullptr : static_cast<const uint8_t*>(d_vals) + lo * eb;
                pa.val_bytes = eb;
                pa.n = cnt;
                pa.index_size = iw;
                pa.out_idx = x->send_idx[b].as<uint8_t>();
                pa.out_vals = scalar ? nullptr : x->send_vals[b].as<uint8_t>();
                pa.out_pos = nullptr;
                pa.dest_counts = nullptr;
                pa.dest_offsets = nullptr;
                pa.err = ctx->d_err;
                pa.prof = ctx->prof;
                pa.stable = false;
                pa.ovf_gidx = x->ovf_idx.as<uint64_t>();
                pa.ovf_vals = scalar ? nullptr : x->ovf_vals.as<uint8_t>();
                pa.ovf_count = x->ovf_count.as<uint32_t>();
                pa.ovf_cap = m;
                if (launch_pack_bucket(pa, rC, rshift, rcb_of(m, chunk, j), x->bfill.as<uint32_t>(),
                                       x->btot.as<uint32_t>(), x->sp) != hipSuccess)
                    return xfail(__LINE__);
            } else if (free_pack) {
                PackArgs pa;
                pa.layout = *layout;
                pa.gidx = gidx + lo;
                pa.vals = scalar ? nullptr : static_cast<const uint8_t*>(d_vals) + lo * eb;
                pa.val_bytes = eb;
                pa.n = cnt;
                pa.index_size = iw;
                pa.out_idx = x->send_idx[b].as<uint8_t>();
                pa.out_vals = scalar ? nullptr : x->send_vals[b].as<uint8_t>();
                pa.out_pos = nullptr;
                pa.dest_counts = x->counts.as<uint64_t>();
                pa.dest_offsets = nullptr;
                pa.err = ctx->d_err;
                pa.prof = ctx->prof;
                pa.stable = false;
                pa.ovf_gidx = x->ovf_idx.as<uint64_t>();
                pa.ovf_vals = scalar ? nullptr : x->ovf_vals.as<uint8_t>();
                pa.ovf_count = x->ovf_count.as<uint32_t>();
                pa.ovf_cap = m;
                pa.fill_zeroed = true;                  // (k_xbegin, then each chunk's counts kernel)
                if (launch_pack_free(pa, x->fill.as<uint32_t>(), uint32_t(region_cap(cnt)), x->sp) != hipSuccess)
                    return xfail(__LINE__);
            } else {
                e = counted_pack(j);
                if (e != LMR_OK) return e;
            }
        }
        // (bucketed regions: no counts in the rows, the slice counts travel in each region's header)
        hipLaunchKernelGGL(k_xhdr, dim3((npes + 255) / 256), dim3(256), 0, x->sp,
                           packed && !rb ? x->counts.as<uint64_t>() : nullptr, npes, mvsi && j == 0 ? mvsi_pe : -1,
                           mvsi_off, int64_t(n), my_flags | (rb ? int64_t(LMR_XHDR_BUCKETS) : 0), sbits, int64_t(my_k),
                           int64_t(m), int64_t(chunk), x->hdr_send[b].as<int64_t>(),
                           free_pack ? x->ovf_count.as<uint32_t>() : nullptr);
        if (hipGetLastError() != hipSuccess) return xfail(__LINE__);
        return hipEventRecord(x->ev_packed[b], x->sp) == hipSuccess ? LMR_OK : LMR_E_HIP;
    };
    uint64_t packed_upto = 0;                          // chunks [0, packed_upto) are enqueued on sp
    auto pack_until = [&](uint64_t upto) -> lmr_status_t {
        while (packed_upto < upto) {
            const lmr_status_t e = pack_chunk(packed_upto);
            if (e != LMR_OK) return e;
            packed_upto++;
        }
        return LMR_OK;
    };
    // ---- the header all-to-all of chunk j (header stream) and its rows to the host. Receive
    // rows b are read on the device by chunk j-2's staging of fixed regions: that is done first.
    // `to_host`: the rows are copied to pinned host memory for the host to read (chunk 0, every
    // chunk the host plans from, and the last chunk, whose flags decide the overflow round); with
    // no host read they stay on the device (fixed-region mode: two copies per chunk saved)
    auto post_header = [&](uint64_t j, bool to_host) -> lmr_status_t {
        const int b = int(j & 1);
        if (hipStreamWaitEvent(shd, x->ev_packed[b], 0) != hipSuccess) return xfail(__LINE__);
        if (x->recv_used[b] && hipStreamWaitEvent(shd, x->ev_recv_free[b], 0) != hipSuccess) return xfail(__LINE__);
        lmr_status_t e = tp_alltoall(tp, x, x->hdr_send[b].p, x->hdr_recv[b].p, LMR_XHDR_WORDS * 8, shd);
        if (e != LMR_OK) { guard.tp_failed = true; return e; }
        int64_t* hs_ = const_cast<int64_t*>(h_send_rows(b));
        if (to_host && (hipMemcpyAsync(hs_, x->hdr_send[b].p, rows * 8, hipMemcpyDeviceToHost, shd) != hipSuccess ||
                        hipMemcpyAsync(hs_ + rows, x->hdr_recv[b].p, rows * 8, hipMemcpyDeviceToHost, shd) != hipSuccess))
            return xfail(__LINE__);
        return hipEventRecord(x->ev_hdr[b], shd) == hipSuccess ? LMR_OK : LMR_E_HIP;
    };
    // ---- owner side with host counts (apply stream): stage every source's records of receive
    // buffer b (counts cnt[p]; own records from send buffer b at the given offsets when bypassed)
    bool bucketed = false;                       // (the peer push's bucketed mode, agreed at the handshake)
    bool bsess = false;                          // (this batch's owner records go to the bucketed session)
    auto stage_host = [&](int b, const int64_t* h_recv, const std::vector<uint64_t>& cnt, uint64_t self_io,
                          uint64_t self_vo, const uint8_t* send_vals, uint64_t j) -> lmr_status_t {
        uint64_t io = 0, vo = 0, ro = 0;
        lmr_stream_t sa = reinterpret_cast<lmr_stream_t>(x->sa);
        lmr_status_t e;
        for (uint32_t p = 0; p < npes;) {
            const int64_t* r = h_recv + uint64_t(p) * LMR_XHDR_WORDS;
            const uint64_t c = cnt[p];
            if (c == 0) { p++; continue; }
            void* res = returning ? x->res[j].as<uint8_t>() + ro * eb : nullptr;
            uint8_t* okp = want_ok ? x->rok[j].as<uint8_t>() + ro : nullptr;
            const bool own = bypass && p == me;         // this PE's own records: from the send buffer
            const uint8_t* src_i = own ? x->send_idx[b].as<uint8_t>() + self_io : x->recv_idx[b].as<uint8_t>() + iro[p];
            const uint8_t* src_v = own ? send_vals + self_vo : x->recv_vals[b].as<uint8_t>() + vro[p];
            if (r[1] >= 0) {                            // MVSI: one atomic block at its index
                lmr_apply_desc_t d = *desc;
                e = lmr_apply_mvsi(ctx, &d, src_v, c, uint64_t(r[1]), res, okp, sa);
                if (e != LMR_OK) return e;
                ro += c;
                p++;
                continue;
            }
            // consecutive sources with the same value form and order flag, adjacent in the
            // receive buffer, go in one stream (an ordered stream of several sources keeps each
            // source's records in its order)
            const int64_t fl = r[2] & (LMR_XHDR_SCALAR | LMR_XHDR_ORDERED), bits = r[3];
            const bool sc = (fl & LMR_XHDR_SCALAR) != 0, ord = (fl & LMR_XHDR_ORDERED) != 0;
            uint32_t q = p;
            uint64_t tot = 0;
            while (q < npes) {
                const int64_t* w = h_recv + uint64_t(q) * LMR_XHDR_WORDS;
                if (cnt[q] == 0) { q++; continue; }
                if (w[1] >= 0 || (w[2] & (LMR_XHDR_SCALAR | LMR_XHDR_ORDERED)) != fl || (sc && w[3] != bits)) break;
                if (bypass && (q == me) != own) break;  // own records are a stream of their own
                if (!own && q != p && iro[q] != iro[p] + tot * iw) break;   // not adjacent (clamped regions)
                tot += cnt[q];
                q++;
                if (own) break;
            }
            const uint64_t ubits = uint64_t(bits);
            if (ord || bsess || rb) {
                // applied now: an ordered stream each element's records in stream order; in the
                // bucketed modes (the overflow round: order-insensitive records, whose workspace
                // holds the session's tile regions, or an owner without one) with device atomics
                lmr_apply_desc_t d = *desc;
                d.strategy = ord ? LMR_STRATEGY_ORDERED : LMR_STRATEGY_DIRECT;
                e = lmr_apply_soa(ctx, &d, src_i, iw, sc ? nullptr : src_v, sc ? &ubits : nullptr, tot, res, okp, sa);
            } else {
                e = lmr_stage_soa(ctx, src_i, iw, sc ? nullptr : src_v, sc ? &ubits : nullptr, tot, res, okp, sa);
            }
            if (e != LMR_OK) return e;
            ro += tot;
            p = q;
        }
        (void)io; (void)vo;
        return LMR_OK;
    };
    uint64_t nchunks = 1;
    bool nowait = false, any_fixed = false;
    std::vector<int64_t> src_m(npes), src_ch(npes), src_fl(npes), src_bits(npes);
    // ---- the peer transport's push: one host handshake per batch; if every PE packs and stages
    // fixed regions that fit the receive regions, every sender's pack writes straight into the
    // owners' regions (lmr_peer.hip) and nothing else crosses between the PEs but the mailbox
    bool push = false;
    const int64_t my_binfo = my_bucket ? int64_t((uint64_t(bC) << 32) | bcap) : 0;
    if (peer) {
        std::vector<int64_t> pi;
        const int64_t fits = (!free_pack || region_cap(cmax) <= peer_region_records(peer)) ? 1 : 0;
        const int64_t info[8] = {my_flags, int64_t(m), int64_t(chunk), int64_t(my_k), int64_t(sbits), fits, my_binfo,
                                 my_bucket ? int64_t(bshift) : 0};
        if ((st = peer_handshake(peer, info, pi)) != LMR_OK) return st == LMR_E_HIP ? xfail(__LINE__) : st;
        push = iw <= 8 && eb <= 8;
        for (uint32_t p = 0; p < npes; p++) {
            const int64_t* r = pi.data() + size_t(p) * 8;
            push = push && (r[0] & LMR_XHDR_FIXED) && (r[0] & LMR_XHDR_DEVCOUNT) && r[5];
            src_fl[p] = r[0];
            src_m[p] = r[1];
            src_ch[p] = r[2];
            src_bits[p] = r[4];
            nchunks = std::max<uint64_t>(nchunks, uint64_t(std::max<int64_t>(r[3], 1)));
        }
        bucketed = push && my_binfo != 0;
        for (uint32_t p = 0; p < npes; p++)
            bucketed = bucketed && pi[size_t(p) * 8 + 6] == my_binfo && pi[size_t(p) * 8 + 7] == int64_t(bshift);
    }
    rb = !push && free_pack && fixed_mode_enabled() && bucket_mode_enabled() &&
         bucket_op_ok(int(desc->dtype), int(desc->op)) && npes <= kBucketMaxSrc &&
         bucket_geometry(*layout, int(desc->dtype), rC, rshift);
    if (!rb) rC = 0;
    // this PE binds bucketed regions into a session when it has the workspace for one (else each
    // chunk's slices are applied with device atomics, launch_bucket_direct)
    const int ts_ = tile_shift(int(desc->dtype));
    const uint64_t my_tiles_ = (desc->shard_len + (uint64_t(1) << ts_) - 1) >> ts_;
    const bool owner_ok = rb && ctx->ws && ctx->rec_cap > 0 && my_tiles_ > 0 &&
                          my_tiles_ <= (uint64_t(rC) << bucket_tpb_log2());
    bsess = bucketed || owner_ok;
    const uint32_t uC = bucketed ? bC : rC;
    if (rb) {
        const uint32_t cb0 = rcb_of(m, chunk, 0);
        for (int b = 0; b < 2; b++)
            if (x->send_idx[b].need(size_t(npes) * bucket_region_idx_bytes(rC, cb0) + 8, x) != hipSuccess ||
                x->send_vals[b].need(size_t(npes) * rC * cb0 * eb + 8, x) != hipSuccess)
                return xfail(__LINE__);
        if (x->bfill.need(size_t(npes) * rC * 4 + 8, x) != hipSuccess || x->btot.need(size_t(npes) * 4 + 8, x) != hipSuccess)
            return xfail(__LINE__);
    }
    if (owner_ok && !x->tfill.p) {
        if (x->tfill.need(size_t(kMaxTiles) * 4 + 8, x) != hipSuccess) return xfail(__LINE__);
        x->tfill_zero = false;
    }
    if (free_pack) {   // (the pack's fill counters and the overflow count: zero at batch start)
        const uint32_t nb = bucketed ? npes * bC : (rb ? npes * rC : 0u), nt = std::max(npes, nb);
        hipLaunchKernelGGL(k_xbegin, dim3((nt + 255) / 256), dim3(256), 0, x->sp, x->fill.as<uint32_t>(), npes,
                           x->bfill.as<uint32_t>(), nb, x->ovf_count.as<uint32_t>());
        if (hipGetLastError() != hipSuccess) return xfail(__LINE__);
    }
    // the bucketed session and the staged one both keep records in the workspace's temp arrays:
    // whichever this batch does not use is applied first
    if (!bsess && bucket_sweep(ctx, x, x->sa) != hipSuccess) return xfail(__LINE__);
    if (bsess && !stage_session_empty(ctx)) {
        if ((st = lmr_stage_finish(ctx, reinterpret_cast<lmr_stream_t>(x->sa))) != LMR_OK) return st;
        if ((st = lmr_stage_begin(ctx, desc)) != LMR_OK) return st;
    }
    auto bucket_open = [&]() -> bool {
        BucketSession& bs = x->bs;
        if (bs.open) return true;
        const int ts = tile_shift(int(desc->dtype));
        const TiledWs w = carve_tiled_ws(ctx->ws, ctx->rec_cap);
        bs.desc = *desc;
        bs.C = uC;
        bs.tpb_log2 = bucket_tpb_log2();
        bs.T = uint32_t((desc->shard_len + (uint64_t(1) << ts) - 1) >> ts);
        bs.cap_t = std::min<uint64_t>(w.tmp_cap, 0xFFFFFFFFull) / bs.T;
        bs.staged = 0;
        bs.tfill = x->tfill.as<uint32_t>();
        bs.err = ctx->d_err;
        bs.prof = ctx->prof;
        if (!x->tfill_zero && hipMemsetAsync(bs.tfill, 0, size_t(bs.T) * 4, x->sa) != hipSuccess) return false;
        x->tfill_zero = true;
        bs.open = true;
        return true;
    };
    if (push) {
        if (xstate_wait_streams(x) != hipSuccess) return xfail(__LINE__);
        any_fixed = true;
        uint32_t* fill = x->fill.as<uint32_t>();
        for (uint64_t j = 0; j < nchunks; j++) {
            const int b = int(j & 1);
            const uint64_t seq = peer_chunk_seq(peer, j);
            // sender (pack stream): every owner has consumed this parity's region, then the pack
            // writes each owner's runs into it and the counts are published
            if (hipStreamWaitEvent(x->sw_free, x->ev_begin, 0) != hipSuccess ||
                peer_wait_freed(peer, b, ctx->d_err, x->sw_free) != hipSuccess ||
                hipEventRecord(x->ev_free_ok[b], x->sw_free) != hipSuccess ||
                hipStreamWaitEvent(x->sp, x->ev_free_ok[b], 0) != hipSuccess)
                return xfail(__LINE__);
            const uint64_t lo = chunk_lo(j), cnt = chunk_hi(j) - lo;
            if (j < my_k && cnt > 0) {
                PackArgs pa;
                pa.layout = *layout;
                pa.gidx = gidx + lo;
                pa.vals = scalar ? nullptr : static_cast<const uint8_t*>(d_vals) + lo * eb;
                pa.val_bytes = eb;
                pa.n = cnt;
                pa.index_size = iw;
                pa.out_idx = nullptr;
                pa.out_vals = nullptr;
                pa.out_pos = nullptr;
                pa.dest_counts = x->counts.as<uint64_t>();
                pa.dest_offsets = nullptr;
                pa.err = ctx->d_err;
                pa.prof = ctx->prof;
                pa.stable = false;
                pa.ovf_gidx = x->ovf_idx.as<uint64_t>();
                pa.ovf_vals = scalar ? nullptr : x->ovf_vals.as<uint8_t>();
                pa.ovf_count = x->ovf_count.as<uint32_t>();
                pa.ovf_cap = m;
                pa.out_idx_tab = peer_idx_table(peer, b);
                pa.out_vals_tab = scalar ? nullptr : peer_vals_table(peer, b);
                if (bucketed) {
                    if (launch_pack_bucket(pa, bC, bshift, bcap, x->bfill.as<uint32_t>(), x->btot.as<uint32_t>(), x->sp) !=
                        hipSuccess)
                        return xfail(__LINE__);
                } else if (launch_pack_free(pa, fill, uint32_t(region_cap(cnt)), x->sp) != hipSuccess) {
                    return xfail(__LINE__);
                }
                if (peer_publish(peer, b, bucketed ? x->btot.as<uint32_t>() : fill, seq, x->sp) != hipSuccess)
                    return xfail(__LINE__);
            } else if (peer_publish(peer, b, nullptr, seq, x->sp) != hipSuccess) {   // (nothing this chunk)
                return xfail(__LINE__);
            }
            // owner (apply stream): every source has published, each region staged with its count
            if (hipStreamWaitEvent(x->sw_pub, x->ev_begin, 0) != hipSuccess ||
                peer_wait_published(peer, b, seq, ctx->d_err, x->sw_pub) != hipSuccess ||
                hipEventRecord(x->ev_pub_ok[b], x->sw_pub) != hipSuccess ||
                hipStreamWaitEvent(x->sa, x->ev_pub_ok[b], 0) != hipSuccess)
                return xfail(__LINE__);
            if (bucketed) {
                // every source's bucket slices binned into the session's tile regions in one launch
                BucketChunk c;
                c.S = npes;
                for (uint32_t p = 0; p < npes; p++) {
                    const uint64_t cap = cap_of(uint64_t(std::max<int64_t>(src_m[p], 0)),
                                                uint64_t(std::max<int64_t>(src_ch[p], 0)), j);
                    if (cap == 0) continue;
                    const bool sc = (src_fl[p] & LMR_XHDR_SCALAR) != 0;
                    const uint64_t ch = uint64_t(std::max<int64_t>(src_ch[p], 1));
                    c.idx[p] = peer_recv_idx(peer, p, b);
                    c.val[p] = sc ? nullptr : peer_recv_vals(peer, p, b);
                    c.sbits[p] = uint64_t(src_bits[p]);
                    c.cap_b[p] = bcap;
                    c.expect += (std::min(ch, uint64_t(std::max<int64_t>(src_m[p], 0))) + npes - 1) / npes;
                }
                if (c.expect > 0) {
                    if (x->bs.open && x->bs.staged + c.expect > bucket_session_limit(x->bs) &&
                        bucket_sweep(ctx, x, x->sa) != hipSuccess)
                        return xfail(__LINE__);
                    if (!bucket_open()) return xfail(__LINE__);
                    TiledWs w = carve_tiled_ws(ctx->ws, ctx->rec_cap);
                    if (launch_fine_bucket(c, x->bs, w, x->sa) != hipSuccess) return xfail(__LINE__);
                    x->bs.staged += c.expect;
                }
                if (peer_mark_free(peer, b, seq, x->sa) != hipSuccess) return xfail(__LINE__);
                continue;
            }
            for (uint32_t p = 0; p < npes; p++) {
                const uint64_t cap = cap_of(uint64_t(std::max<int64_t>(src_m[p], 0)),
                                            uint64_t(std::max<int64_t>(src_ch[p], 0)), j);
                if (cap == 0) continue;
                const bool sc = (src_fl[p] & LMR_XHDR_SCALAR) != 0;
                const uint64_t ch = uint64_t(std::max<int64_t>(src_ch[p], 1));
                const uint64_t expect = (std::min(ch, uint64_t(std::max<int64_t>(src_m[p], 0))) + npes - 1) / npes;
                const uint64_t ubits = uint64_t(src_bits[p]);
                st = stage_soa_dev(ctx, peer_recv_idx(peer, p, b), iw, sc ? nullptr : peer_recv_vals(peer, p, b),
                                   sc ? &ubits : nullptr, cap, expect, peer_recv_count(peer, p, b), x->sa);
                if (st != LMR_OK) return st;
            }
            if ((st = lmr_stage_flush(ctx, reinterpret_cast<lmr_stream_t>(x->sa))) != LMR_OK) return st;
            if (peer_mark_free(peer, b, seq, x->sa) != hipSuccess) return xfail(__LINE__);
        }
    } else {
    // chunk 0: pack, header exchange; chunk 1's pack (local work) runs during the wait
    if ((st = pack_until(1)) != LMR_OK) return st;
    if ((st = post_header(0, true)) != LMR_OK) return st;
    if ((st = pack_until(std::min<uint64_t>(my_k, 2))) != LMR_OK) return st;
    nchunks = 1;
    for (uint64_t j = 0; j < nchunks; j++) {
        const int b = int(j & 1);
        const int64_t* h_send = h_send_rows(b);
        const int64_t* h_recv = h_recv_rows(b);
        if (j == 0 || !nowait) {
            // ---- the host reads chunk j's header rows (RCCL's send / recv counts are host
            // arguments); meanwhile the pack stream runs chunk j+1's pack and the apply stream
            // chunk j-1's staging
            if (hipEventSynchronize(x->ev_hdr[b]) != hipSuccess) return xfail(__LINE__);
            const uint64_t k = lmr_exchange_plan(npes, iw, eb, h_send, h_recv, isb.data(), iso.data(), irb.data(),
                                                 iro.data(), vsb.data(), vso.data(), vrb.data(), vro.data());
            if (j == 0) {
                nchunks = std::max<uint64_t>(k, 1);
                nowait = true;
                for (uint32_t p = 0; p < npes; p++) {
                    const int64_t* r = h_recv + uint64_t(p) * LMR_XHDR_WORDS;
                    src_fl[p] = r[2];
                    src_bits[p] = r[3];
                    src_m[p] = r[5];
                    src_ch[p] = r[6];
                    any_fixed = any_fixed || (r[2] & LMR_XHDR_FIXED);
                    // (bucketed regions need no device counts: every PE takes them, session or not)
                    nowait = nowait && (r[2] & LMR_XHDR_FIXED) && (r[2] & (LMR_XHDR_DEVCOUNT | LMR_XHDR_BUCKETS));
                    // every FIXED sender packs bucketed regions or none does (the same inputs on every
                    // PE, LAMELLAR_EXCHANGE_BUCKETS included): anything else is a configuration error
                    if ((r[2] & LMR_XHDR_FIXED) && bool(r[2] & LMR_XHDR_BUCKETS) != rb) return LMR_E_INVALID;
                }
            }
        }
        if (split && j + 1 < nchunks) {                 // the next header before this chunk's records
            if ((st = pack_until(j + 2)) != LMR_OK) return st;
            if ((st = post_header(j + 1, !nowait || j + 2 == nchunks)) != LMR_OK) return st;
        }
        const uint64_t lo = chunk_lo(j), hi = chunk_hi(j);
        const uint64_t my_cap = free_pack ? cap_of(m, chunk, j) : 0;
        std::vector<uint64_t> capr(npes, 0), cnt(npes, 0);
        for (uint32_t p = 0; p < npes; p++)
            if (src_fl[p] & LMR_XHDR_FIXED) capr[p] = cap_of(uint64_t(std::max<int64_t>(src_m[p], 0)),
                                                          uint64_t(std::max<int64_t>(src_ch[p], 0)), j);
        // bucketed regions: whole, index area header + C slices of u32, values C slices
        const uint32_t my_cb = rb ? rcb_of(m, chunk, j) : 0;
        std::vector<uint32_t> rcb(npes, 0);
        for (uint32_t p = 0; p < npes; p++)
            if (src_fl[p] & LMR_XHDR_BUCKETS)
                rcb[p] = rcb_of(uint64_t(std::max<int64_t>(src_m[p], 0)), uint64_t(std::max<int64_t>(src_ch[p], 0)), j);
        const uint64_t my_rib = my_cb ? bucket_region_idx_bytes(rC, my_cb) : 0, my_rvb = uint64_t(rC) * my_cb * eb;
        auto send_bucketed = [&](uint32_t p) {          // this PE's whole region for PE p
            isb[p] = my_rib;
            iso[p] = uint64_t(p) * my_rib;
            vsb[p] = scalar ? 0 : my_rvb;
            vso[p] = scalar ? 0 : uint64_t(p) * my_rvb;
        };
        auto recv_bucketed = [&](uint32_t p) {          // PE p's whole region for this PE
            irb[p] = rcb[p] ? bucket_region_idx_bytes(rC, rcb[p]) : 0;
            vrb[p] = (src_fl[p] & LMR_XHDR_SCALAR) ? 0 : uint64_t(rC) * rcb[p] * eb;
        };
        if (nowait) {
            // whole fixed regions both ways: every size follows from chunk 0's rows
            uint64_t a = 0, c = 0;
            for (uint32_t p = 0; p < npes; p++) {
                isb[p] = my_cap * iw;
                iso[p] = uint64_t(p) * my_cap * iw;
                vsb[p] = scalar ? 0 : my_cap * eb;
                vso[p] = scalar ? 0 : uint64_t(p) * my_cap * eb;
                irb[p] = capr[p] * iw;
                vrb[p] = (src_fl[p] & LMR_XHDR_SCALAR) ? 0 : capr[p] * eb;
                if (rb) send_bucketed(p);
                if (src_fl[p] & LMR_XHDR_BUCKETS) recv_bucketed(p);
                iro[p] = a; a += irb[p];
                vro[p] = c; c += vrb[p];
            }
        } else {
            // exact counts; a FIXED sender's region holds at most its capacity (the rest is in its
            // overflow list) and starts at the region's base
            for (uint32_t p = 0; p < npes; p++) {
                const uint64_t sc_ = uint64_t(std::max<int64_t>(h_send[p * LMR_XHDR_WORDS], 0));
                const uint64_t rc_ = uint64_t(std::max<int64_t>(h_recv[p * LMR_XHDR_WORDS], 0));
                if (free_pack && !mvsi && j < my_k && hi > lo) {
                    const uint64_t s1 = std::min(sc_, my_cap);
                    isb[p] = s1 * iw;
                    iso[p] = uint64_t(p) * my_cap * iw;
                    vsb[p] = scalar ? 0 : s1 * eb;
                    vso[p] = scalar ? 0 : uint64_t(p) * my_cap * eb;
                }
                if (h_recv[p * LMR_XHDR_WORDS + 2] & LMR_XHDR_FIXED) {
                    const uint64_t r1 = std::min(rc_, capr[p]);
                    irb[p] = h_recv[p * LMR_XHDR_WORDS + 1] < 0 ? r1 * iw : 0;
                    vrb[p] = (h_recv[p * LMR_XHDR_WORDS + 2] & LMR_XHDR_SCALAR) ? 0 : r1 * eb;
                }
                cnt[p] = (h_recv[p * LMR_XHDR_WORDS + 2] & LMR_XHDR_FIXED) ? std::min(rc_, capr[p]) : rc_;
                if (rb && j < my_k && hi > lo) send_bucketed(p);
                if (src_fl[p] & LMR_XHDR_BUCKETS) {
                    recv_bucketed(p);
                    cnt[p] = 0;                          // (the owner reads the region's header)
                }
            }
            uint64_t a = 0, c = 0;
            for (uint32_t p = 0; p < npes; p++) {
                iro[p] = a; a += irb[p];
                vro[p] = c; c += vrb[p];
            }
        }
        // own records: out of the transport's splits (the receive layout keeps their gap)
        const uint64_t self_io = iso[me], self_vo = vso[me];
        if (bypass) isb[me] = irb[me] = vsb[me] = vrb[me] = 0;
        ChunkRec cr;
        cr.lo = mvsi ? 0 : lo;
        cr.hi = mvsi ? n : hi;
        cr.send_cnt.resize(npes);
        cr.recv_cnt.resize(npes);
        cr.total = 0;
        if (!nowait)
            for (uint32_t p = 0; p < npes; p++) {
                cr.send_cnt[p] = uint64_t(std::max<int64_t>(h_send[p * LMR_XHDR_WORDS], 0));
                cr.recv_cnt[p] = cnt[p];
                cr.total += cr.recv_cnt[p];
            }
        // ---- receive buffers of this chunk (double-buffered against the apply stream)
        if (x->recv_used[b] && hipStreamWaitEvent(x->sx, x->ev_recv_free[b], 0) != hipSuccess) return xfail(__LINE__);
        const uint64_t ib = iro[npes - 1] + irb[npes - 1], vb = vro[npes - 1] + vrb[npes - 1];
        if (x->recv_idx[b].need(ib + 8, x) != hipSuccess || x->recv_vals[b].need(vb + 8, x) != hipSuccess)
            return xfail(__LINE__);
        const uint8_t* send_vals = mvsi ? static_cast<const uint8_t*>(d_vals) : x->send_vals[b].as<uint8_t>();
        // the records after the chunk's header rows (and so after its pack): with no host read of
        // the rows in between, only this orders them (and the owner's staging, which reads the rows)
        if (nowait && hipStreamWaitEvent(x->sx, x->ev_hdr[b], 0) != hipSuccess) return xfail(__LINE__);
        // (bucketed regions are u32 areas: the index unit divides both them and iw-wide segments)
        st = tp_alltoallv(tp, x, x->send_idx[b].p, isb.data(), iso.data(), x->recv_idx[b].p, irb.data(), iro.data(),
                          rb ? std::min<uint32_t>(4, unit_for(iw)) : unit_for(iw), x->sx);
        if (st == LMR_OK)
            st = tp_alltoallv(tp, x, send_vals, vsb.data(), vso.data(), x->recv_vals[b].p, vrb.data(), vro.data(),
                              unit_for(eb), x->sx);
        if (st != LMR_OK) { guard.tp_failed = true; return st; }
        if (hipEventRecord(x->ev_send_free[b], x->sx) != hipSuccess) return xfail(__LINE__);
        x->send_used[b] = true;
        if (hipEventRecord(x->ev_x[b], x->sx) != hipSuccess || hipStreamWaitEvent(x->sa, x->ev_x[b], 0) != hipSuccess)
            return xfail(__LINE__);
        // ---- owner side: stage every source's records (apply stream)
        if (returning) {
            if (x->res.size() <= j) { x->res.resize(j + 1); x->rok.resize(j + 1); }
            if (x->res[j].need(cr.total * eb + 8, x) != hipSuccess) return xfail(__LINE__);
            if (want_ok && x->rok[j].need(cr.total + 8, x) != hipSuccess) return xfail(__LINE__);
        }
        // bucketed regions: every source's slices binned in one launch (or applied directly)
        {
            BucketChunk c;
            c.S = npes;
            bool any = false;
            for (uint32_t p = 0; p < npes; p++) {
                if (!(src_fl[p] & LMR_XHDR_BUCKETS) || rcb[p] == 0) continue;
                const bool own = bypass && p == me;
                const bool sc = (src_fl[p] & LMR_XHDR_SCALAR) != 0;
                c.idx[p] = own ? x->send_idx[b].as<uint8_t>() + self_io : x->recv_idx[b].as<uint8_t>() + iro[p];
                c.val[p] = sc ? nullptr : own ? send_vals + self_vo : x->recv_vals[b].as<uint8_t>() + vro[p];
                c.sbits[p] = uint64_t(src_bits[p]);
                c.cap_b[p] = rcb[p];
                const uint64_t ch = uint64_t(std::max<int64_t>(src_ch[p], 1));
                c.expect += (std::min(ch, uint64_t(std::max<int64_t>(src_m[p], 0))) + npes - 1) / npes;
                any = true;
            }
            if (any && bsess) {
                if (x->bs.open && x->bs.staged + c.expect > bucket_session_limit(x->bs) &&
                    bucket_sweep(ctx, x, x->sa) != hipSuccess)
                    return xfail(__LINE__);
                if (!bucket_open()) return xfail(__LINE__);
                TiledWs w = carve_tiled_ws(ctx->ws, ctx->rec_cap);
                if (launch_fine_bucket(c, x->bs, w, x->sa) != hipSuccess) return xfail(__LINE__);
                x->bs.staged += c.expect;
            } else if (any && launch_bucket_direct(c, *desc, rC, rshift, ctx->d_err, x->sa) != hipSuccess) {
                return xfail(__LINE__);
            }
        }
        if (nowait) {
            // fixed regions with their counts in the header rows (device), each its own stream
            for (uint32_t p = 0; p < npes; p++) {
                const bool own = bypass && p == me;
                const uint64_t cap = own ? my_cap : capr[p];
                if (cap == 0 || (src_fl[p] & LMR_XHDR_BUCKETS)) continue;
                const uint8_t* src_i = own ? x->send_idx[b].as<uint8_t>() + self_io : x->recv_idx[b].as<uint8_t>() + iro[p];
                const bool sc = (src_fl[p] & LMR_XHDR_SCALAR) != 0;
                const uint8_t* src_v = sc ? nullptr : own ? send_vals + self_vo : x->recv_vals[b].as<uint8_t>() + vro[p];
                const int64_t* d_n = own ? x->hdr_send[b].as<int64_t>() + uint64_t(me) * LMR_XHDR_WORDS
                                         : x->hdr_recv[b].as<int64_t>() + uint64_t(p) * LMR_XHDR_WORDS;
                const uint64_t ch = uint64_t(std::max<int64_t>(src_ch[p], 1));
                const uint64_t expect = (std::min(ch, uint64_t(std::max<int64_t>(src_m[p], 0))) + npes - 1) / npes;
                const uint64_t ubits = uint64_t(src_bits[p]);
                st = stage_soa_dev(ctx, src_i, iw, src_v, sc ? &ubits : nullptr, cap, expect, d_n, x->sa);
                if (st != LMR_OK) return st;
            }
        } else {
            st = stage_host(b, h_recv, cnt, self_io, self_vo, send_vals, j);
            if (st != LMR_OK) return st;
        }
        // this chunk's streams partitioned now (fused), before its receive buffers are reused
        if ((st = lmr_stage_flush(ctx, reinterpret_cast<lmr_stream_t>(x->sa))) != LMR_OK) return st;
        if (hipEventRecord(x->ev_recv_free[b], x->sa) != hipSuccess) return xfail(__LINE__);
        x->recv_used[b] = true;
        chunks.push_back(std::move(cr));
        // ---- the next chunk's header exchange (after this chunk's all-to-all-v on the
        // exchange stream: every PE posts the collectives in the same order), and the pack of
        // the chunk after it, which runs while the host waits for that header
        if (j + 1 < nchunks) {
            if (!split) {
                if ((st = pack_until(j + 2)) != LMR_OK) return st;
                if ((st = post_header(j + 1, !nowait || j + 2 == nchunks)) != LMR_OK) return st;
            }
            if ((st = pack_until(std::min<uint64_t>(j + 3, nchunks))) != LMR_OK) return st;
        }
    }
    }   // (not push)
    // ---- overflow round (some PE packed fixed regions): the records that did not fit their
    // region, from every FIXED sender's overflow list, packed by the counted pack and exchanged
    // with exact counts (one more header exchange, read by the host once per batch)
    // (skipped when no PE's last-chunk rows carry LMR_XHDR_OVERFLOW: every PE reads the same rows,
    // so every PE skips it alike)
    bool any_ovf = false;
    if (any_fixed && !push) {
        const int bl = int((nchunks - 1) & 1);
        if (hipEventSynchronize(x->ev_hdr[bl]) != hipSuccess) return xfail(__LINE__);
        const int64_t* h_last = h_recv_rows(bl);
        for (uint32_t p = 0; p < npes; p++) any_ovf = any_ovf || (h_last[p * LMR_XHDR_WORDS + 2] & LMR_XHDR_OVERFLOW);
    }
    if (any_fixed && (push || any_ovf)) {
        const uint64_t J = nchunks;
        const int b = int(J & 1);
        uint64_t novf = 0;
        if (free_pack) {
            uint32_t c32 = 0;
            if (hipMemcpyAsync(&c32, x->ovf_count.p, 4, hipMemcpyDeviceToHost, x->sp) != hipSuccess ||
                hipStreamSynchronize(x->sp) != hipSuccess)
                return xfail(__LINE__);
            novf = std::min<uint64_t>(c32, m);
        }
        if ((st = wait_send_slot(b)) != LMR_OK) return st;
        if (novf > 0) {
            if (x->send_idx[b].need(novf * iw + 8, x) != hipSuccess ||
                x->send_vals[b].need(novf * eb + 8, x) != hipSuccess)
                return xfail(__LINE__);
            st = lmr_pack_unordered(ctx, layout, x->ovf_idx.as<uint64_t>(), novf, scalar ? nullptr : x->ovf_vals.p,
                                    desc->dtype, iw, x->send_idx[b].p, scalar ? nullptr : x->send_vals[b].p, nullptr,
                                    x->counts.as<uint64_t>(), x->offsets.as<uint64_t>(),
                                    reinterpret_cast<lmr_stream_t>(x->sp));
            if (st != LMR_OK) return st;
        }
        hipLaunchKernelGGL(k_xhdr, dim3((npes + 255) / 256), dim3(256), 0, x->sp,
                           novf > 0 ? x->counts.as<uint64_t>() : nullptr, npes, int64_t(-1), int64_t(0), int64_t(0),
                           int64_t(scalar ? LMR_XHDR_SCALAR : 0), sbits, int64_t(1), int64_t(novf), int64_t(novf),
                           x->hdr_send[b].as<int64_t>(), nullptr);
        if (hipGetLastError() != hipSuccess || hipEventRecord(x->ev_packed[b], x->sp) != hipSuccess) return xfail(__LINE__);
        if ((st = post_header(J, true)) != LMR_OK) return st;
        if (hipEventSynchronize(x->ev_hdr[b]) != hipSuccess) return xfail(__LINE__);
        const int64_t* h_send = h_send_rows(b);
        const int64_t* h_recv = h_recv_rows(b);
        (void)lmr_exchange_plan(npes, iw, eb, h_send, h_recv, isb.data(), iso.data(), irb.data(), iro.data(),
                                vsb.data(), vso.data(), vrb.data(), vro.data());
        std::vector<uint64_t> cnt(npes);
        for (uint32_t p = 0; p < npes; p++) cnt[p] = uint64_t(std::max<int64_t>(h_recv[p * LMR_XHDR_WORDS], 0));
        {   // every PE takes part even with nothing to send or receive: a transport's all-to-all-v
            // may be a collective (the host transports' are)
            const uint64_t self_io = iso[me], self_vo = vso[me];
            if (bypass) isb[me] = irb[me] = vsb[me] = vrb[me] = 0;
            if (x->recv_used[b] && hipStreamWaitEvent(x->sx, x->ev_recv_free[b], 0) != hipSuccess) return xfail(__LINE__);
            const uint64_t ib = iro[npes - 1] + irb[npes - 1], vb = vro[npes - 1] + vrb[npes - 1];
            if (x->recv_idx[b].need(ib + 8, x) != hipSuccess || x->recv_vals[b].need(vb + 8, x) != hipSuccess)
                return xfail(__LINE__);
            const uint8_t* send_vals = x->send_vals[b].as<uint8_t>();
            st = tp_alltoallv(tp, x, x->send_idx[b].p, isb.data(), iso.data(), x->recv_idx[b].p, irb.data(),
                              iro.data(), unit_for(iw), x->sx);
            if (st == LMR_OK)
                st = tp_alltoallv(tp, x, send_vals, vsb.data(), vso.data(), x->recv_vals[b].p, vrb.data(), vro.data(),
                                  unit_for(eb), x->sx);
            if (st != LMR_OK) { guard.tp_failed = true; return st; }
            if (hipEventRecord(x->ev_send_free[b], x->sx) != hipSuccess) return xfail(__LINE__);
            x->send_used[b] = true;
            if (hipEventRecord(x->ev_x[b], x->sx) != hipSuccess || hipStreamWaitEvent(x->sa, x->ev_x[b], 0) != hipSuccess)
                return xfail(__LINE__);
            if ((st = stage_host(b, h_recv, cnt, self_io, self_vo, send_vals, J)) != LMR_OK) return st;
            if ((st = lmr_stage_flush(ctx, reinterpret_cast<lmr_stream_t>(x->sa))) != LMR_OK) return st;
            if (hipEventRecord(x->ev_recv_free[b], x->sa) != hipSuccess) return xfail(__LINE__);
            x->recv_used[b] = true;
        }
    }
    // ---- one shard sweep (or, deferred, the session left open for the next batch), then results
    // back to their senders
    if (ctx->xdefer_on && !returning && !ordered && stage_session_free(ctx)) {
        ctx->xdefer_open = true;
    } else {
        st = lmr_stage_finish(ctx, reinterpret_cast<lmr_stream_t>(x->sa));
        if (st != LMR_OK) return st;
        if (bucket_sweep(ctx, x, x->sa) != hipSuccess) return xfail(__LINE__);
    }
    guard.armed = false;
    if (returning) {
        std::vector<uint64_t> sb(npes), so(npes), rb(npes), ro(npes), osb(npes), oso(npes), orb(npes), oro(npes);
        for (uint64_t j = 0; j < chunks.size(); j++) {
            const ChunkRec& cr = chunks[j];
            uint64_t a = 0, bb = 0, nsent = 0;
            for (uint32_t p = 0; p < npes; p++) {
                sb[p] = cr.recv_cnt[p] * eb; so[p] = a; a += sb[p];
                rb[p] = cr.send_cnt[p] * eb; ro[p] = bb; bb += rb[p];
                osb[p] = cr.recv_cnt[p]; oso[p] = so[p] / eb;
                orb[p] = cr.send_cnt[p]; oro[p] = ro[p] / eb;
                nsent += cr.send_cnt[p];
            }
            if (x->back.need(nsent * eb + 8, x) != hipSuccess || (want_ok && x->back_ok.need(nsent + 8, x) != hipSuccess))
                return xfail(__LINE__);
            if (bypass && cr.recv_cnt[me]) {           // own results: a device copy, not the transport
                if (hipMemcpyAsync(static_cast<uint8_t*>(x->back.p) + ro[me], x->res[j].as<uint8_t>() + so[me], sb[me],
                                   hipMemcpyDeviceToDevice, x->sa) != hipSuccess ||
                    (want_ok && hipMemcpyAsync(x->back_ok.as<uint8_t>() + oro[me], x->rok[j].as<uint8_t>() + oso[me],
                                               osb[me], hipMemcpyDeviceToDevice, x->sa) != hipSuccess))
                    return xfail(__LINE__);
            }
            if (bypass) sb[me] = rb[me] = osb[me] = orb[me] = 0;
            st = tp_alltoallv(tp, x, x->res[j].p, sb.data(), so.data(), x->back.p, rb.data(), ro.data(), unit_for(eb),
                              x->sa);
            if (st == LMR_OK && want_ok)
                st = tp_alltoallv(tp, x, x->rok[j].p, osb.data(), oso.data(), x->back_ok.p, orb.data(), oro.data(), 1,
                                  x->sa);
            if (st != LMR_OK) {                         // (the session is already applied)
                transport_abort(tp);
                (void)x->drain();
                return st;
            }
            if (nsent == 0) continue;
            if (mvsi) {                                 // results come back in value order
                if (hipMemcpyAsync(d_results, x->back.p, nsent * eb, hipMemcpyDeviceToDevice, x->sa) != hipSuccess ||
                    (want_ok && hipMemcpyAsync(d_ok, x->back_ok.p, nsent, hipMemcpyDeviceToDevice, x->sa) != hipSuccess))
                    return xfail(__LINE__);
            } else {
                st = lmr_scatter_results(x->back.p, x->pos[j].as<uint32_t>(), nsent, eb,
                                         static_cast<uint8_t*>(d_results) + cr.lo * eb, want_ok ? x->back_ok.as<uint8_t>() : nullptr,
                                         want_ok ? d_ok + cr.lo : nullptr, reinterpret_cast<lmr_stream_t>(x->sa));
                if (st != LMR_OK) return st;
            }
        }
    }
    // ---- the caller's stream continues after the internal streams
    if (hipEventRecord(x->ev_pack_done, x->sp) != hipSuccess || hipEventRecord(x->ev_x_done, x->sx) != hipSuccess ||
        hipEventRecord(x->ev_apply_done, x->sa) != hipSuccess || hipEventRecord(x->ev_h_done, x->sh) != hipSuccess ||
        hipStreamWaitEvent(s0, x->ev_pack_done, 0) != hipSuccess || hipStreamWaitEvent(s0, x->ev_x_done, 0) != hipSuccess ||
        hipStreamWaitEvent(s0, x->ev_apply_done, 0) != hipSuccess || hipStreamWaitEvent(s0, x->ev_h_done, 0) != hipSuccess)
        return xfail(__LINE__);
    if (push && (hipEventRecord(x->ev_marked[0], x->sw_free) != hipSuccess ||
                 hipEventRecord(x->ev_marked[1], x->sw_pub) != hipSuccess ||
                 hipStreamWaitEvent(s0, x->ev_marked[0], 0) != hipSuccess ||
                 hipStreamWaitEvent(s0, x->ev_marked[1], 0) != hipSuccess))
        return xfail(__LINE__);
    return LMR_OK;
}

lmr_status_t lmr_ctx_exchange_defer(lmr_ctx_t* ctx, int on) {
    if (!ctx) return LMR_E_INVALID;
    ctx->xdefer_on = on != 0;
    return LMR_OK;
}

lmr_status_t lmr_exchange_flush(lmr_ctx_t* ctx, lmr_stream_t stream) {
    if (!ctx) return LMR_E_INVALID;
    if (!ctx->xdefer_open) return LMR_OK;
    ctx->xdefer_open = false;
    XState* x = ctx->xch;
    const bool bopen = x && x->bs.open;
    if (!stage_session_open(ctx) && !bopen) return LMR_OK;
    // the session was staged on the exchange's apply stream: `stream` (any stream, per the
    // header) waits for that staging before the sweep
    if (x) {
        if (hipEventRecord(x->ev_apply_done, x->sa) != hipSuccess ||
            hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), x->ev_apply_done, 0) != hipSuccess)
            return LMR_E_HIP;
    }
    if (bopen && bucket_sweep(ctx, x, reinterpret_cast<hipStream_t>(stream)) != hipSuccess) return LMR_E_HIP;
    if (!stage_session_open(ctx)) return LMR_OK;
    return lmr_stage_finish(ctx, stream);
}

}  // extern "C"
