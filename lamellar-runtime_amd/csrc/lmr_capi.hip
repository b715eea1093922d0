// lmr_capi.hip — the extern "C" entry points of liblamellar_gpu_ops.so
// (declared in include/lamellar_gpu_ops.h): context/workspace management,
// host index math, argument checking and strategy dispatch.
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "../../include/lamellar_gpu_ops.h"
#include "lmr_internal.hpp"
#include "lmr_device.hpp"

namespace lmr {
// Stage timer: a pool of HIP events recorded on the launch stream around each
// kernel stage; read back (and the pool recycled) by lmr_ctx_profile_read.
struct Prof {
    std::vector<hipEvent_t> pool;
    size_t next = 0;
    struct Rec { int stage; hipEvent_t a, b; uint64_t n; };
    std::vector<Rec> pending;
    hipEvent_t open_ev[LMR_NUM_STAGES] = {};
    double ms[LMR_NUM_STAGES] = {};
    uint64_t cnt[LMR_NUM_STAGES] = {};
    uint64_t recs[LMR_NUM_STAGES] = {};
    hipEvent_t get() {
        if (next == pool.size()) {
            hipEvent_t e = nullptr;
            // device-scope release: the stage events only time kernels, and a system-scope fence
            // (the default) writes back and invalidates the caches at every stage boundary
            if (hipEventCreateWithFlags(&e, device_scope_events() ? hipEventReleaseToDevice : hipEventDefault) !=
                hipSuccess)
                return nullptr;
            pool.push_back(e);
        }
        return pool[next++];
    }
};
void prof_begin(Prof* p, int st, hipStream_t s) {
    hipEvent_t e = p->get();
    if (e && hipEventRecord(e, s) == hipSuccess) p->open_ev[st] = e;
    else p->open_ev[st] = nullptr;
}
void prof_end(Prof* p, int st, hipStream_t s, uint64_t n) {
    hipEvent_t e = p->get();
    if (e && p->open_ev[st] && hipEventRecord(e, s) == hipSuccess)
        p->pending.push_back({st, p->open_ev[st], e, n});
}

// Staged-apply session of a context (lmr_stage_begin / _soa / _finish).
struct StageState {
    bool open = false;
    lmr_apply_desc_t desc{};
    StageSession s;
};
void stage_state_free(StageState* s) { delete s; }
void stage_abort(StageState* s) {
    if (!s) return;
    s->open = false;
    s->s = StageSession();
}
// A count-free session whose regions are only recorded (none partitioned, none with a device-side
// count) and whose shard takes the wide path becomes a counted session: its regions keep their op
// and are the first phase of the mixed session that follows (lmr_stage_op).
bool stage_free_to_wide(StageSession& s, uint64_t cap) {
    if (!s.free || s.parted != 0 || s.nreg == 0 || !wide_applies(s.dtype, s.pend[0].a.shard_len, cap)) return false;
    for (int r = 0; r < s.nreg; r++)
        if (s.pend[r].n_dev) return false;
    uint64_t b = 0;
    for (int r = 0; r < s.nreg; r++) {
        s.reg[r].base = b;
        s.reg[r].results = nullptr;
        s.reg[r].ok = nullptr;
        s.reg[r].ret = LMR_RET_NONE;
        b += s.reg[r].n;
    }
    s.staged = b;
    s.free = false;
    return true;
}
bool stage_pending_other_op(const StageSession& s, const ApplyArgs& a) {
    for (int r = 0; r < s.nreg; r++)
        if (s.reg[r].op != a.op || s.reg[r].cmp_bits != a.cmp_bits || s.reg[r].eps_bits != a.eps_bits) return true;
    return false;
}
}  // namespace lmr

using namespace lmr;

namespace {

// the context's workspace carved for `cap` records, with its side lane
TiledWs ctx_ws(const lmr_ctx* ctx, uint64_t cap) {
    TiledWs w = carve_tiled_ws(ctx->ws, cap);
    w.side = SideLane{ctx->side, ctx->side_fork, ctx->side_join};
    return w;
}

constexpr size_t kPackScratchCounts = size_t(kMaxPackPes) * kMaxBinBlocks;

struct CtxExtra {
    uint32_t* pack_counts = nullptr;
    uint32_t* pack_partials = nullptr;
    uint32_t* pack_total = nullptr;
    uint64_t* red_part = nullptr;      // [kReduceBlocks]
    uint8_t* red_has = nullptr;        // [kReduceBlocks]
};

// The small pack / reduce scratch lives right after the error word in one allocation.
size_t pack_scratch_bytes() {
    return 256 + kPackScratchCounts * 4 + 256 + scan_scratch_words(kPackScratchCounts) * 4 + 256 +
           size_t(kReduceBlocks) * 9 + 512;
}

CtxExtra pack_scratch(lmr_ctx* c) {
    CtxExtra x;
    uint8_t* p = reinterpret_cast<uint8_t*>(c->d_err) + 256;
    x.pack_counts = reinterpret_cast<uint32_t*>(p);
    p += ((kPackScratchCounts * 4 + 255) & ~size_t(255));
    x.pack_partials = reinterpret_cast<uint32_t*>(p);
    p += ((scan_scratch_words(kPackScratchCounts) * 4 + 255) & ~size_t(255));
    x.pack_total = reinterpret_cast<uint32_t*>(p);
    p += 256;
    x.red_part = reinterpret_cast<uint64_t*>(p);
    p += size_t(kReduceBlocks) * 8;
    x.red_has = p;
    return x;
}

lmr_status_t status_of_bits(uint32_t b) {
    if (b & LMR_ERRBIT_OOB) return LMR_E_OOB;
    if (b & LMR_ERRBIT_DIVZERO) return LMR_E_DIVZERO;
    if (b & LMR_ERRBIT_OVERFLOW) return LMR_E_OVERFLOW;
    if (b & LMR_ERRBIT_UNSUPPORTED) return LMR_E_UNSUPPORTED;
    if (b & LMR_ERRBIT_TRANSPORT) return LMR_E_HIP;
    return LMR_OK;
}

inline lmr_status_t hip_status(hipError_t e) { return e == hipSuccess ? LMR_OK : LMR_E_HIP; }

// ---- host index math (src/array/unsafe.rs) ----
bool start_index_for_pe(const lmr_layout_t& L, uint64_t pe, uint64_t& out) {  // :1889-1941
    if (L.distribution == LMR_DIST_BLOCK) {
        uint64_t gs = L.orig_elem_per_pe * pe + (pe < L.orig_remaining_elems ? pe : L.orig_remaining_elems);
        if (gs >= L.offset) {
            if (gs - L.offset < L.size) { out = gs - L.offset; return true; }
            return false;
        }
        uint64_t ge = gs + L.orig_elem_per_pe + (pe < L.orig_remaining_elems ? 1 : 0);
        if (L.offset < ge) { out = 0; return true; }
        return false;
    }
    uint64_t start_pe;
    if (!pe_for_dist_index(L, 0, start_pe)) return false;
    uint64_t tl = L.size < L.num_pes ? L.size : L.num_pes;
    for (uint64_t i = 0; i < tl; i++)
        if ((i + start_pe) % L.num_pes == pe) { out = i; return true; }
    return false;
}

uint64_t num_elems_pe(const lmr_layout_t& L, uint64_t pe) {  // :1966-2016
    if (L.distribution == LMR_DIST_BLOCK) {
        uint64_t si, ei;
        if (!start_index_for_pe(L, pe, si)) return 0;
        if (!start_index_for_pe(L, pe + 1, ei)) ei = L.size;
        return ei - si;
    }
    uint64_t sp, ep;
    if (!pe_for_dist_index(L, 0, sp) || !pe_for_dist_index(L, L.size - 1, ep)) return 0;
    uint64_t n = L.size / L.num_pes;
    if (L.size % L.num_pes) {
        if (sp <= ep) { if (pe >= sp && pe <= ep) n++; }
        else if (pe >= sp || pe <= ep) n++;
    }
    return n;
}

bool valid_layout(const lmr_layout_t* L) {
    return L && L->num_pes > 0 && L->my_pe < L->num_pes && L->distribution <= 1 &&
           L->orig_elem_per_pe > 0;
}

bool valid_iw(uint32_t iw) { return iw == 1 || iw == 2 || iw == 4 || iw == 8; }

lmr_status_t check_desc(const lmr_apply_desc_t* d) {
    if (!d || d->dtype >= LMR_NUM_DTYPES || d->op >= LMR_NUM_OPS || d->kind > LMR_KIND_READ_ONLY ||
        d->strategy > LMR_STRATEGY_ORDERED)
        return LMR_E_INVALID;
    if (!lmr_op_supported(d->kind, d->dtype, d->op)) return LMR_E_UNSUPPORTED;
    return LMR_OK;
}

ApplyArgs base_args(lmr_ctx* ctx, const lmr_apply_desc_t* d, void* results, uint8_t* ok) {
    ApplyArgs a{};
    a.shard = d->shard;
    a.shard_len = d->shard_len;
    a.kind = int(d->kind);
    a.op = int(d->op);
    uint32_t rk = lmr_op_ret_kind(d->op);
    a.ret = results ? int(rk) : LMR_RET_NONE;
    a.cmp_bits = d->cmp_bits;
    a.eps_bits = d->eps_bits;
    a.err = ctx->d_err;
    a.results = results;
    a.ok = (rk == LMR_RET_RESULT) ? ok : nullptr;
    if (a.ret == LMR_RET_RESULT && !a.ok) a.ret = LMR_RET_VALS;
    a.prof = ctx->prof;
    return a;
}

uint64_t load_scalar_bits(const void* val, int dtype) {
    uint64_t b = 0;
    if (val) memcpy(&b, val, size_t(dtype_bytes(dtype)));
    return b;
}

// Stage the records of `a` as one or more regions (workspace-sized pieces),
// applying what is staged first whenever the workspace or the region table is full.
hipError_t stage_records(lmr_ctx* ctx, StageSession& ss, const ApplyArgs& a, int dtype, int iw, uint64_t split,
                         hipStream_t s) {
    TiledWs w = ctx_ws(ctx, ctx->rec_cap);
    const int eb = dtype_bytes(dtype);
    uint64_t piece = ctx->rec_cap < kStageMaxRegion ? ctx->rec_cap : kStageMaxRegion;
    if (split > 1) {
        const uint64_t per = (a.n + split - 1) / split;
        if (per < piece) piece = per;
    }
    for (uint64_t p0 = 0; p0 < a.n; p0 += piece) {
        const uint64_t m = a.n - p0 < piece ? a.n - p0 : piece;
        if (ss.staged + m > ctx->rec_cap || ss.nreg == kMaxRegions) {
            hipError_t e = launch_stage_finish(w, ss, s);
            if (e != hipSuccess) return e;
        }
        ApplyArgs b = a;
        b.n = m;
        b.idx = a.idx + p0 * a.idx_stride;
        if (a.val) b.val = a.val + p0 * a.val_stride;
        if (a.results) b.results = reinterpret_cast<uint8_t*>(a.results) + p0 * uint64_t(eb);
        if (a.ok) b.ok = a.ok + p0;
        hipError_t e = launch_stage_region(dtype, iw, b, w, ss, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// LMR_STAGED=1 routes the one-shot tiled path through the staged pipeline
// (LMR_STAGE_SPLIT=k: k regions per call); read per call, tests switch it.
// Unset: automatic -- the piece-based (staged) partition when the segment-based
// fine pass would see short segments (piece_partition_pays), e.g. C5's 27 M-record
// u32 batches: fine 1.25 -> 0.83 ms, unless the count-free partition applies (it has
// no segments); LMR_STAGED=0 keeps the one-shot path.
uint64_t staged_mode_split(int dtype, int op, int ret, uint64_t shard_len, uint64_t n, uint64_t cap) {
    const char* e = getenv("LMR_STAGED");
    if (e && e[0] == '0') return 0;
    if (!e || e[0] != '1')
        return (piece_partition_pays(dtype, shard_len, n) && !free_partition_applies(dtype, op, ret, shard_len, n, cap))
                   ? 1 : 0;
    const char* k = getenv("LMR_STAGE_SPLIT");
    const long v = (k && *k) ? atol(k) : 1;
    return v < 1 ? 1 : uint64_t(v);
}

// Run a record stream with the chosen strategy, in workspace-sized pieces.
lmr_status_t run_apply(lmr_ctx* ctx, const lmr_apply_desc_t* d, ApplyArgs a, int iw,
                       hipStream_t s) {
    // a deferred exchange session's records live in the workspace this call may use: applied first
    if (ctx->xdefer_open) {
        const lmr_status_t st = lmr_exchange_flush(ctx, reinterpret_cast<lmr_stream_t>(s));
        if (st != LMR_OK) return st;
    }
    const int eb = dtype_bytes(int(d->dtype));
    if (d->strategy == LMR_STRATEGY_ORDERED || (d->strategy == LMR_STRATEGY_AUTO && a.n < kOrderedAuto))
        return hip_status(launch_apply_ordered(ctx, int(d->dtype), iw, a, s));
    bool tiled = false;
    if (d->strategy == LMR_STRATEGY_TILED) {
        if (!ctx->ws || ctx->rec_cap == 0) return LMR_E_WORKSPACE;
        tiled = true;
    } else if (d->strategy == LMR_STRATEGY_AUTO) {
        tiled = ctx->ws && ctx->rec_cap > 0 && a.n >= 65536;
    }
    if (tiled && !tiled_supported(int(d->dtype), d->shard_len)) {
        // shard above one tiled window: records by window, each window tiled
        const hipError_t e = apply_windowed(ctx, d, a, iw, s, [ctx](const lmr_apply_desc_t* dw, const ApplyArgs& b,
                                                                    hipStream_t st) {
            return run_apply(ctx, dw, b, 4, st) == LMR_OK ? hipSuccess : hipErrorUnknown;
        });
        if (e == hipErrorNotSupported) return hip_status(launch_apply_direct(int(d->dtype), iw, a, s));
        return hip_status(e);
    }
    if (!tiled) return hip_status(launch_apply_direct(int(d->dtype), iw, a, s));
    if (const uint64_t split = staged_mode_split(int(d->dtype), a.op, a.ret, d->shard_len,
                                                 a.n < ctx->rec_cap ? a.n : ctx->rec_cap, ctx->rec_cap)) {
        StageSession ss;
        ss.a = a;
        ss.dtype = int(d->dtype);
        ss.free = stage_free_applies(int(d->dtype), a.op, a.ret, d->shard_len, ctx->rec_cap);
        hipError_t e = stage_records(ctx, ss, a, int(d->dtype), iw, split, s);
        if (e == hipSuccess) e = launch_stage_finish(ctx_ws(ctx, ctx->rec_cap), ss, s);
        return hip_status(e);
    }
    TiledWs w = ctx_ws(ctx, ctx->rec_cap);
    const uint64_t n = a.n;
    for (uint64_t p0 = 0; p0 < n; p0 += ctx->rec_cap) {
        uint64_t m = n - p0 < ctx->rec_cap ? n - p0 : ctx->rec_cap;
        ApplyArgs b = a;
        b.n = m;
        b.idx = a.idx + p0 * a.idx_stride;
        if (a.val) b.val = a.val + p0 * a.val_stride;
        if (a.results) b.results = reinterpret_cast<uint8_t*>(a.results) + p0 * uint64_t(eb);
        if (a.ok) b.ok = a.ok + p0;
        hipError_t e = launch_apply_tiled(int(d->dtype), iw, b, w, s);
        if (e != hipSuccess) return LMR_E_HIP;
    }
    return LMR_OK;
}

}  // namespace

namespace lmr {

bool stage_session_free(const lmr_ctx* ctx) { return ctx->stage && ctx->stage->open && ctx->stage->s.free; }
bool stage_session_open(const lmr_ctx* ctx) { return ctx->stage && ctx->stage->open; }
bool stage_session_empty(const lmr_ctx* ctx) { return !stage_session_open(ctx) || ctx->stage->s.nreg == 0; }
bool stage_session_of(const lmr_ctx* ctx, const lmr_apply_desc_t& d) {
    if (!stage_session_open(ctx)) return false;
    const lmr_apply_desc_t& c = ctx->stage->desc;
    return c.shard == d.shard && c.shard_len == d.shard_len && c.kind == d.kind && c.dtype == d.dtype &&
           c.op == d.op && c.strategy == d.strategy && c.cmp_bits == d.cmp_bits && c.eps_bits == d.eps_bits;
}

lmr_status_t stage_soa_dev(lmr_ctx* ctx, const void* d_indices, uint32_t index_size, const void* d_vals,
                           const void* val, uint64_t cap, uint64_t expect, const int64_t* d_n, hipStream_t s) {
    if (!stage_session_free(ctx) || !valid_iw(index_size) || !d_n) return LMR_E_INVALID;
    if (cap == 0) return LMR_OK;
    if (!d_indices || (!d_vals && !val)) return LMR_E_INVALID;
    StageState* S = ctx->stage;
    const lmr_apply_desc_t* d = &S->desc;
    ApplyArgs a = base_args(ctx, d, nullptr, nullptr);
    a.idx = reinterpret_cast<const uint8_t*>(d_indices);
    a.idx_stride = index_size;
    a.val = reinterpret_cast<const uint8_t*>(d_vals);
    a.val_stride = d_vals ? uint64_t(dtype_bytes(int(d->dtype))) : 0;
    a.val_bits = d_vals ? 0 : load_scalar_bits(val, int(d->dtype));
    a.n = cap;
    a.ret = S->s.a.ret;
    const TiledWs w = ctx_ws(ctx, ctx->rec_cap);
    const uint64_t e = std::min(expect, cap);
    if (S->s.staged + e > ctx->rec_cap || S->s.nreg == kMaxRegions) {
        const hipError_t he = launch_stage_finish(w, S->s, s);
        if (he != hipSuccess) return hip_status(he);
    }
    return hip_status(launch_stage_region_dev(int(d->dtype), int(index_size), a, d_n, e, w, S->s, s));
}

}  // namespace lmr

extern "C" {

uint32_t lmr_abi_version(void) { return LMR_ABI_VERSION; }

const char* lmr_status_string(lmr_status_t st) {
    switch (st) {
    case LMR_OK: return "ok";
    case LMR_E_INVALID: return "invalid argument";
    case LMR_E_OOB: return "index out of bounds";
    case LMR_E_DIVZERO: return "integer division or remainder by zero";
    case LMR_E_OVERFLOW: return "integer overflow (MIN / -1)";
    case LMR_E_UNSUPPORTED: return "op not available for this array kind / element type";
    case LMR_E_HIP: return "HIP runtime error";
    case LMR_E_WORKSPACE: return "workspace too small / not reserved";
    case LMR_E_LENGTH: return "index and value inputs differ in length";
    default: return "unknown status";
    }
}

lmr_status_t lmr_ctx_create(int device, lmr_ctx_t** out) {
    if (!out) return LMR_E_INVALID;
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return LMR_E_HIP;
    lmr_ctx* c = new lmr_ctx();
    c->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
    void* p = nullptr;
    if (hipMalloc(&p, pack_scratch_bytes()) != hipSuccess) { delete c; return LMR_E_HIP; }
    c->d_err = reinterpret_cast<uint32_t*>(p);
    // the error word and the pack scan's look-back scratch start zeroed
    if (hipMemset(p, 0, pack_scratch_bytes()) != hipSuccess) { (void)hipFree(p); delete c; return LMR_E_HIP; }
    if (ord_reserve(c, kOrderedMinPiece) != hipSuccess ||
        hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->side_fork, side_event_flags()) != hipSuccess ||
        hipEventCreateWithFlags(&c->side_join, side_event_flags()) != hipSuccess) {
        lmr_ctx_destroy(c);
        return LMR_E_HIP;
    }
    *out = c;
    return LMR_OK;
}

lmr_status_t lmr_ctx_destroy(lmr_ctx_t* ctx) {
    if (!ctx) return LMR_E_INVALID;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();                      // every buffer below may still be in use
    host_stage_free(ctx->host);
    stage_state_free(ctx->stage);
    xstate_free(ctx->xch);
    win_state_free(ctx->win);
    wire_bufs_free(ctx->wire);
    ord_bufs_free(ctx->ord);
    if (ctx->side) (void)hipStreamSynchronize(ctx->side);
    if (ctx->side_fork) (void)hipEventDestroy(ctx->side_fork);
    if (ctx->side_join) (void)hipEventDestroy(ctx->side_join);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    if (ctx->ws_alloc) (void)hipFree(ctx->ws_alloc);
    if (ctx->d_err) (void)hipFree(ctx->d_err);
    if (ctx->prof) {
        for (hipEvent_t e : ctx->prof->pool) (void)hipEventDestroy(e);
        delete ctx->prof;
    }
    delete ctx;
    return LMR_OK;
}

lmr_status_t lmr_ctx_reserve(lmr_ctx_t* ctx, uint64_t max_records) {
    if (!ctx) return LMR_E_INVALID;
    if (max_records > max_rec_cap()) max_records = max_rec_cap();
    // a deferred exchange session lives in the workspace: applied first (the free below waits for it)
    if (ctx->xdefer_open) {
        const lmr_status_t st = lmr_exchange_flush(ctx, nullptr);
        if (st != LMR_OK) return st;
    }
    if (ctx->stage && ctx->stage->s.nreg > 0) return LMR_E_INVALID;   // staged records live in the workspace
    (void)hipSetDevice(ctx->device);
    if (ctx->ws_alloc) (void)hipFree(ctx->ws_alloc);
    ctx->ws = ctx->ws_alloc = nullptr; ctx->ws_bytes = 0; ctx->rec_cap = 0;
    if (max_records == 0) return LMR_OK;
    if (ord_reserve(ctx, max_records) != hipSuccess) return LMR_E_HIP;
    size_t b = tiled_ws_bytes(max_records);
    void* p = nullptr;
    if (hipMalloc(&p, b) != hipSuccess) return LMR_E_HIP;
    ctx->ws_alloc = reinterpret_cast<uint8_t*>(p);
    ctx->ws = ctx->ws_alloc;
    ctx->ws_bytes = b;
    {   // the scan's look-back scratch starts zeroed (every scan leaves it so)
        const TiledWs w = ctx_ws(ctx, max_records);
        if (hipMemset(w.partials, 0, scan_scratch_words(size_t(kMaxTiles) * kMaxBinBlocks) * 4) != hipSuccess)
            return LMR_E_HIP;
    }
    ctx->rec_cap = max_records;
    return LMR_OK;
}

lmr_status_t lmr_ctx_error(lmr_ctx_t* ctx, lmr_stream_t stream, uint32_t* errbits, int clear) {
    if (!ctx) return LMR_E_INVALID;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (hipStreamSynchronize(s) != hipSuccess) return LMR_E_HIP;
    uint32_t b = 0;
    if (hipMemcpy(&b, ctx->d_err, 4, hipMemcpyDeviceToHost) != hipSuccess) return LMR_E_HIP;
    if (clear && b) {
        if (hipMemset(ctx->d_err, 0, 4) != hipSuccess) return LMR_E_HIP;
    }
    if (errbits) *errbits = b;
    return status_of_bits(b);
}

lmr_status_t lmr_ctx_profile(lmr_ctx_t* ctx, int enable) {
    if (!ctx) return LMR_E_INVALID;
    if (enable && !ctx->prof) ctx->prof = new Prof();
    if (!enable && ctx->prof) {
        for (auto& r : ctx->prof->pending) (void)hipEventSynchronize(r.b);   // the recorded stages only
        for (hipEvent_t e : ctx->prof->pool) (void)hipEventDestroy(e);
        delete ctx->prof;
        ctx->prof = nullptr;
    }
    return LMR_OK;
}

lmr_status_t lmr_ctx_profile_read(lmr_ctx_t* ctx, lmr_stream_t stream, double* stage_ms,
                                  uint64_t* stage_launches, uint64_t* stage_records, int reset) {
    if (!ctx) return LMR_E_INVALID;
    Prof* p = ctx->prof;
    if (!p) {
        for (int i = 0; i < LMR_NUM_STAGES; i++) {
            if (stage_ms) stage_ms[i] = 0;
            if (stage_launches) stage_launches[i] = 0;
            if (stage_records) stage_records[i] = 0;
        }
        return LMR_OK;
    }
    if (hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)) != hipSuccess) return LMR_E_HIP;
    for (auto& r : p->pending) {
        float ms = 0.f;
        if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            p->ms[r.stage] += ms;
            p->cnt[r.stage] += 1;
            p->recs[r.stage] += r.n;
        }
    }
    p->pending.clear();
    p->next = 0;
    for (int i = 0; i < LMR_NUM_STAGES; i++) {
        if (stage_ms) stage_ms[i] = p->ms[i];
        if (stage_launches) stage_launches[i] = p->cnt[i];
        if (stage_records) stage_records[i] = p->recs[i];
        if (reset) { p->ms[i] = 0; p->cnt[i] = 0; p->recs[i] = 0; }
    }
    return LMR_OK;
}

// ---------------------------------------------------------------- layout
lmr_status_t lmr_layout_new(lmr_layout_t* L, uint64_t array_size, uint32_t num_pes, uint32_t my_pe,
                            uint32_t distribution) {
    if (!L || num_pes == 0 || my_pe >= num_pes || distribution > 1) return LMR_E_INVALID;
    uint64_t full = array_size > num_pes ? array_size : num_pes;   // unsafe.rs:187
    memset(L, 0, sizeof(*L));
    L->distribution = distribution;
    L->num_pes = num_pes;
    L->my_pe = my_pe;
    L->orig_elem_per_pe = full / num_pes;
    L->orig_remaining_elems = full % num_pes;
    L->size = full;
    if (full != array_size) {                                       // unsafe.rs:265-270
        lmr_layout_t t = *L;
        return lmr_layout_sub(&t, 0, array_size, L);
    }
    return LMR_OK;
}

lmr_status_t lmr_layout_sub(const lmr_layout_t* parent, uint64_t start, uint64_t end,
                            lmr_layout_t* out) {
    if (!parent || !out || start > end || end > parent->size) return LMR_E_INVALID;
    lmr_layout_t L = *parent;
    L.offset += start;
    L.size = end - start;
    L.sub = 1;
    *out = L;
    return LMR_OK;
}

int lmr_pe_and_offset(const lmr_layout_t* L, uint64_t index, uint64_t* pe, uint64_t* offset) {
    if (!valid_layout(L) || !pe || !offset) return 0;
    return pe_and_offset(*L, index, *pe, *offset) ? 1 : 0;
}

uint64_t lmr_num_elems_pe(const lmr_layout_t* L, uint32_t pe) {
    if (!valid_layout(L)) return 0;
    return num_elems_pe(*L, pe);
}

uint64_t lmr_local_slice_start(const lmr_layout_t* L, uint32_t pe) {   // unsafe.rs:2023-2066
    if (!valid_layout(L)) return 0;
    if (L->distribution == LMR_DIST_BLOCK) {
        uint64_t sp;
        if (!pe_for_dist_index(*L, 0, sp) || sp != pe) return 0;
        uint64_t gs = L->orig_elem_per_pe * pe + (pe < L->orig_remaining_elems ? pe : L->orig_remaining_elems);
        return L->offset - gs;
    }
    uint64_t g = L->offset;
    return g / L->num_pes + ((pe >= g % L->num_pes) ? 0 : 1);
}

uint32_t lmr_index_size(const lmr_layout_t* L) {
    if (!valid_layout(L)) return 8;
    uint64_t m = 0;
    for (uint32_t p = 0; p < L->num_pes; p++) {
        uint64_t n = num_elems_pe(*L, p);
        if (n > m) m = n;
    }
    if (m <= 0xFFull) return 1;
    if (m <= 0xFFFFull) return 2;
    if (m <= 0xFFFFFFFFull) return 4;
    return 8;
}

uint32_t lmr_record_val_offset(uint32_t index_size, uint32_t dtype) {
    uint32_t tb = uint32_t(dtype_bytes(int(dtype)));
    if (!tb) return 0;
    return (index_size + tb - 1) / tb * tb;
}

uint32_t lmr_record_bytes(uint32_t index_size, uint32_t dtype) {
    uint32_t tb = uint32_t(dtype_bytes(int(dtype)));
    if (!tb || !valid_iw(index_size)) return 0;
    uint32_t a = index_size > tb ? index_size : tb;
    uint32_t raw = lmr_record_val_offset(index_size, dtype) + tb;
    return (raw + a - 1) / a * a;
}

uint32_t lmr_op_ret_kind(uint32_t op) {
    switch (op) {
    case LMR_OP_FETCH_ADD: case LMR_OP_FETCH_SUB: case LMR_OP_FETCH_MUL:
    case LMR_OP_FETCH_DIV: case LMR_OP_FETCH_REM: case LMR_OP_FETCH_AND:
    case LMR_OP_FETCH_OR: case LMR_OP_FETCH_XOR: case LMR_OP_LOAD:
    case LMR_OP_SWAP: case LMR_OP_GET: case LMR_OP_FETCH_SHL: case LMR_OP_FETCH_SHR:
        return LMR_RET_VALS;
    case LMR_OP_COMPARE_EXCHANGE: case LMR_OP_COMPARE_EXCHANGE_EPS:
        return LMR_RET_RESULT;
    default:
        return LMR_RET_NONE;
    }
}

int lmr_op_supported(uint32_t kind, uint32_t dtype, uint32_t op) {
    if (dtype >= LMR_NUM_DTYPES || op >= LMR_NUM_OPS || kind > LMR_KIND_READ_ONLY) return 0;
    if (kind == LMR_KIND_READ_ONLY) return op == LMR_OP_LOAD;
    if (dtype != LMR_F32 && dtype != LMR_F64) return 1;
    switch (op) {
    case LMR_OP_AND: case LMR_OP_FETCH_AND: case LMR_OP_OR: case LMR_OP_FETCH_OR:
    case LMR_OP_XOR: case LMR_OP_FETCH_XOR: case LMR_OP_COMPARE_EXCHANGE:
    case LMR_OP_SHL: case LMR_OP_FETCH_SHL: case LMR_OP_SHR: case LMR_OP_FETCH_SHR:
        return 0;
    default:
        return 1;
    }
}

// ---------------------------------------------------------------- pack
static lmr_status_t pack_common(lmr_ctx_t* ctx, const lmr_layout_t* layout, const uint64_t* d_gidx,
                                uint64_t n, const void* d_vals, uint32_t dtype, uint32_t index_size,
                                void* d_out_idx, void* d_out_vals, uint32_t* d_out_pos,
                                uint64_t* d_dest_counts, uint64_t* d_dest_offsets, bool stable,
                                lmr_stream_t stream) {
    if (!ctx || !valid_layout(layout) || !valid_iw(index_size) || dtype >= LMR_NUM_DTYPES ||
        !d_dest_offsets || n > 0xFFFFFFFFull || layout->num_pes > uint32_t(kMaxPackPes))
        return LMR_E_INVALID;
    if (n > 0 && (!d_gidx || !d_out_idx || (d_vals && !d_out_vals))) return LMR_E_INVALID;
    CtxExtra x = pack_scratch(ctx);
    PackArgs a;
    a.layout = *layout;
    a.gidx = d_gidx;
    a.vals = reinterpret_cast<const uint8_t*>(d_vals);
    a.val_bytes = uint32_t(dtype_bytes(int(dtype)));
    a.n = n;
    a.index_size = index_size;
    a.out_idx = reinterpret_cast<uint8_t*>(d_out_idx);
    a.out_vals = reinterpret_cast<uint8_t*>(d_out_vals);
    a.out_pos = d_out_pos;
    a.dest_counts = d_dest_counts;
    a.dest_offsets = d_dest_offsets;
    a.err = ctx->d_err;
    a.prof = ctx->prof;
    a.stable = stable;
    return hip_status(launch_pack(a, x.pack_counts, x.pack_partials, x.pack_total,
                                  reinterpret_cast<hipStream_t>(stream)));
}

lmr_status_t lmr_pack(lmr_ctx_t* ctx, const lmr_layout_t* layout, const uint64_t* d_gidx, uint64_t n,
                      const void* d_vals, uint32_t dtype, uint32_t index_size, void* d_out_idx,
                      void* d_out_vals, uint32_t* d_out_pos, uint64_t* d_dest_counts,
                      uint64_t* d_dest_offsets, lmr_stream_t stream) {
    return pack_common(ctx, layout, d_gidx, n, d_vals, dtype, index_size, d_out_idx, d_out_vals, d_out_pos,
                       d_dest_counts, d_dest_offsets, true, stream);
}

lmr_status_t lmr_pack_unordered(lmr_ctx_t* ctx, const lmr_layout_t* layout, const uint64_t* d_gidx,
                                uint64_t n, const void* d_vals, uint32_t dtype, uint32_t index_size,
                                void* d_out_idx, void* d_out_vals, uint32_t* d_out_pos,
                                uint64_t* d_dest_counts, uint64_t* d_dest_offsets, lmr_stream_t stream) {
    return pack_common(ctx, layout, d_gidx, n, d_vals, dtype, index_size, d_out_idx, d_out_vals, d_out_pos,
                       d_dest_counts, d_dest_offsets, false, stream);
}

lmr_status_t lmr_pack_regions(lmr_ctx_t* ctx, const lmr_layout_t* layout, const uint64_t* d_gidx, uint64_t n,
                              const void* d_vals, uint32_t dtype, uint32_t index_size, void* d_out_idx,
                              void* d_out_vals, uint64_t region_cap, uint32_t* d_fill, uint64_t* d_dest_counts,
                              lmr_stream_t stream) {
    if (!ctx || !valid_layout(layout) || !valid_iw(index_size) || dtype >= LMR_NUM_DTYPES || !d_fill ||
        !d_dest_counts || n > 0xFFFFFFFFull || layout->num_pes > uint32_t(kMaxPackPes) || region_cap == 0 ||
        uint64_t(layout->num_pes) * region_cap > 0xFFFFFFFFull)
        return LMR_E_INVALID;
    if (n > 0 && (!d_gidx || !d_out_idx || (d_vals && !d_out_vals))) return LMR_E_INVALID;
    PackArgs a;
    a.layout = *layout;
    a.gidx = d_gidx;
    a.vals = reinterpret_cast<const uint8_t*>(d_vals);
    a.val_bytes = uint32_t(dtype_bytes(int(dtype)));
    a.n = n;
    a.index_size = index_size;
    a.out_idx = reinterpret_cast<uint8_t*>(d_out_idx);
    a.out_vals = reinterpret_cast<uint8_t*>(d_out_vals);
    a.out_pos = nullptr;
    a.dest_counts = d_dest_counts;
    a.dest_offsets = nullptr;
    a.err = ctx->d_err;
    a.prof = ctx->prof;
    a.stable = false;
    return hip_status(launch_pack_free(a, d_fill, uint32_t(region_cap), reinterpret_cast<hipStream_t>(stream)));
}

// ---------------------------------------------------------------- reduce
lmr_status_t lmr_reduce(lmr_ctx_t* ctx, uint32_t dtype, uint32_t op, const void* d_shard, uint64_t len,
                        uint64_t* d_out, uint8_t* d_has, lmr_stream_t stream) {
    if (!ctx || dtype >= LMR_NUM_DTYPES || op > LMR_REDUCE_MIN || !d_out || (len > 0 && !d_shard))
        return LMR_E_INVALID;
    CtxExtra x = pack_scratch(ctx);
    return hip_status(launch_reduce(int(dtype), int(op), d_shard, len, d_out, d_has, x.red_part, x.red_has,
                                    reinterpret_cast<hipStream_t>(stream)));
}

// ---------------------------------------------------------------- apply
lmr_status_t lmr_apply_mvmi(lmr_ctx_t* ctx, const lmr_apply_desc_t* desc, const void* d_idx_vals,
                            uint64_t nbytes, uint32_t index_size, void* d_results, uint8_t* d_ok,
                            lmr_stream_t stream) {
    if (!ctx) return LMR_E_INVALID;
    index_size = am_index_width(index_size);
    lmr_status_t st = check_desc(desc);
    if (st != LMR_OK) return st;
    const uint32_t rb = lmr_record_bytes(index_size, desc->dtype);
    const uint64_t n = nbytes / rb;
    if (n == 0) return LMR_OK;
    if (!d_idx_vals || !desc->shard) return LMR_E_INVALID;
    ApplyArgs a = base_args(ctx, desc, d_results, d_ok);
    a.idx = reinterpret_cast<const uint8_t*>(d_idx_vals);
    a.idx_stride = rb;
    a.val = a.idx + lmr_record_val_offset(index_size, desc->dtype);
    a.val_stride = rb;
    a.n = n;
    return run_apply(ctx, desc, a, int(index_size), reinterpret_cast<hipStream_t>(stream));
}

lmr_status_t lmr_apply_svmi(lmr_ctx_t* ctx, const lmr_apply_desc_t* desc, const void* val,
                            const void* d_indices, uint64_t n, uint32_t index_size, void* d_results,
                            uint8_t* d_ok, lmr_stream_t stream) {
    if (!ctx || !val) return LMR_E_INVALID;
    index_size = am_index_width(index_size);
    lmr_status_t st = check_desc(desc);
    if (st != LMR_OK) return st;
    if (n == 0) return LMR_OK;
    if (!d_indices || !desc->shard) return LMR_E_INVALID;
    ApplyArgs a = base_args(ctx, desc, d_results, d_ok);
    a.idx = reinterpret_cast<const uint8_t*>(d_indices);
    a.idx_stride = index_size;
    a.val = nullptr;
    a.val_stride = 0;
    a.val_bits = load_scalar_bits(val, int(desc->dtype));
    a.n = n;
    return run_apply(ctx, desc, a, int(index_size), reinterpret_cast<hipStream_t>(stream));
}

lmr_status_t lmr_apply_mvsi(lmr_ctx_t* ctx, const lmr_apply_desc_t* desc, const void* d_vals,
                            uint64_t n, uint64_t index, void* d_results, uint8_t* d_ok,
                            lmr_stream_t stream) {
    if (!ctx) return LMR_E_INVALID;
    lmr_status_t st = check_desc(desc);
    if (st != LMR_OK) return st;
    if (n == 0) return LMR_OK;
    if (!d_vals || !desc->shard) return LMR_E_INVALID;
    ApplyArgs a = base_args(ctx, desc, d_results, d_ok);
    a.val = reinterpret_cast<const uint8_t*>(d_vals);
    a.val_stride = uint64_t(dtype_bytes(int(desc->dtype)));
    a.n = n;
    return hip_status(launch_apply_mvsi(int(desc->dtype), a, index,
                                        reinterpret_cast<hipStream_t>(stream)));
}

lmr_status_t lmr_apply_soa(lmr_ctx_t* ctx, const lmr_apply_desc_t* desc, const void* d_indices,
                           uint32_t index_size, const void* d_vals, const void* val, uint64_t n,
                           void* d_results, uint8_t* d_ok, lmr_stream_t stream) {
    if (!ctx || !valid_iw(index_size)) return LMR_E_INVALID;
    lmr_status_t st = check_desc(desc);
    if (st != LMR_OK) return st;
    if (n == 0) return LMR_OK;
    if (!d_indices || !desc->shard || (!d_vals && !val)) return LMR_E_INVALID;
    ApplyArgs a = base_args(ctx, desc, d_results, d_ok);
    a.idx = reinterpret_cast<const uint8_t*>(d_indices);
    a.idx_stride = index_size;
    a.val = reinterpret_cast<const uint8_t*>(d_vals);
    a.val_stride = d_vals ? uint64_t(dtype_bytes(int(desc->dtype))) : 0;
    a.val_bits = d_vals ? 0 : load_scalar_bits(val, int(desc->dtype));
    a.n = n;
    return run_apply(ctx, desc, a, int(index_size), reinterpret_cast<hipStream_t>(stream));
}

// ---------------------------------------------------------------- staged apply
lmr_status_t lmr_stage_begin(lmr_ctx_t* ctx, const lmr_apply_desc_t* desc) {
    if (!ctx || ctx->xdefer_open) return LMR_E_INVALID;      // (a deferred exchange session: flush first)
    lmr_status_t st = check_desc(desc);
    if (st != LMR_OK) return st;
    if (!desc->shard) return LMR_E_INVALID;
    if (!ctx->stage) ctx->stage = new StageState();
    StageState* S = ctx->stage;
    if (S->s.nreg > 0) return LMR_E_INVALID;          // the previous session was never finished
    S->open = true;
    S->desc = *desc;
    S->s = StageSession();
    S->s.a = base_args(ctx, desc, nullptr, nullptr);
    S->s.a.ret = int(lmr_op_ret_kind(desc->op));     // keep the result maps for every returning op
    S->s.free = ctx->rec_cap > 0 && stage_free_applies(int(desc->dtype), int(desc->op), S->s.a.ret,
                                                       desc->shard_len, ctx->rec_cap);
    S->s.dtype = int(desc->dtype);
    return LMR_OK;
}

lmr_status_t lmr_stage_soa(lmr_ctx_t* ctx, const void* d_indices, uint32_t index_size, const void* d_vals,
                           const void* val, uint64_t n, void* d_results, uint8_t* d_ok, lmr_stream_t stream) {
    if (!ctx || ctx->xdefer_open || !ctx->stage || !ctx->stage->open || !valid_iw(index_size)) return LMR_E_INVALID;
    if (n == 0) return LMR_OK;
    if (!d_indices || (!d_vals && !val)) return LMR_E_INVALID;
    StageState* S = ctx->stage;
    const lmr_apply_desc_t* d = &S->desc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    ApplyArgs a = base_args(ctx, d, d_results, d_ok);
    a.idx = reinterpret_cast<const uint8_t*>(d_indices);
    a.idx_stride = index_size;
    a.val = reinterpret_cast<const uint8_t*>(d_vals);
    a.val_stride = d_vals ? uint64_t(dtype_bytes(int(d->dtype))) : 0;
    a.val_bits = d_vals ? 0 : load_scalar_bits(val, int(d->dtype));
    a.n = n;
    const bool tiled = ctx->ws && ctx->rec_cap > 0 && d->strategy != LMR_STRATEGY_DIRECT &&
                       tiled_supported(int(d->dtype), d->shard_len) &&
                       !(d->strategy == LMR_STRATEGY_AUTO && n < 65536);
    if (!tiled) {                                                     // small stream: applied now,
        if (S->s.nreg > 0 && stage_pending_other_op(S->s, a)) {      // after earlier op phases
            const hipError_t e = launch_stage_finish(ctx_ws(ctx, ctx->rec_cap), S->s, s);
            if (e != hipSuccess) return hip_status(e);
        }
        return run_apply(ctx, d, a, int(index_size), s);
    }
    a.ret = S->s.a.ret;
    return hip_status(stage_records(ctx, S->s, a, int(d->dtype), int(index_size), 1, s));
}

lmr_status_t lmr_stage_op(lmr_ctx_t* ctx, uint32_t op, uint64_t cmp_bits, uint64_t eps_bits, lmr_stream_t stream) {
    if (!ctx || ctx->xdefer_open || !ctx->stage || !ctx->stage->open) return LMR_E_INVALID;
    StageState* S = ctx->stage;
    lmr_apply_desc_t d = S->desc;
    d.op = op;
    d.cmp_bits = cmp_bits;
    d.eps_bits = eps_bits;
    lmr_status_t st = check_desc(&d);
    if (st != LMR_OK) return st;
    const lmr_apply_desc_t& c = S->desc;
    if (c.op == op && c.cmp_bits == cmp_bits && c.eps_bits == eps_bits) return LMR_OK;
    if (S->s.nreg > 0) {
        // count-free regions share their bucket regions: apply them before the next op phase,
        // unless the session takes the wide path and nothing is partitioned yet: then they are
        // counted regions of its first phase (one partition and one sweep for every phase)
        if (S->s.free && !stage_free_to_wide(S->s, ctx->rec_cap)) {
            const hipError_t e = launch_stage_finish(ctx_ws(ctx, ctx->rec_cap), S->s,
                                                     reinterpret_cast<hipStream_t>(stream));
            if (e != hipSuccess) return hip_status(e);
        }
        S->s.switched = true;
    }
    S->desc = d;
    S->s.a = base_args(ctx, &d, nullptr, nullptr);
    S->s.a.ret = int(lmr_op_ret_kind(op));
    // count-free only while the session has had one op: a mixed session's later phases are
    // counted regions, so one sweep applies them all
    S->s.free = !S->s.switched && S->s.nreg == 0 && ctx->rec_cap > 0 &&
                stage_free_applies(int(d.dtype), int(op), S->s.a.ret, d.shard_len, ctx->rec_cap);
    return LMR_OK;
}

lmr_status_t lmr_stage_flush(lmr_ctx_t* ctx, lmr_stream_t stream) {
    if (!ctx || ctx->xdefer_open || !ctx->stage || !ctx->stage->open) return LMR_E_INVALID;
    StageSession& ss = ctx->stage->s;
    if (ss.parted == ss.nreg) return LMR_OK;
    return hip_status(launch_stage_partition(ctx_ws(ctx, ctx->rec_cap), ss,
                                             reinterpret_cast<hipStream_t>(stream)));
}

lmr_status_t lmr_stage_finish(lmr_ctx_t* ctx, lmr_stream_t stream) {
    if (!ctx || ctx->xdefer_open || !ctx->stage || !ctx->stage->open) return LMR_E_INVALID;
    StageState* S = ctx->stage;
    S->open = false;
    if (S->s.nreg == 0) return LMR_OK;
    return hip_status(launch_stage_finish(ctx_ws(ctx, ctx->rec_cap), S->s,
                                          reinterpret_cast<hipStream_t>(stream)));
}

// ---------------------------------------------------------------- results
lmr_status_t lmr_scatter_results(const void* d_in, const uint32_t* d_pos, uint64_t n,
                                 uint32_t elem_bytes, void* d_out, const uint8_t* d_ok_in,
                                 uint8_t* d_ok_out, lmr_stream_t stream) {
    if (n == 0) return LMR_OK;
    if (!d_in || !d_pos || !d_out) return LMR_E_INVALID;
    if (elem_bytes != 1 && elem_bytes != 2 && elem_bytes != 4 && elem_bytes != 8) return LMR_E_INVALID;
    return hip_status(launch_scatter_results(
        reinterpret_cast<const uint8_t*>(d_in), d_pos, n, elem_bytes, reinterpret_cast<uint8_t*>(d_out),
        (d_ok_in && d_ok_out) ? d_ok_in : nullptr, (d_ok_in && d_ok_out) ? d_ok_out : nullptr,
        nullptr, reinterpret_cast<hipStream_t>(stream)));
}

}  // extern "C"
