// lmr_window.hip — shards larger than one tiled window.
//
// The tiled apply partitions a record stream into at most kMaxTiles shard tiles
// (LDS histograms and tile tables are sized for that): 2^27 u64 / 2^28 u32
// elements. The reference puts no limit on a PE's shard (UnsafeArray::async_new,
// src/array/unsafe.rs:178-274), so a larger shard is cut into windows of
// kMaxTiles tiles: one partition pass groups the records by window (u32
// window-local offsets, values, and input positions for returned values), each
// window's records then take the tiled path on its slice of the shard, and
// returned values go back to input order (lmr_scatter_results).
//
// k_win_count  : per-window record counts (LDS histogram per block, one global
//                atomic per window per block); out-of-bounds records raise
//                LMR_ERRBIT_OOB and are dropped, as on every other path.
// k_win_scatter: each block reserves one contiguous run per window (atomic on
//                the window cursor) and writes its records there in LDS-ranked
//                order: long runs, coalesced writes.
#include "lmr_internal.hpp"
#include "lmr_device.hpp"
#include <algorithm>

namespace lmr {

namespace {

constexpr int kWinThreads = 1024;
constexpr int kWinRpt = 8;                  // records per thread per block
constexpr int kWinPerBlock = kWinThreads * kWinRpt;

template <int IW>
__device__ __forceinline__ uint64_t win_idx(const uint8_t* base, uint64_t stride, uint64_t k) {
    using I = typename idx_t<IW>::I;
    return uint64_t(*reinterpret_cast<const I*>(base + k * stride));
}

template <int IW>
__global__ __launch_bounds__(kWinThreads) void k_win_count(const uint8_t* idx, uint64_t stride, uint64_t n,
                                                            uint64_t shard_len, uint32_t shift, uint32_t W,
                                                            uint32_t* counts, uint32_t* err) {
    __shared__ uint32_t hist[kMaxWindows];
    if (threadIdx.x < W) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t b0 = uint64_t(blockIdx.x) * kWinPerBlock;
    bool oob = false;
#pragma unroll
    for (int r = 0; r < kWinRpt; r++) {
        const uint64_t k = b0 + uint64_t(r) * kWinThreads + threadIdx.x;
        if (k >= n) break;
        const uint64_t g = win_idx<IW>(idx, stride, k);
        if (g >= shard_len) { oob = true; continue; }
        atomicAdd(&hist[uint32_t(g >> shift)], 1u);
    }
    if (oob) raise_err(err, LMR_ERRBIT_OOB);
    __syncthreads();
    if (threadIdx.x < W && hist[threadIdx.x]) atomicAdd(&counts[threadIdx.x], hist[threadIdx.x]);
}

// offsets[w] = exclusive scan of counts (W <= kMaxWindows, one wave); cursor = offsets
__global__ void k_win_scan(const uint32_t* counts, uint32_t W, uint32_t* offsets, uint32_t* cursor) {
    if (threadIdx.x != 0) return;
    uint32_t s = 0;
    for (uint32_t w = 0; w < W; w++) {
        offsets[w] = s;
        cursor[w] = s;
        s += counts[w];
    }
    offsets[W] = s;
}

template <int IW, int VB>
__global__ __launch_bounds__(kWinThreads) void k_win_scatter(const uint8_t* idx, uint64_t stride, const uint8_t* val,
                                                              uint64_t val_stride, uint64_t n, uint64_t shard_len,
                                                              uint32_t shift, uint32_t W, uint32_t* cursor,
                                                              uint32_t* out_idx, uint8_t* out_val, uint32_t* out_pos) {
    using V = typename idx_t<VB>::I;
    __shared__ uint32_t hist[kMaxWindows], base[kMaxWindows];
    if (threadIdx.x < W) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t b0 = uint64_t(blockIdx.x) * kWinPerBlock;
    uint64_t g[kWinRpt];
    uint32_t rank[kWinRpt];
#pragma unroll
    for (int r = 0; r < kWinRpt; r++) {
        const uint64_t k = b0 + uint64_t(r) * kWinThreads + threadIdx.x;
        g[r] = ~uint64_t(0);
        if (k < n) {
            const uint64_t x = win_idx<IW>(idx, stride, k);
            if (x < shard_len) {
                g[r] = x;
                rank[r] = atomicAdd(&hist[uint32_t(x >> shift)], 1u);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < W) base[threadIdx.x] = hist[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], hist[threadIdx.x]) : 0;
    __syncthreads();
    const uint64_t mask = (uint64_t(1) << shift) - 1;
#pragma unroll
    for (int r = 0; r < kWinRpt; r++) {
        if (g[r] == ~uint64_t(0)) continue;
        const uint64_t k = b0 + uint64_t(r) * kWinThreads + threadIdx.x;
        const uint32_t slot = base[uint32_t(g[r] >> shift)] + rank[r];
        out_idx[slot] = uint32_t(g[r] & mask);
        if (out_val) reinterpret_cast<V*>(out_val)[slot] = *reinterpret_cast<const V*>(val + k * val_stride);
        if (out_pos) out_pos[slot] = uint32_t(k);
    }
}

template <typename F>
hipError_t win_dispatch(int iw, int vb, F&& f) {
    auto with_vb = [&](auto IWc) -> hipError_t {
        switch (vb) {
        case 1: return f(IWc, std::integral_constant<int, 1>{});
        case 2: return f(IWc, std::integral_constant<int, 2>{});
        case 4: return f(IWc, std::integral_constant<int, 4>{});
        case 8: return f(IWc, std::integral_constant<int, 8>{});
        default: return hipErrorInvalidValue;
        }
    };
    switch (iw) {
    case 1: return with_vb(std::integral_constant<int, 1>{});
    case 2: return with_vb(std::integral_constant<int, 2>{});
    case 4: return with_vb(std::integral_constant<int, 4>{});
    case 8: return with_vb(std::integral_constant<int, 8>{});
    default: return hipErrorInvalidValue;
    }
}

struct WinBuf {
    void* p = nullptr;
    size_t cap = 0;
    // grow-only; the old buffer may still be read by this context's earlier work, which is
    // ordered on the call's stream (the context contract, lamellar_gpu_ops.h)
    hipError_t need(size_t bytes, hipStream_t s) {
        if (bytes <= cap) return hipSuccess;
        if (p) {
            hipError_t e = hipStreamSynchronize(s);
            if (e != hipSuccess) return e;
            (void)hipFree(p);
            p = nullptr;
            cap = 0;
        }
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) { p = nullptr; return e; }
        cap = bytes;
        return hipSuccess;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
};

}  // namespace

struct WinState {
    WinBuf ctl, idx, val, pos, res, ok;
    uint32_t* h_counts = nullptr;          // pinned [kMaxWindows + 1] (offsets)
    hipEvent_t ev = nullptr;
};

void win_state_free(WinState* w) {
    if (!w) return;                                  // (lmr_ctx_destroy has drained the device)
    for (WinBuf* b : {&w->ctl, &w->idx, &w->val, &w->pos, &w->res, &w->ok}) b->release();
    if (w->h_counts) (void)hipHostFree(w->h_counts);
    if (w->ev) (void)hipEventDestroy(w->ev);
    delete w;
}

// the window (elements) of one tiled pass; a power of two
uint64_t tiled_window_len(int dtype) { return uint64_t(kMaxTiles) << tile_shift(dtype); }

hipError_t apply_windowed(lmr_ctx* ctx, const lmr_apply_desc_t* d, const ApplyArgs& a, int iw, hipStream_t s,
                          const WindowApplyFn& apply_one) {
    const int dtype = int(d->dtype);
    const int eb = dtype_bytes(dtype);
    const uint64_t win = tiled_window_len(dtype);
    uint32_t shift = 0;
    while ((uint64_t(1) << shift) < win) shift++;
    const uint64_t W64 = (d->shard_len + win - 1) / win;
    if (W64 > uint64_t(kMaxWindows)) return hipErrorNotSupported;
    const uint32_t W = uint32_t(W64);
    if (!ctx->win) ctx->win = new WinState();
    WinState* ws = ctx->win;
    hipError_t e = hipSuccess;
    if (!ws->h_counts) {
        e = hipHostMalloc(reinterpret_cast<void**>(&ws->h_counts), (kMaxWindows + 1) * 4, hipHostMallocDefault);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ws->ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    const bool ret = a.ret != LMR_RET_NONE && a.results;
    const bool want_ok = ret && a.ret == LMR_RET_RESULT && a.ok;
    // pieces: positions are u32 and the temp arrays grow to one piece
    const uint64_t piece = std::min<uint64_t>(a.n, std::max<uint64_t>(ctx->rec_cap, uint64_t(1) << 22));
    const uint64_t pc = std::min<uint64_t>(piece, uint64_t(1) << 31);
    if ((e = ws->ctl.need((3 * kMaxWindows + 1) * 4, s)) != hipSuccess ||
        (e = ws->idx.need(pc * 4 + 16, s)) != hipSuccess ||
        (a.val && (e = ws->val.need(pc * eb + 16, s)) != hipSuccess) ||
        (ret && (e = ws->pos.need(pc * 4 + 16, s)) != hipSuccess) ||
        (ret && (e = ws->res.need(pc * eb + 16, s)) != hipSuccess) ||
        (want_ok && (e = ws->ok.need(pc + 16, s)) != hipSuccess))
        return e;
    uint32_t* counts = reinterpret_cast<uint32_t*>(ws->ctl.p);
    uint32_t* offsets = counts + kMaxWindows;
    uint32_t* cursor = offsets + kMaxWindows + 1;
    for (uint64_t p0 = 0; p0 < a.n; p0 += pc) {
        const uint64_t m = std::min<uint64_t>(pc, a.n - p0);
        const uint8_t* idx = a.idx + p0 * a.idx_stride;
        const uint8_t* val = a.val ? a.val + p0 * a.val_stride : nullptr;
        const unsigned grid = unsigned((m + kWinPerBlock - 1) / kWinPerBlock);
        {
            ProfScope ps(a.prof, LMR_STAGE_WINDOW, s, m);
            if ((e = hipMemsetAsync(counts, 0, kMaxWindows * 4, s)) != hipSuccess) return e;
            e = win_dispatch(iw, eb, [&](auto IWc, auto VBc) -> hipError_t {
                constexpr int IW = decltype(IWc)::value, VB = decltype(VBc)::value;
                hipLaunchKernelGGL((k_win_count<IW>), dim3(grid), dim3(kWinThreads), 0, s, idx, a.idx_stride, m,
                                   d->shard_len, shift, W, counts, a.err);
                hipLaunchKernelGGL(k_win_scan, dim3(1), dim3(64), 0, s, counts, W, offsets, cursor);
                hipLaunchKernelGGL((k_win_scatter<IW, VB>), dim3(grid), dim3(kWinThreads), 0, s, idx, a.idx_stride,
                                   val, a.val_stride, m, d->shard_len, shift, W, cursor,
                                   reinterpret_cast<uint32_t*>(ws->idx.p), reinterpret_cast<uint8_t*>(val ? ws->val.p : nullptr),
                                   reinterpret_cast<uint32_t*>(ret ? ws->pos.p : nullptr));
                return hipGetLastError();
            });
            if (e != hipSuccess) return e;
        }
        // the host sizes each window's apply: one wait per piece
        if ((e = hipMemcpyAsync(ws->h_counts, offsets, (W + 1) * 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipEventRecord(ws->ev, s)) != hipSuccess || (e = hipEventSynchronize(ws->ev)) != hipSuccess)
            return e;
        for (uint32_t w = 0; w < W; w++) {
            const uint64_t o = ws->h_counts[w], c = uint64_t(ws->h_counts[w + 1]) - o;
            if (c == 0) continue;
            lmr_apply_desc_t dw = *d;
            dw.shard = static_cast<uint8_t*>(d->shard) + uint64_t(w) * win * eb;
            dw.shard_len = std::min<uint64_t>(win, d->shard_len - uint64_t(w) * win);
            ApplyArgs b = a;
            b.shard = dw.shard;
            b.shard_len = dw.shard_len;
            b.idx = reinterpret_cast<const uint8_t*>(ws->idx.p) + o * 4;
            b.idx_stride = 4;
            b.val = val ? reinterpret_cast<const uint8_t*>(ws->val.p) + o * eb : nullptr;
            b.val_stride = val ? uint64_t(eb) : 0;
            b.n = c;
            b.results = ret ? static_cast<uint8_t*>(ws->res.p) + o * eb : nullptr;
            b.ok = want_ok ? static_cast<uint8_t*>(ws->ok.p) + o : nullptr;
            if ((e = apply_one(&dw, b, s)) != hipSuccess) return e;
        }
        if (ret) {
            const uint64_t tot = ws->h_counts[W];
            e = launch_scatter_results(static_cast<const uint8_t*>(ws->res.p), reinterpret_cast<const uint32_t*>(ws->pos.p),
                                       tot, uint32_t(eb), static_cast<uint8_t*>(a.results) + p0 * eb,
                                       want_ok ? static_cast<const uint8_t*>(ws->ok.p) : nullptr,
                                       want_ok ? a.ok + p0 : nullptr, a.prof, s);
            if (e != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

}  // namespace lmr
