// lmr_apply.hip — gfx950 apply kernels for batched element ops.
//
// Replaces the element loops of the reference's generated AM exec bodies
// (impl/src/array_ops.rs:203-250 loop shapes, :863-1408 bodies):
//   * k_apply_direct : one device-scope atomic RMW per record (any op/type);
//                      the path for small op buffers (one AM of ~6250 records).
//   * k_apply_mvsi   : many values at one index, applied in buffer order as
//                      one atomic block (array_ops.rs:235-250: lock once, loop).
//   * tiled path     : k_bin_count -> scan -> k_bin_scatter -> k_tile_apply.
//                      Records are counting-sorted into 64 KiB shard tiles; one
//                      workgroup owns a tile, stages it in LDS, applies every
//                      record with LDS atomics (ds_add_u64, ds_cmpst_b64, ...)
//                      and writes the tile back once: random 8-B HBM RMWs become
//                      streaming reads of the binned records plus one coalesced
//                      read+write of the shard.
#include "lmr_internal.hpp"
#include "lmr_device.hpp"
#include "lmr_tile.hpp"
#include <stdlib.h>
#include <algorithm>

// k_coarse_free loads two consecutive u64 records per thread with 16-B loads (0: one at a time)
#ifndef LMR_COARSE_PAIRS
#define LMR_COARSE_PAIRS 1
#endif
constexpr bool kCoarsePairs = LMR_COARSE_PAIRS != 0;

namespace lmr {

template <typename T>
__device__ __forceinline__ T load_val(const ApplyArgs& a, uint64_t k) {
    if (a.val) return *reinterpret_cast<const T*>(a.val + k * a.val_stride);
    return from_bits<T>(typename bits_of<T>::U(a.val_bits));
}

template <int IW>
__device__ __forceinline__ uint64_t load_idx(const uint8_t* base, uint64_t stride, uint64_t k) {
    using I = typename idx_t<IW>::I;
    return uint64_t(*reinterpret_cast<const I*>(base + k * stride));
}

// ------------------------------------------------------------------ direct
template <typename T, int IW>
__global__ __launch_bounds__(256) void k_apply_direct(ApplyArgs a) {
    using U = typename bits_of<T>::U;
    T* shard = reinterpret_cast<T*>(a.shard);
    const T cmp = from_bits<T>(U(a.cmp_bits)), eps = from_bits<T>(U(a.eps_bits));
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < a.n; k += stride) {
        uint64_t idx = load_idx<IW>(a.idx, a.idx_stride, k);
        T v = load_val<T>(a, k);
        if (idx >= a.shard_len) {
            raise_err(a.err, LMR_ERRBIT_OOB);
            continue;
        }
        uint8_t ok = 0;
        T r = rmw_global<T>(shard + idx, a.op, a.kind, v, cmp, eps, ok, a.err);
        if (a.ret != LMR_RET_NONE) reinterpret_cast<T*>(a.results)[k] = r;
        if (a.ret == LMR_RET_RESULT) a.ok[k] = ok;
    }
}

// ------------------------------------------------------------------ MVSI
// One thread walks the values in order on a register copy of the element and
// publishes the final value with one CAS (retrying the whole block if another
// kernel raced on the element): the block of values is applied atomically, as
// under the reference's per-AM lock.
template <typename T>
__global__ __launch_bounds__(64) void k_apply_mvsi(ApplyArgs a, uint64_t index) {
    using U = typename bits_of<T>::U;
    if (threadIdx.x != 0 || a.n == 0) return;
    if (index >= a.shard_len) { raise_err(a.err, LMR_ERRBIT_OOB); return; }
    const T cmp = from_bits<T>(U(a.cmp_bits)), eps = from_bits<T>(U(a.eps_bits));
    T* p = reinterpret_cast<T*>(a.shard) + index;
    const bool ret = a.ret != LMR_RET_NONE;
    if constexpr (sizeof(T) >= 4) {
        U cur = __hip_atomic_load(reinterpret_cast<U*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (true) {
            T s = from_bits<T>(cur);
            uint32_t errs = 0;
            for (uint64_t k = 0; k < a.n; k++) {
                T v = load_val<T>(a, k), nw, r;
                uint8_t ok = 0;
                uint32_t eb = 0;
                if (op_math<T>(a.op, a.kind, s, v, cmp, eps, nw, r, ok, eb)) s = nw;
                else errs |= eb;
                if (ret) reinterpret_cast<T*>(a.results)[k] = r;
                if (a.ret == LMR_RET_RESULT) a.ok[k] = ok;
            }
            U expected = cur;
            if (to_bits(s) == cur ||
                __hip_atomic_compare_exchange_strong(reinterpret_cast<U*>(p), &expected, to_bits(s),
                                                     __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)) {
                if (errs) raise_err(a.err, errs);
                return;
            }
            cur = expected;
        }
    } else {
        uintptr_t ad = reinterpret_cast<uintptr_t>(p);
        uint32_t* wp = reinterpret_cast<uint32_t*>(ad & ~uintptr_t(3));
        const unsigned sh = unsigned(ad & 3) * 8;
        const uint32_t mask = uint32_t((1u << (8 * sizeof(T))) - 1u) << sh;
        uint32_t cur = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (true) {
            T s = T(U((cur & mask) >> sh));
            uint32_t errs = 0;
            for (uint64_t k = 0; k < a.n; k++) {
                T v = load_val<T>(a, k), nw, r;
                uint8_t ok = 0;
                uint32_t eb = 0;
                if (op_math<T>(a.op, a.kind, s, v, cmp, eps, nw, r, ok, eb)) s = nw;
                else errs |= eb;
                if (ret) reinterpret_cast<T*>(a.results)[k] = r;
                if (a.ret == LMR_RET_RESULT) a.ok[k] = ok;
            }
            uint32_t nb = (cur & ~mask) | (uint32_t(U(s)) << sh);
            uint32_t expected = cur;
            if (nb == cur ||
                __hip_atomic_compare_exchange_strong(wp, &expected, nb, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                if (errs) raise_err(a.err, errs);
                return;
            }
            cur = expected;
        }
    }
}

// ------------------------------------------------------------------ tiled
struct BinArgs {
    const uint8_t* idx;
    uint64_t idx_stride;
    const uint8_t* val;
    uint64_t val_stride;
    uint64_t n;
    uint64_t shard_len;
    uint64_t chunk;        // records per block
    int tile_shift;
    uint32_t num_tiles;
    uint32_t G;
    uint32_t* counts;      // [num_tiles * G], tile-major
    uint16_t* bin_lidx;
    uint8_t* bin_val;
    uint32_t* rpos;        // [n] record k -> binned position (~0 = out of bounds); null when nothing is returned
    uint32_t* err;
};

template <int IW>
__global__ __launch_bounds__(kBinBlock) void k_bin_count(BinArgs b) {
    extern __shared__ uint32_t hist[];
    for (uint32_t t = threadIdx.x; t < b.num_tiles; t += blockDim.x) hist[t] = 0;
    __syncthreads();
    const uint64_t lo = uint64_t(blockIdx.x) * b.chunk;
    const uint64_t hi = min(lo + b.chunk, b.n);
    bool oob = false;
    constexpr int U = 4;                      // U loads in flight per thread before the LDS atomics
    for (uint64_t k0 = lo + threadIdx.x; k0 < hi; k0 += U * uint64_t(blockDim.x)) {
        uint64_t ix[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t k = k0 + uint64_t(j) * blockDim.x;
            ix[j] = k < hi ? load_idx<IW>(b.idx, b.idx_stride, k) : ~uint64_t(0);
        }
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t k = k0 + uint64_t(j) * blockDim.x;
            if (k >= hi) continue;
            if (ix[j] >= b.shard_len) { oob = true; continue; }
            atomicAdd(&hist[uint32_t(ix[j] >> b.tile_shift)], 1u);
        }
    }
    if (oob) raise_err(b.err, LMR_ERRBIT_OOB);
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < b.num_tiles; t += blockDim.x)
        b.counts[uint64_t(t) * b.G + blockIdx.x] = hist[t];
}

template <int IW, int VB>
__global__ __launch_bounds__(kBinBlock) void k_bin_scatter(BinArgs b) {
    using V = typename idx_t<VB>::I;   // raw value bits of VB bytes
    extern __shared__ uint32_t cursor[];
    for (uint32_t t = threadIdx.x; t < b.num_tiles; t += blockDim.x)
        cursor[t] = b.counts[uint64_t(t) * b.G + blockIdx.x];
    __syncthreads();
    const uint64_t lo = uint64_t(blockIdx.x) * b.chunk;
    const uint64_t hi = min(lo + b.chunk, b.n);
    const uint32_t lmask = (1u << b.tile_shift) - 1u;
    for (uint64_t k = lo + threadIdx.x; k < hi; k += blockDim.x) {
        uint64_t idx = load_idx<IW>(b.idx, b.idx_stride, k);
        if (idx >= b.shard_len) {
            if (b.rpos) b.rpos[k] = 0xFFFFFFFFu;
            continue;
        }
        uint32_t pos = atomicAdd(&cursor[uint32_t(idx >> b.tile_shift)], 1u);
        b.bin_lidx[pos] = uint16_t(uint32_t(idx) & lmask);
        if (b.val) reinterpret_cast<V*>(b.bin_val)[pos] = *reinterpret_cast<const V*>(b.val + k * b.val_stride);
        if (b.rpos) b.rpos[k] = pos;
    }
}

__global__ void k_tile_starts(const uint32_t* counts, uint32_t num_tiles, uint32_t G,
                              const uint32_t* total, uint32_t* tile_start) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < num_tiles) tile_start[t] = counts[uint64_t(t) * G];
    if (t == num_tiles) tile_start[t] = *total;
}

// ---- two-level partition (num_tiles > kFine) --------------------------------
// A one-pass scatter into thousands of tiles writes every record to a different
// cache line (measured: ~20 G random transactions/s on MI355X, the same limit
// as random atomics). Two LDS-staged passes keep every write a contiguous run:
//   coarse pass : each block sorts rounds of kRound records by coarse bucket
//                 (kFine tiles) in LDS and writes ~kRound/C-record runs;
//   fine pass   : block (c, g) sorts block g's coarse-c records by tile and
//                 writes ~kRound/kFine-record runs at their final positions.
// Final positions are the single-level ones (tile-major [t][g] exclusive scan of
// the per-block tile counts), so the tile apply is unchanged.
constexpr int kFine = 128;
constexpr int kFineShift = 7;
constexpr int kMaxCoarse = kMaxTiles / kFine;

struct PartArgs {
    const uint8_t* idx;
    uint64_t idx_stride;
    const uint8_t* val;
    uint64_t val_stride;
    uint64_t n;
    uint64_t shard_len;
    uint64_t chunk;
    int tile_shift;
    uint32_t num_tiles;
    uint32_t G;
    uint32_t C;
    const uint32_t* fine_off;     // exclusive-scanned counts [num_tiles][G]
    const uint32_t* tile_start;   // [num_tiles + 1]
    uint32_t* coarse_off;         // [C * G + 1]
    uint32_t* tmp_idx;
    uint8_t* tmp_val;
    uint32_t* qpos;               // [n] record k -> temp position (~0 = out of bounds); null: no results
    uint16_t* bin_lidx;
    uint8_t* bin_val;
    uint32_t* rpos;               // [total] temp position -> binned position; null: no results
    uint32_t* counts;             // count-free partition: [G][num_tiles] per-block tile count rows
    uint32_t* err;
    // count-free partition (k_coarse_free / k_fine_free)
    uint32_t* ff_fill;            // [C * kSegs] records reserved in each segment of every bucket region
    uint32_t* ff_tfill;           // [num_tiles] records reserved in each tile
    uint32_t capc;                // records per coarse bucket region (kXcds sub-regions + a shared area)
    uint64_t tmp_cap;             // temp arrays' capacity (records)
    int spill;                    // 1: records beyond a full bucket region are applied to the shard
                                  //    at once (device atomics); 0: they are dropped (never used)
    int accumulate;               // 1: add this launch's tile counts to the rows (staged regions)
    int xcd_swz;                  // 1: k_fine_free's ranges dealt by xcd_block (one bucket's blocks share an XCD)
    void* shard;                  // spill target
    int op;
    uint64_t val_bits;            // the scalar value when val is null (spilled records)
    // staged regions: coarse_off holds k_ccount's raw (bucket, block) counts; k_coarse_scatter
    // derives its cursors from them and block 0 stores the bucket starts [C + 1] and the
    // in-bounds total (no scan launch between the two passes)
    uint32_t* bstart_out;         // non-null: coarse_off is raw counts
    uint32_t* total_out;
    uint32_t csub;                // staged regions: k_ccount blocks per producer block (count rows C x G*csub)
    uint32_t* trows;              // staged regions: [G * csub][num_tiles] per-count-block tile counts (k_ccount)
    uint32_t* ttot;               // staged regions: [num_tiles] tile totals (k_coarse_scatter folds the rows)
    uint32_t* tfill;              // staged regions: [num_tiles] fine-pass fill counters (zeroed by k_coarse_scatter)
    // staged returning regions, round-wise second un-partition gather (crt non-null): qpos holds
    // as u16 record k's position in its coarse round's LDS staging (0xFFFF: out of bounds; the u16
    // array starts where the region's u32 map would), and each round's bucket runs are
    // recorded, crt[g * rpb + round][c] = {temp start, length}
    uint32_t* crt;
    uint32_t rpb;                 // rounds per producer block
};

__device__ __forceinline__ void small_excl_scan(const uint32_t* hist, uint32_t* base, uint32_t m, uint32_t* tot);

// cursor[c] = (records of buckets < c) + (records of bucket c in blocks < g), from the raw
// per-(bucket, block) counts cnt[c * G + g'] (C <= 128, G <= kMaxBinBlocks): wave w folds
// buckets w, w + 16, ...; block 0 also stores the bucket starts and the total
__device__ void coarse_cursors_from_counts(const PartArgs& p, uint32_t g, uint32_t* cursor, uint32_t* tot_s,
                                           uint32_t* pre_s, uint32_t* tot_scan, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t S = p.csub ? p.csub : 1u, GS = p.G * S, gs = g * S;
    for (uint32_t c = wv; c < p.C; c += blockDim.x >> 6) {
        const uint32_t* row = p.coarse_off + uint64_t(c) * GS;
        uint32_t all = 0, pre = 0;
        for (uint32_t j = lane; j < GS; j += 64) {
            const uint32_t v = row[j];
            all += v;
            pre += j < gs ? v : 0u;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            all += __shfl_xor(all, o, 64);
            pre += __shfl_xor(pre, o, 64);
        }
        if (lane == 0) {
            tot_s[c] = all;
            pre_s[c] = pre;
        }
    }
    __syncthreads();
    small_excl_scan(tot_s, tot_scan, p.C, total);
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < p.C; c += blockDim.x) cursor[c] = tot_scan[c] + pre_s[c];
    if (g == 0) {
        for (uint32_t c = threadIdx.x; c < p.C; c += blockDim.x) p.bstart_out[c] = tot_scan[c];
        if (threadIdx.x == 0) {
            p.bstart_out[p.C] = *total;
            *p.total_out = *total;
        }
    }
}

// coarse_off[c][g] = start of block g's coarse-c records in the temp buffer
//                  = tile_start[c*kFine] + sum_{t in c} (fine_off[t][g] - tile_start[t])
__global__ void k_coarse_offsets(PartArgs p) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t cg = uint64_t(p.C) * p.G;
    if (i < cg) {
        const uint32_t c = uint32_t(i / p.G), g = uint32_t(i % p.G);
        const uint32_t t0 = c * kFine, t1 = min(t0 + kFine, p.num_tiles);
        uint32_t s = p.tile_start[t0];
#pragma unroll 16
        for (uint32_t t = t0; t < t1; t++) s += p.fine_off[uint64_t(t) * p.G + g] - p.tile_start[t];
        p.coarse_off[i] = s;
    } else if (i == cg) {
        p.coarse_off[i] = p.tile_start[p.num_tiles];
    }
}

// exclusive scan of hist[0..m) (m <= 128) into base[], total into *tot; wave 0 only
__device__ __forceinline__ void small_excl_scan(const uint32_t* hist, uint32_t* base, uint32_t m,
                                                uint32_t* tot) {
    if (threadIdx.x < 64) {
        const uint32_t l = threadIdx.x;
        uint32_t a = (2 * l < m) ? hist[2 * l] : 0u, b = (2 * l + 1 < m) ? hist[2 * l + 1] : 0u;
        uint32_t x = a + b, inc = x;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            uint32_t y = __shfl_up(inc, d, 64);
            if (int(l) >= d) inc += y;
        }
        uint32_t ex = inc - x;
        if (2 * l < m) base[2 * l] = ex;
        if (2 * l + 1 < m) base[2 * l + 1] = ex + a;
        if (l == 63) *tot = inc;
    }
}

// Both passes are software-pipelined: the next round's global loads are issued
// into registers right after the current round is staged in LDS, so they are
// in flight while the staged round is written out.
// RPT records per thread per round (kRound = RPT * 1024 records staged in LDS).
template <int IW, int VB, int RPT>
__device__ __forceinline__ void coarse_scatter_body(const PartArgs& p, const uint32_t g) {
    using V = typename idx_t<VB>::I;
    constexpr uint32_t kRound = RPT * 1024;
    static_assert(kRound < 0xFFFFu, "round staging positions are u16");
    __shared__ uint32_t hist[kMaxCoarse], base[kMaxCoarse], cursor[kMaxCoarse], tot;
    __shared__ uint32_t s_idx[kRound];
    __shared__ V s_val[kRound];
    const uint32_t C = p.C;
    const int cshift = p.tile_shift + kFineShift;
    if (p.bstart_out) {
        coarse_cursors_from_counts(p, g, cursor, hist, base, reinterpret_cast<uint32_t*>(s_idx), &tot);
        // tile totals of the region: block g folds every count row over its slice of tpb tiles
        // (thread = (row group, tile); rows read in tpb-word segments), the fine pass turns them
        // into tile starts; the slice's fill counters are cleared
        const uint32_t rows = p.G * (p.csub ? p.csub : 1u);
        const uint32_t tpb = (p.num_tiles + p.G - 1) / p.G;
        const uint32_t t_lo = g * tpb, t_hi = min(t_lo + tpb, p.num_tiles);
        uint32_t* part = reinterpret_cast<uint32_t*>(s_val);   // [1024] partial sums (LDS round buffer, free here)
        for (uint32_t t0 = t_lo; t0 < t_hi; t0 += 1024) {
            const uint32_t nt = min(1024u, t_hi - t0);
            const uint32_t ng = 1024 / nt;                     // row groups
            const uint32_t j = threadIdx.x % nt, rg = threadIdx.x / nt;
            uint32_t x = 0;
            if (rg < ng)
                for (uint32_t b = rg; b < rows; b += ng) x += p.trows[uint64_t(b) * p.num_tiles + t0 + j];
            part[threadIdx.x] = x;
            __syncthreads();
            if (threadIdx.x < nt) {
                uint32_t sum = 0;
                for (uint32_t r = 0; r < ng; r++) sum += part[r * nt + threadIdx.x];
                p.ttot[t0 + threadIdx.x] = sum;
                p.tfill[t0 + threadIdx.x] = 0;
            }
            __syncthreads();
        }
    } else
        for (uint32_t c = threadIdx.x; c < C; c += blockDim.x) cursor[c] = p.coarse_off[uint64_t(c) * p.G + g];
    const uint64_t lo = uint64_t(g) * p.chunk;
    const uint64_t hi = min(lo + p.chunk, p.n);
    uint64_t m_raw[RPT];
    V m_val[RPT];
    auto load_round = [&](uint64_t r0) {
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint64_t k = r0 + uint64_t(j) * 1024 + threadIdx.x;
            const bool in = k < hi;
            m_raw[j] = in ? load_idx<IW>(p.idx, p.idx_stride, k) : ~uint64_t(0);
            m_val[j] = (in && p.val) ? *reinterpret_cast<const V*>(p.val + k * p.val_stride) : V(0);
        }
    };
    load_round(lo);
    for (uint64_t r0 = lo; r0 < hi; r0 += kRound) {
        for (uint32_t c = threadIdx.x; c < C; c += blockDim.x) hist[c] = 0;
        __syncthreads();
        uint32_t m_rank[RPT], m_c[RPT];
        bool m_ok[RPT];
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            m_ok[j] = m_raw[j] < p.shard_len;
            m_c[j] = m_ok[j] ? uint32_t(m_raw[j] >> cshift) : 0u;
            if (m_ok[j]) m_rank[j] = atomicAdd(&hist[m_c[j]], 1u);
        }
        __syncthreads();
        small_excl_scan(hist, base, C, &tot);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint64_t k = r0 + uint64_t(j) * 1024 + threadIdx.x;
            if (!m_ok[j]) {
                if (p.qpos && k < hi) {
                    if (p.crt) reinterpret_cast<uint16_t*>(p.qpos)[k] = 0xFFFFu;
                    else p.qpos[k] = 0xFFFFFFFFu;
                }
                continue;
            }
            const uint32_t q = base[m_c[j]] + m_rank[j];
            s_idx[q] = uint32_t(m_raw[j]);
            s_val[q] = m_val[j];
            if (p.qpos) {                                  // coalesced in k
                if (p.crt) reinterpret_cast<uint16_t*>(p.qpos)[k] = uint16_t(q);
                else p.qpos[k] = cursor[m_c[j]] + m_rank[j];
            }
        }
        if (p.crt && threadIdx.x < kMaxCoarse) {
            uint32_t* rr = p.crt + (uint64_t(g) * p.rpb + (r0 - lo) / kRound) * (2 * kMaxCoarse) + 2 * threadIdx.x;
            const bool in = threadIdx.x < C;
            rr[0] = in ? cursor[threadIdx.x] : 0u;
            rr[1] = in ? hist[threadIdx.x] : 0u;
        }
        if (r0 + kRound < hi) load_round(r0 + kRound);     // prefetch the next round
        __syncthreads();
        if (p.val)
            bucket_writeout(hist, base, cursor, C, [&](uint32_t q, uint32_t dst) {
                p.tmp_idx[dst] = s_idx[q];
                reinterpret_cast<V*>(p.tmp_val)[dst] = s_val[q];
            });
        else
            bucket_writeout(hist, base, cursor, C, [&](uint32_t q, uint32_t dst) { p.tmp_idx[dst] = s_idx[q]; });
        __syncthreads();
        for (uint32_t c = threadIdx.x; c < C; c += blockDim.x) cursor[c] += hist[c];
    }
}

template <int IW, int VB, int RPT>
__global__ __launch_bounds__(1024) void k_coarse_scatter(PartArgs p) {
    coarse_scatter_body<IW, VB, RPT>(p, blockIdx.x);
}

// Persistent over (coarse bucket c, producer block g) segments, a contiguous
// record-balanced range of them per block; the first round of the next segment
// is prefetched while the current segment's last round is written out.
template <int VB, int RPT>
__global__ __launch_bounds__(1024) void k_fine_scatter(PartArgs p) {
    using V = typename idx_t<VB>::I;
    constexpr uint32_t kRound = RPT * 1024;
    __shared__ uint32_t hist[kFine], base[kFine], cursor[kFine], tot;
    __shared__ uint16_t s_l[kRound];
    __shared__ V s_val[kRound];
    const uint32_t lmask = (1u << p.tile_shift) - 1u;
    const uint32_t nseg = p.C * p.G;
    uint32_t m_idx[RPT];
    V m_val[RPT];
    auto load_round = [&](uint32_t r0, uint32_t hi) {
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint32_t k = r0 + uint32_t(j) * 1024 + threadIdx.x;
            const bool in = k < hi;
            m_idx[j] = in ? p.tmp_idx[k] : 0xFFFFFFFFu;
            m_val[j] = (in && p.tmp_val) ? reinterpret_cast<const V*>(p.tmp_val)[k] : V(0);
        }
    };
    // Block b owns the segments whose records start in [total*b/B, total*(b+1)/B)
    // (coarse_off is monotone in cg = c*G + g): a contiguous run of producers
    // g of one bucket, so each tile's output run keeps growing from one CU (one
    // XCD's L2 merges its partial lines) and work is balanced by records.
    const uint64_t total_recs = p.coarse_off[nseg] - p.coarse_off[0];
    auto seg_lower_bound = [&](uint64_t target) {
        uint32_t lo_s = 0, hi_s = nseg;
        while (lo_s < hi_s) {
            const uint32_t mid = (lo_s + hi_s) >> 1;
            if (uint64_t(p.coarse_off[mid]) < target) lo_s = mid + 1; else hi_s = mid;
        }
        return lo_s;
    };
    const uint64_t rec_lo = p.coarse_off[0];
    const uint32_t cg_begin = seg_lower_bound(rec_lo + total_recs * blockIdx.x / gridDim.x);
    const uint32_t cg_end = (blockIdx.x + 1 == gridDim.x) ? nseg
                                                          : seg_lower_bound(rec_lo + total_recs * (blockIdx.x + 1) / gridDim.x);
    uint32_t cg = cg_begin;
    // segment cg's tile cursors (threads f < 128 hold tile f's), prefetched with the
    // segment's first round so the strided fine_off loads are off the critical path
    uint32_t pf_cur = 0;
    auto load_cursor = [&](uint32_t cgn) {
        const uint32_t cn = cgn / p.G, gn = cgn % p.G, tn = cn * kFine;
        if (threadIdx.x < min(uint32_t(kFine), p.num_tiles - tn))
            pf_cur = p.fine_off[uint64_t(tn + threadIdx.x) * p.G + gn];
    };
    // Consecutive segments (c, g..g') of one bucket are one stream: tile t's records
    // of producers g..g' own the contiguous range [fine_off[t][g], fine_off[t][g'+1])
    // and their order inside it is free, so rounds run across segment boundaries
    // (no partial round per segment, one cursor load per bucket and block).
    auto range_end = [&](uint32_t c0) { return min(cg_end, (c0 / p.G + 1) * p.G); };
    if (cg < cg_end) {
        load_round(p.coarse_off[cg], p.coarse_off[range_end(cg)]);
        load_cursor(cg);
    }
    for (uint32_t ce; cg < cg_end; cg = ce) {
        ce = range_end(cg);
        const uint32_t c = cg / p.G;
        const uint32_t t0 = c * kFine;
        const uint32_t nf = min(uint32_t(kFine), p.num_tiles - t0);
        const uint32_t lo = p.coarse_off[cg], hi = p.coarse_off[ce];
        if (lo == hi) {   // empty range: its (all-invalid) prefetch is replaced by the next one's
            if (ce < cg_end) {
                load_round(p.coarse_off[ce], p.coarse_off[range_end(ce)]);
                load_cursor(ce);
            }
            continue;
        }
        if (threadIdx.x < nf) cursor[threadIdx.x] = pf_cur;
        for (uint32_t r0 = lo; r0 < hi; r0 += kRound) {
            for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x) hist[f] = 0;
            __syncthreads();
            // (tile, validity) recomputed from m_idx and the position: no per-record arrays
            // beyond the ranks (51 -> 3 spilled VGPRs for 8-byte values; fine pass
            // 0.546 -> 0.522 ms on C3, same box)
            uint32_t m_rank[RPT];
#pragma unroll
            for (int j = 0; j < RPT; j++)
                m_rank[j] = (r0 + uint32_t(j) * 1024 + threadIdx.x < hi)
                                ? atomicAdd(&hist[(m_idx[j] >> p.tile_shift) - t0], 1u) : 0u;
            __syncthreads();
            small_excl_scan(hist, base, nf, &tot);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < RPT; j++) {
                const uint32_t k = r0 + uint32_t(j) * 1024 + threadIdx.x;
                if (k >= hi) continue;
                const uint32_t f = (m_idx[j] >> p.tile_shift) - t0;
                const uint32_t q = base[f] + m_rank[j];
                s_l[q] = uint16_t(m_idx[j] & lmask);
                s_val[q] = m_val[j];
                if (p.rpos) p.rpos[k] = cursor[f] + m_rank[j];
            }
            if (r0 + kRound < hi) {
                load_round(r0 + kRound, hi);
            } else if (ce < cg_end) {
                load_round(p.coarse_off[ce], p.coarse_off[range_end(ce)]);
                load_cursor(ce);
            }
            __syncthreads();
            V* bv = reinterpret_cast<V*>(p.bin_val);
            if (p.tmp_val)
                bucket_writeout(hist, base, cursor, nf, [&](uint32_t q, uint32_t dst) {
                    p.bin_lidx[dst] = s_l[q];
                    bv[dst] = s_val[q];
                });
            else
                bucket_writeout(hist, base, cursor, nf, [&](uint32_t q, uint32_t dst) { p.bin_lidx[dst] = s_l[q]; });
            __syncthreads();
            for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x) cursor[f] += hist[f];
        }
        __syncthreads();
    }
}

// ---- count-free two-level partition (order-insensitive ops) -----------------
// For ops whose result does not depend on the order records are applied in
// (wrapping integer add / sub / mul / and / or / xor) with nothing returned, the
// records of one tile need not keep their input order, and the count pass (a
// full read of the indices, 8 B/op at 1 PE) is dropped:
//   k_coarse_free : as k_coarse_scatter, but each round reserves its bucket runs
//                   with one atomicAdd per bucket on that bucket's fill counter,
//                   inside a fixed region of capc records per bucket; on the way
//                   it counts the records of every tile in LDS (one row per block)
//   k_free_tile_totals + scan : exact tile starts from those rows
//   k_fine_free   : as k_fine_scatter over record-balanced ranges of the bucket
//                   regions; each round reserves its tile runs with one atomicAdd
//                   per tile on that tile's fill counter
// A bucket that outgrows its region (a batch concentrated on a few 8 MB stretches
// of the shard) applies its extra records to the shard at once with device atomics
// (spill): the op is order-insensitive, so any split between the two is exact.
// Bucket region layout (count-free): kXcds sub-regions of capc / 16 slots, one per XCD, then
// a shared area (the rest, ~capc / 2). A block appends its runs to its own XCD's sub-region,
// so the runs of one bucket written through one L2 are adjacent there and their partial lines
// merge in it; what a sub-region cannot take goes to the shared area (skewed streams, e.g.
// each block's records on a few buckets), and past that to the spill.
constexpr uint32_t kXcds = 8;
constexpr uint32_t kSegs = kXcds + 1;                 // segments per bucket region
__host__ __device__ inline uint32_t sub_cap(uint32_t capc) { return capc / 16; }
__host__ __device__ inline uint32_t seg_base(uint32_t capc, uint32_t x) { return x * sub_cap(capc); }
__host__ __device__ inline uint32_t seg_cap(uint32_t capc, uint32_t x) {
    return x < kXcds ? sub_cap(capc) : capc - kXcds * sub_cap(capc);
}
__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & (kXcds - 1); }  // HW_REG_XCC_ID

template <int IW, int VB, int RPT, bool PAIRS>
__device__ __forceinline__ void coarse_free_body(const PartArgs& p, const uint32_t g) {
    using V = typename idx_t<VB>::I;
    constexpr uint32_t kRound = RPT * 1024;
    extern __shared__ uint32_t th[];                   // [num_tiles] this block's tile counts
    __shared__ uint32_t hist[kMaxCoarse], base[kMaxCoarse], tot;
    __shared__ uint32_t seg_a[kMaxCoarse], len_a[kMaxCoarse], seg_b[kMaxCoarse];   // a round's run: 2 pieces
    __shared__ uint32_t s_spill;                      // this round has records past their bucket region
    __shared__ uint32_t s_idx[kRound];
    __shared__ V s_val[kRound];
    const uint32_t C = p.C;
    const uint32_t xcc = xcc_id();
    const uint32_t capx = sub_cap(p.capc), caps = seg_cap(p.capc, kXcds);
    const int cshift = p.tile_shift + kFineShift;
    for (uint32_t t = threadIdx.x; t < p.num_tiles; t += blockDim.x) th[t] = 0;
    const uint64_t lo = uint64_t(g) * p.chunk;
    const uint64_t hi = min(lo + p.chunk, p.n);
    uint64_t m_raw[RPT];
    V m_val[RPT];
    bool oob = false;
    // pairs: two consecutive 8-B records per thread with one 16-B load of indices and one of
    // values (contiguous u64 indices and 8-B values, 16-B aligned); record j of a round is then
    // record 2 * ((j / 2) * 1024 + thread) + j % 2 (C2 coarse pass 1.585 -> 1.562 ms, same box)
    // PAIRS (compile time, chosen on the host: u64 indices and 8-B values, both contiguous and
    // 16-B aligned, even chunks): without the one-at-a-time path in the same kernel, no dead
    // path's pending loads make the compiler wait for the prefetch before the write-out
    constexpr bool pairs = PAIRS;
    // every pair is loaded from an even offset <= kl (the last record's pair); the host picks
    // PAIRS only when every block's range holds whole pairs, so no load passes the range's end
    const uint64_t kl = lo < hi ? lo + ((hi - 1 - lo) & ~uint64_t(1)) : lo;
    auto kof = [&](uint64_t r0, int j) -> uint64_t {
        return pairs ? r0 + 2 * (uint64_t(j >> 1) * 1024 + threadIdx.x) + (j & 1) : r0 + uint64_t(j) * 1024 + threadIdx.x;
    };
    auto load_round = [&](uint64_t r0) {
        if (pairs) {
            // branch-free from a clamped offset and used as loaded (the round masks the records
            // past hi), so all RPT / 2 pairs are in flight at once: a guarded load per pair made
            // the compiler wait for each pair before the next
#pragma unroll
            for (int j = 0; j < RPT; j += 2) {
                const uint64_t k = kof(r0, j);
                const uint64_t kc = k <= kl ? k : kl;
                const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(p.idx + kc * 8);
                const ulonglong2 y = *reinterpret_cast<const ulonglong2*>(p.val + kc * 8);
                m_raw[j] = x.x;
                m_raw[j + 1] = x.y;
                m_val[j] = V(y.x);
                m_val[j + 1] = V(y.y);
            }
            return;
        }
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint64_t k = r0 + uint64_t(j) * 1024 + threadIdx.x;
            const bool in = k < hi;
            m_raw[j] = in ? load_idx<IW>(p.idx, p.idx_stride, k) : ~uint64_t(0);
            m_val[j] = !in ? V(0) : p.val ? *reinterpret_cast<const V*>(p.val + k * p.val_stride) : V(p.val_bits);
        }
    };
    if (lo < hi) load_round(lo);
    for (uint64_t r0 = lo; r0 < hi; r0 += kRound) {
        for (uint32_t c = threadIdx.x; c < C; c += blockDim.x) hist[c] = 0;
        __syncthreads();
        uint32_t m_rank[RPT], m_c[RPT];
        bool m_ok[RPT];
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint64_t k = kof(r0, j);
            m_ok[j] = k < hi && m_raw[j] < p.shard_len;
            if (!m_ok[j] && k < hi) oob = true;
            m_c[j] = m_ok[j] ? uint32_t(m_raw[j] >> cshift) : 0u;
            if (m_ok[j]) {
                m_rank[j] = atomicAdd(&hist[m_c[j]], 1u);
                atomicAdd(&th[uint32_t(m_raw[j] >> p.tile_shift)], 1u);
            }
        }
        __syncthreads();
        small_excl_scan(hist, base, C, &tot);
        __syncthreads();
        // reserve this round's run of every bucket in the XCD's sub-region; the returned
        // fill is consumed after the LDS staging below, which hides the atomic's latency
        uint32_t rsv = 0, cnt = 0;
        if (threadIdx.x < C) {
            cnt = hist[threadIdx.x];
            if (cnt) rsv = atomicAdd(&p.ff_fill[threadIdx.x * kSegs + xcc], cnt);
        }
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            if (!m_ok[j]) continue;
            const uint32_t q = base[m_c[j]] + m_rank[j];
            s_idx[q] = uint32_t(m_raw[j]);
            s_val[q] = m_val[j];
        }
        if (threadIdx.x == 0) s_spill = 0;
        if (threadIdx.x < C) {
            const uint32_t c = threadIdx.x;
            const uint32_t a = rsv >= capx ? 0u : min(cnt, capx - rsv);
            seg_a[c] = seg_base(p.capc, xcc) + rsv;
            len_a[c] = a;
            // the rest (a full sub-region) goes to the shared area (rare for mixed streams)
            seg_b[c] = (cnt > a) ? atomicAdd(&p.ff_fill[c * kSegs + kXcds], cnt - a) : 0u;
        }
        if (r0 + kRound < hi) load_round(r0 + kRound);     // prefetch the next round
        __syncthreads();
        if (threadIdx.x < C && len_a[threadIdx.x] < hist[threadIdx.x] &&
            seg_b[threadIdx.x] + (hist[threadIdx.x] - len_a[threadIdx.x]) > caps)
            s_spill = 1;
        const uint32_t nw = blockDim.x >> 6, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const uint32_t wpb = C >= nw ? 1u : nw / C, bstep = nw / wpb;
        const uint32_t sb = seg_base(p.capc, kXcds);
        // the write-out holds no device atomic (their returned values made the compiler wait
        // for every outstanding load and store, the next round's prefetch included, at each
        // iteration); records past their bucket region are handled by the loop after it
        for (uint32_t c = wave / wpb; c < C; c += bstep) {
            const uint32_t len = hist[c], b = base[c], la = len_a[c], da = seg_a[c], db = seg_b[c];
            const uint64_t reg = uint64_t(c) * p.capc;
            for (uint32_t i = (wave % wpb) * 64 + lane; i < len; i += wpb * 64) {
                const uint32_t q = b + i;
                const uint32_t j = i - la;                  // position in the shared part
                if (i < la || db + j < caps) {
                    const uint64_t d = reg + (i < la ? da + i : sb + db + j);
                    p.tmp_idx[d] = s_idx[q];
                    if (p.tmp_val) reinterpret_cast<V*>(p.tmp_val)[d] = s_val[q];
                }
            }
        }
        __syncthreads();
        // Records past the end of their bucket's region are applied to the shard with
        // device atomics (the op is order-insensitive) and taken out of the tile counts.
        if (s_spill && p.spill) {
            for (uint32_t c = wave / wpb; c < C; c += bstep) {
                const uint32_t len = hist[c], b = base[c], la = len_a[c], db = seg_b[c];
                for (uint32_t i = (wave % wpb) * 64 + lane; i < len; i += wpb * 64) {
                    const uint32_t q = b + i;
                    if (i < la || db + (i - la) < caps) continue;
                    atomicSub(&th[s_idx[q] >> p.tile_shift], 1u);
                    uint8_t ok;
                    rmw_global<V>(reinterpret_cast<V*>(p.shard) + s_idx[q], p.op, LMR_KIND_NATIVE_ATOMIC, s_val[q],
                                  V(0), V(0), ok, p.err);
                }
            }
            __syncthreads();
        }
    }
    if (oob) raise_err(p.err, LMR_ERRBIT_OOB);
    __syncthreads();
    uint32_t* row = p.counts + uint64_t(g) * p.num_tiles;   // row g (coalesced)
    for (uint32_t t = threadIdx.x; t < p.num_tiles; t += blockDim.x) row[t] = p.accumulate ? row[t] + th[t] : th[t];
}

template <int IW, int VB, int RPT, bool PAIRS>
__global__ __launch_bounds__(1024) void k_coarse_free(PartArgs p) {
    coarse_free_body<IW, VB, RPT, PAIRS>(p, blockIdx.x);
}

// Count-free staged regions partitioned together (the exchange's sources of one chunk): one
// launch for up to kFuseFree regions, each with its own block range and rows of the tile-count
// rows (p.counts + row0 * num_tiles); the bucket regions and their fill counters are the session's.
constexpr int kFuseFree = 8;
struct FreeRegion {
    const uint8_t* idx;
    uint64_t idx_stride;
    const uint8_t* val;
    uint64_t val_stride, val_bits, n, chunk;
    uint32_t G, row0, block0;
    // device-count region (a fixed receive region of the exchange): n is the region's capacity and
    // *n_dev (written by an earlier kernel or collective on the stream) its record count, clamped
    // to n; the G blocks split the actual count
    const int64_t* n_dev;
};
struct FreeTable {
    FreeRegion r[kFuseFree];
    uint32_t nr;
};
template <int IW, int VB, int RPT, bool PAIRS>
__global__ __launch_bounds__(1024) void k_coarse_free_stage(PartArgs q, FreeTable t) {
    uint32_t i = 0;
    while (i + 1 < t.nr && t.r[i + 1].block0 <= blockIdx.x) i++;
    const FreeRegion& g = t.r[i];
    PartArgs p = q;
    p.idx = g.idx; p.idx_stride = g.idx_stride; p.val = g.val; p.val_stride = g.val_stride;
    p.val_bits = g.val_bits; p.n = g.n; p.chunk = g.chunk; p.G = g.G;
    if (g.n_dev) {
        const int64_t c = *g.n_dev;
        p.n = c <= 0 ? 0 : min(g.n, uint64_t(c));
        p.chunk = ((p.n + g.G - 1) / g.G + 1) & ~uint64_t(1);   // even: whole pairs per block
    }
    p.counts = q.counts + uint64_t(g.row0) * q.num_tiles;
    coarse_free_body<IW, VB, RPT, PAIRS>(p, blockIdx.x - g.block0);
}

// tile_start[t] = sum over blocks of the coarse pass's row counts (scanned after).
// One block per 64 tiles: wave w sums rows w, w + 16, ... (256 B per row read),
// then the 16 partial sums are added in LDS.
__global__ __launch_bounds__(1024) void k_free_tile_totals(const uint32_t* rows, uint32_t num_tiles, uint32_t G,
                                                           uint32_t* out) {
    __shared__ uint32_t part[16][64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t t = blockIdx.x * 64 + lane;
    uint32_t s = 0;
    if (t < num_tiles)
        for (uint32_t g = w; g < G; g += 16) s += rows[uint64_t(g) * num_tiles + t];
    part[w][lane] = s;
    __syncthreads();
    if (w == 0 && t < num_tiles) {
        uint32_t tot = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) tot += part[i][lane];
        out[t] = tot;
    }
}

// exclusive scan of in[0..m) (m <= 2 * NT) into out[], total into *tot; every thread calls it
template <int NT>
__device__ __noinline__ void block_excl_scan(const uint32_t* in, uint32_t* out, uint32_t m, uint32_t* part,
                                                uint32_t* tot) {
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t a = 2 * t < m ? in[2 * t] : 0u, b = 2 * t + 1 < m ? in[2 * t + 1] : 0u;
    uint32_t inc = a + b;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (int(lane) >= d) inc += y;
    }
    if (lane == 63) part[w] = inc;
    __syncthreads();
    if (t == 0) {
        uint32_t run = 0;
        for (int i = 0; i < NT / 64; i++) { const uint32_t x = part[i]; part[i] = run; run += x; }
        *tot = run;
    }
    __syncthreads();
    const uint32_t ex = part[w] + inc - (a + b);
    if (2 * t < m) out[2 * t] = ex;
    if (2 * t + 1 < m) out[2 * t + 1] = ex + a;
    __syncthreads();
}

// Rounds are read through buffer descriptors (BufStream): with flat loads the compiler kept
// one 64-bit pointer per record of the round alive and spilled them. Measured on one box
// (tools/ab_mix.sh): fine pass 1.558 -> 1.548 ms at 12K rounds; 768-thread blocks with
// 16 records per thread (168 VGPRs) and 1024 threads with 8 or 10 were all slower.
template <int VB, int RPT, int NT>
__global__ __launch_bounds__(NT) void k_fine_free(PartArgs p) {
    using V = typename idx_t<VB>::I;
    constexpr uint32_t kRound = RPT * NT;
    __shared__ uint32_t hist[kFine], base[kFine], cursor[kFine], tot;
    __shared__ uint32_t s_fill[kMaxCoarse * kSegs], s_vs[kMaxCoarse * kSegs + 1];
    __shared__ uint32_t s_part[NT / 64], s_total;
    __shared__ uint16_t s_l[kRound];
    __shared__ V s_val[kRound];
    const uint32_t NB = p.C, C = p.C * kSegs;          // buckets; segments (bucket, sub-region / shared area)
    const uint32_t lmask = (1u << p.tile_shift) - 1u;
    for (uint32_t c = threadIdx.x; c < C; c += blockDim.x)
        s_fill[c] = min(p.ff_fill[c], seg_cap(p.capc, c % kSegs));   // overflowed: clipped
    __syncthreads();
    block_excl_scan<NT>(s_fill, s_vs, C, s_part, &s_total);   // segment c = virtual records [s_vs[c], s_vs[c + 1])
    if (threadIdx.x == 0) s_vs[C] = s_total;
    __syncthreads();
    const uint64_t total = s_total;
    // consecutive ranges (one bucket's) on one XCD: the runs they append to a tile merge in its L2
    const uint32_t nb = gridDim.x;
    const uint32_t lb = xcd_block(p.xcd_swz != 0);
    const uint32_t v_lo = uint32_t(total * lb / nb);
    const uint32_t v_hi = uint32_t(total * (lb + 1) / nb);
    auto bstart = [&](uint32_t b) { return s_vs[b * kSegs]; };     // bucket b = virtual [bstart(b), bstart(b + 1))
    uint32_t m_idx[RPT];
    V m_val[RPT];
    // Round [v0, min(v0 + kRound, e)) of bucket b's virtual records: a round runs across the
    // bucket's segments (no partial round per segment); each record's slot is its segment's
    // base + its offset in it, read through buffer descriptors over the bucket's region
    // (records past e read 0). free_partition_rpt keeps capc * VB below 2^31.
    auto load_round = [&](uint32_t b, uint32_t v0, uint32_t e) {
        const BufStream bi(p.tmp_idx + uint64_t(b) * p.capc, p.capc * 4u);
        const BufStream bv(p.tmp_val + uint64_t(b) * p.capc * VB, p.tmp_val ? p.capc * uint32_t(VB) : 0u);
        const uint32_t* vs = s_vs + b * kSegs;
        uint32_t k = 0;
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint32_t v = v0 + uint32_t(j) * NT + threadIdx.x;
            uint32_t off = 0x3FFFFFFFu;                              // past the region: reads 0
            if (v < e) {
                while (v >= vs[k + 1]) k++;
                off = seg_base(p.capc, k) + (v - vs[k]);
            }
            m_idx[j] = bi.load<uint32_t>(off * 4u);
            m_val[j] = bv.load<V>(off * uint32_t(VB));
        }
    };
    // the next bucket at or after bb with records in [v_lo, v_hi)
    auto next_bucket = [&](uint32_t bb) {
        while (bb < NB && bstart(bb) < v_hi && max(v_lo, bstart(bb)) >= min(v_hi, bstart(bb + 1))) bb++;
        return bb;
    };
    uint32_t b = 0;
    while (b + 1 < NB && bstart(b + 1) <= v_lo) b++;
    b = next_bucket(b);
    // invariant: the current bucket's first round is loaded (prefetched) on entry
    if (b < NB && bstart(b) < v_hi) load_round(b, max(v_lo, bstart(b)), min(v_hi, bstart(b + 1)));
    while (b < NB && bstart(b) < v_hi) {
        const uint32_t a = max(v_lo, bstart(b)), e = min(v_hi, bstart(b + 1));
        const uint32_t bn = next_bucket(b + 1);
        const bool has_next = bn < NB && bstart(bn) < v_hi;
        const uint32_t t0 = b * kFine;
        const uint32_t nf = min(uint32_t(kFine), p.num_tiles - t0);
        const uint32_t ts = threadIdx.x < nf ? p.tile_start[t0 + threadIdx.x] : 0u;
        for (uint32_t v0 = a; v0 < e; v0 += kRound) {
            for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x) hist[f] = 0;
            __syncthreads();
            // (tile, validity) are recomputed from m_idx where needed (registers)
            uint32_t m_rank[RPT];
#pragma unroll
            for (int j = 0; j < RPT; j++)
                m_rank[j] = (v0 + uint32_t(j) * NT + threadIdx.x < e)
                                ? atomicAdd(&hist[(m_idx[j] >> p.tile_shift) - t0], 1u) : 0u;
            __syncthreads();
            small_excl_scan(hist, base, nf, &tot);
            __syncthreads();
            uint32_t rsv = 0, cnt = 0;
            if (threadIdx.x < nf) {
                cnt = hist[threadIdx.x];
                if (cnt) rsv = atomicAdd(&p.ff_tfill[t0 + threadIdx.x], cnt);
            }
#pragma unroll
            for (int j = 0; j < RPT; j++) {
                if (v0 + uint32_t(j) * NT + threadIdx.x >= e) continue;
                const uint32_t q = base[(m_idx[j] >> p.tile_shift) - t0] + m_rank[j];
                s_l[q] = uint16_t(m_idx[j] & lmask);
                s_val[q] = m_val[j];
            }
            if (threadIdx.x < nf) cursor[threadIdx.x] = ts + rsv;
            {   // one prefetch site (the next round of this bucket, else the next bucket's
                // first; nothing left: an empty range reads nothing): one set of registers
                const bool more = v0 + kRound < e;
                const uint32_t nbk = more ? b : (has_next ? bn : b);
                load_round(nbk, more ? v0 + kRound : (has_next ? max(v_lo, bstart(bn)) : e),
                           more ? e : (has_next ? min(v_hi, bstart(bn + 1)) : e));
            }
            __syncthreads();
            V* bvp = reinterpret_cast<V*>(p.bin_val);
            if (p.tmp_val)
                bucket_writeout(hist, base, cursor, nf, [&](uint32_t q, uint32_t dst) {
                    p.bin_lidx[dst] = s_l[q];
                    bvp[dst] = s_val[q];
                });
            else
                bucket_writeout(hist, base, cursor, nf, [&](uint32_t q, uint32_t dst) { p.bin_lidx[dst] = s_l[q]; });
            __syncthreads();
        }
        b = bn;
    }
}

// One block (T <= kMaxTiles): per-tile item counts, their scan and the fill in one launch
// (the counts / scan / fill as three launches cost ~15 us per sweep). Mode 0 owner item,
// mode 2 a skip marker (empty or split tile), delta pieces (mode 1) of split tiles listed
// in tile order; *delta_count = their number.
__global__ __launch_bounds__(1024) void k_tile_plan(const uint32_t* tile_start, uint32_t num_tiles, uint32_t thresh,
                                                    int combinable, TileItem* items, TileItem* delta,
                                                    uint32_t* delta_count) {
    __shared__ uint32_t tot;
    uint32_t carry = 0;
    for (uint32_t t0 = 0; t0 < num_tiles; t0 += 1024) {
        const uint32_t t = t0 + threadIdx.x;
        uint32_t lo = 0, hi = 0, m = 0;
        if (t < num_tiles) {
            lo = tile_start[t];
            hi = tile_start[t + 1];
            const uint32_t c = hi - lo;
            m = (c == 0) ? 0u : ((combinable && c > thresh) ? (c + kSplit - 1) / kSplit : 1u);
        }
        const uint32_t x = m > 1 ? m : 0u;
        const uint32_t base = carry + block_excl_scan(x, &tot);
        if (t < num_tiles) {
            items[t] = TileItem{t, lo, hi, m == 1 ? 0u : 2u};
            for (uint32_t j = 0; j < x; j++) {
                const uint32_t l = lo + j * kSplit;
                delta[base + j] = TileItem{t, l, min(hi, l + kSplit), 1u};
            }
        }
        carry += tot;
    }
    if (threadIdx.x == 0) *delta_count = carry;
}

// ---- un-partition of returned values ----------------------------------------
// dst[k] = src[map[k]] over block-contiguous ranges of k (the forward pass's
// chunks), so each block's reads stay within the runs its chunk produced and
// hit L2; map[k] == ~0 marks an out-of-bounds record (left unwritten).
template <int VB, int U>
__device__ __forceinline__ void unpartition_range(const uint32_t* __restrict__ map, uint64_t n,
                                                  const uint32_t* n_dev, uint64_t chunk, uint32_t blk,
                                                  const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                  const uint8_t* __restrict__ ok_src, uint8_t* __restrict__ ok_dst) {
    using V = typename idx_t<VB>::I;
    const uint64_t m = n_dev ? uint64_t(*n_dev) : n;
    const uint64_t lo = uint64_t(blk) * chunk;
    const uint64_t hi = min(lo + chunk, m);
    const V* s = reinterpret_cast<const V*>(src);
    V* d = reinterpret_cast<V*>(dst);
    const uint32_t nt = blockDim.x;
    // U records per thread per iteration: all U map loads, then all U gathers, then the stores.
    // Measured and not kept: a branch-free form (clamped loads, Ok flags gathered with the values,
    // so every load stays in flight): C5 0.576 -> 0.572 ms, C3 0.619 -> 0.632 ms
    for (uint64_t k0 = lo + threadIdx.x; k0 < hi; k0 += uint64_t(U) * nt) {
        uint32_t p[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t k = k0 + uint64_t(j) * nt;
            p[j] = k < hi ? map[k] : 0xFFFFFFFFu;
        }
        V v[U];
#pragma unroll
        for (int j = 0; j < U; j++) v[j] = (p[j] != 0xFFFFFFFFu) ? s[p[j]] : V(0);
#pragma unroll
        for (int j = 0; j < U; j++) {
            if (p[j] == 0xFFFFFFFFu) continue;
            const uint64_t k = k0 + uint64_t(j) * nt;
            d[k] = v[j];
            if (ok_src) ok_dst[k] = ok_src[p[j]];
        }
    }
}

template <int VB, int U>
__global__ __launch_bounds__(1024) void k_unpartition(const uint32_t* __restrict__ map, uint64_t n,
                                                      const uint32_t* n_dev, uint64_t chunk,
                                                      const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                      const uint8_t* __restrict__ ok_src, uint8_t* __restrict__ ok_dst) {
    unpartition_range<VB, U>(map, n, n_dev, chunk, blockIdx.x, src, dst, ok_src, ok_dst);
}

// the same gather over several staged regions in one launch: region i owns blocks
// [block0[i], block0[i + 1])
struct UnpartRegion {
    const uint32_t* map;
    const uint32_t* n_dev;
    uint64_t n, chunk;
    const uint8_t* src;
    uint8_t* dst;
    const uint8_t* oks;
    uint8_t* okd;
    uint32_t block0;
};
struct UnpartTable {
    UnpartRegion r[kMaxRegions];
    uint32_t nr;
};

template <int VB, int U>
__global__ __launch_bounds__(1024) void k_unpartition_multi(UnpartTable t) {
    uint32_t i = 0;
    while (i + 1 < t.nr && t.r[i + 1].block0 <= blockIdx.x) i++;
    const UnpartRegion& g = t.r[i];
    unpartition_range<VB, U>(g.map, g.n, g.n_dev, g.chunk, blockIdx.x - g.block0, g.src, g.dst, g.oks, g.okd);
}

// ------------------------------------------------------------------ dispatch
template <typename F>
static hipError_t dispatch_dtype(int dtype, F&& f) {
    switch (dtype) {
    case LMR_U8: return f(uint8_t{});
    case LMR_U16: return f(uint16_t{});
    case LMR_U32: return f(uint32_t{});
    case LMR_U64: return f(uint64_t{});
    case LMR_I8: return f(int8_t{});
    case LMR_I16: return f(int16_t{});
    case LMR_I32: return f(int32_t{});
    case LMR_I64: return f(int64_t{});
    case LMR_F32: return f(float{});
    case LMR_F64: return f(double{});
    default: return hipErrorInvalidValue;
    }
}

template <typename F>
static hipError_t dispatch_iw(int iw, F&& f) {
    switch (iw) {
    case 1: return f(std::integral_constant<int, 1>{});
    case 2: return f(std::integral_constant<int, 2>{});
    case 4: return f(std::integral_constant<int, 4>{});
    case 8: return f(std::integral_constant<int, 8>{});
    default: return hipErrorInvalidValue;
    }
}

static unsigned grid_for(uint64_t n, unsigned block, unsigned cap) {
    uint64_t g = (n + block - 1) / block;
    if (g > cap) g = cap;
    return unsigned(g ? g : 1);
}

hipError_t launch_apply_direct(int dtype, int index_size, const ApplyArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    ProfScope ps(a.prof, LMR_STAGE_DIRECT, s, a.n);
    return dispatch_dtype(dtype, [&](auto tag) {
        using T = decltype(tag);
        return dispatch_iw(index_size, [&](auto iw) {
            hipLaunchKernelGGL((k_apply_direct<T, decltype(iw)::value>),
                               dim3(grid_for(a.n, 256, 256 * 32)), dim3(256), 0, s, a);
            return hipGetLastError();
        });
    });
}

hipError_t launch_apply_mvsi(int dtype, const ApplyArgs& a, uint64_t index, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    ProfScope ps(a.prof, LMR_STAGE_MVSI, s, a.n);
    return dispatch_dtype(dtype, [&](auto tag) {
        using T = decltype(tag);
        hipLaunchKernelGGL((k_apply_mvsi<T>), dim3(1), dim3(64), 0, s, a, index);
        return hipGetLastError();
    });
}

static int tile_shift_for(int dtype) {
    int wb = dtype_bytes(dtype) < 4 ? 4 : dtype_bytes(dtype);
    int len = kTileBytes / wb;
    int sh = 0;
    while ((1 << (sh + 1)) <= len) sh++;
    return sh;
}

int tile_shift(int dtype) { return tile_shift_for(dtype); }

bool tiled_supported(int dtype, uint64_t shard_len) {
    uint64_t tiles = (shard_len + (uint64_t(1) << tile_shift_for(dtype)) - 1) >> tile_shift_for(dtype);
    return tiles >= 1 && tiles <= uint64_t(kMaxTiles);
}

// count-free partition counters: [0] unused (was the overflow flag), [64, 64 + C) bucket
// fills, then one fill per tile
static size_t ff_words() { return 64 + size_t(kMaxCoarse) * kSegs + size_t(kMaxTiles); }

// temp arrays: 25 % (+ 8192 records per coarse bucket) above the piece capacity, the
// headroom the count-free partition's fixed per-bucket regions need (3 B per record)
// temp slots: a count-free bucket region is 8 XCD sub-regions of capc / 16 (a uniform stream's
// share with 12 % headroom) and a shared area of ~capc / 2 (a bucket's whole share): 2.25 x
static uint64_t tmp_cap_for(uint64_t cap) {
    return 2 * cap + cap / 4 + uint64_t(kMaxCoarse) * 8192;
}

uint64_t max_rec_cap() {
    // every temp slot index (< tmp_cap_for(cap)) must fit the kernels' uint32 slot math
    return (uint64_t(0xFFFFFFFFull) - uint64_t(kMaxCoarse) * 8192) / 9 * 4;
}

// fine rounds of staged regions (>= 4K records each, up to 4 partial rounds per bucket and region)
static uint64_t rt_rounds_for(uint64_t cap) { return cap / 4096 + uint64_t(kMaxRegions) * (kMaxCoarse + 2) * 4; }
// coarse rounds of staged regions (>= 4K records each, one partial round per producer block of <= 64K)
static uint64_t crt_rounds_for(uint64_t cap) { return cap / 4096 + cap / 65536 + uint64_t(kMaxRegions) * 2; }

// The workspace layout, in one place: ws_layout(cap, base, &w) carves it, ws_layout(cap) sizes it.
// (Measured and not kept, profiles/r4/ab/r4p_*, r4q_*: staggered padding between the record arrays,
// their spacing as for a larger capacity, a larger allocation or a shifted base: all within 0.5 %.)
static size_t ws_layout(uint64_t cap, uint8_t* base = nullptr, TiledWs* w = nullptr) {
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += al(bytes);
        return base ? base + o : nullptr;
    };
    uint8_t* counts = take(size_t(kMaxTiles) * kMaxBinBlocks * 4);
    uint8_t* partials = take(scan_scratch_words(size_t(kMaxTiles) * kMaxBinBlocks) * 4);
    uint8_t* tile_start = take((size_t(kMaxTiles) + 1) * 4);
    uint8_t* bin_lidx = take(cap * 2);
    uint8_t* bin_val = take(cap * 8);
    uint8_t* rpos = take(cap * 4);
    uint8_t* total = take(4);
    uint8_t* coarse_off = take((size_t(kMaxCoarse) * kMaxBinBlocks + 1) * 4);
    uint8_t* tmp_idx = take(tmp_cap_for(cap) * 4);
    uint8_t* tmp_val = take(tmp_cap_for(cap) * 8);
    uint8_t* qpos = take(cap * 4);
    uint8_t* tile_items = take((size_t(kMaxTiles) + 1) * 4);
    uint8_t* tile_items2 = take((size_t(kMaxTiles) + 1) * 4);
    uint8_t* plan_partials = take(size_t(kMaxTiles) / kScanItems * 4 + 256);
    uint8_t* item_count = take(4);
    uint8_t* items = take((size_t(kMaxTiles) + 2 * (cap / kSplit) + 2) * 16);   // owner items + delta pieces
    uint8_t* rts = take(size_t(kMaxRegions) * (kMaxTiles + 1) * 4);             // staged regions' tile starts
    uint8_t* sinfo = take(size_t(kStageInfoWords) * 4);                          // staged piece table / totals
    uint8_t* ff = take(ff_words() * 4);                                          // count-free fill counters
    uint8_t* runtab = take(rt_rounds_for(cap) * 256 * 4);                       // staged run tables
    uint8_t* ptab = take(size_t(kMaxRegions) * 2 * (kMaxCoarse + 1) * 4);       // staged piece tables
    uint8_t* crtab = take(crt_rounds_for(cap) * 256 * 4);                       // staged coarse run tables
    uint8_t* rtot = take(size_t(kMaxRegions) * kMaxTiles * 4);                  // staged regions' tile totals
    uint8_t* rfill = take(size_t(kMaxRegions) * kMaxTiles * 4);                 //   and fills
    if (w) {
        w->counts = reinterpret_cast<uint32_t*>(counts);
        w->partials = reinterpret_cast<uint32_t*>(partials);
        w->tile_start = reinterpret_cast<uint32_t*>(tile_start);
        w->bin_lidx = reinterpret_cast<uint16_t*>(bin_lidx);
        w->bin_val = bin_val;
        w->rpos = reinterpret_cast<uint32_t*>(rpos);
        w->total = reinterpret_cast<uint32_t*>(total);
        w->coarse_off = reinterpret_cast<uint32_t*>(coarse_off);
        w->tmp_idx = reinterpret_cast<uint32_t*>(tmp_idx);
        w->tmp_val = tmp_val;
        w->qpos = reinterpret_cast<uint32_t*>(qpos);
        w->tile_items = reinterpret_cast<uint32_t*>(tile_items);
        w->tile_items2 = reinterpret_cast<uint32_t*>(tile_items2);
        w->plan_partials = reinterpret_cast<uint32_t*>(plan_partials);
        w->item_count = reinterpret_cast<uint32_t*>(item_count);
        w->items = items;
        w->rts = reinterpret_cast<uint32_t*>(rts);
        w->sinfo = reinterpret_cast<uint32_t*>(sinfo);
        w->ff = reinterpret_cast<uint32_t*>(ff);
        w->runtab = reinterpret_cast<uint32_t*>(runtab);
        w->rt_rounds = rt_rounds_for(cap);
        w->ptab = reinterpret_cast<uint32_t*>(ptab);
        w->crtab = reinterpret_cast<uint32_t*>(crtab);
        w->crt_rounds = crt_rounds_for(cap);
        w->rtot = reinterpret_cast<uint32_t*>(rtot);
        w->rfill = reinterpret_cast<uint32_t*>(rfill);
        w->cap = cap;
        w->tmp_cap = tmp_cap_for(cap);
    }
    return off;
}

size_t tiled_ws_bytes(uint64_t cap) { return ws_layout(cap); }

TiledWs carve_tiled_ws(uint8_t* base, uint64_t cap) {
    TiledWs w;
    ws_layout(cap, base, &w);
    return w;
}

// Block counts of the partition passes (tunable for measurements through
// LMR_BIN_BLOCKS / LMR_FINE_BLOCKS; defaults fill 256 CUs twice).
static int env_int(const char* name, int dflt, int lo, int hi) {
    const char* v = getenv(name);
    if (!v || !*v) return dflt;
    int x = atoi(v);
    return x < lo ? lo : (x > hi ? hi : x);
}
static int coarse_rpt(int vb);
// Coarse-pass blocks G (also the count pass's): one per CU when a coarse block
// takes more than half the LDS (rounds of >= 8K records), two otherwise. G = 256
// vs 512 on one box (tools/sweep_c2.sh): C2 4.40 -> 4.33 ms, C3 2.72 -> 2.47 ms
// (larger producer chunks also keep the un-partition gathers local).
// Staged regions' un-partition gathers round-wise through LDS (LMR_UNPART_ROUNDS bits): 1 = the
// first gather (k_unpart_rounds, fine rounds), 2 = the second (k_unpart_crounds, coarse rounds)
// for values of <= 4 bytes, 4 = the second for 8-byte values. The coarse round gather of 8-byte
// values holds a 12K-record round (108 KB of LDS, one block per CU): C3 0.52 -> 0.64 ms
static int unpart_rounds() {
    static int v = env_int("LMR_UNPART_ROUNDS", 3, 0, 7);
    return v;
}
static int ccount_split() {
    static int v = env_int("LMR_CCOUNT_SPLIT", 1, 1, 16);   // (4: C5 count -0.027 ms, coarse +0.015)
    return v;
}
static int bin_blocks_cap(int vb) {
    static int v = env_int("LMR_BIN_BLOCKS", 0, 0, kMaxBinBlocks);
    return v ? v : (coarse_rpt(vb) >= 8 ? 256 : 512);
}
// Delta-mode threshold: a tile of a combinable op splits into delta pieces when it holds more
// than max(LMR_DELTA_MUL x the average tile's records, LMR_DELTA_MIN) records. Round 4 (same box,
// profiles/r4/ab/r4g_*, r4h_*): 2 x / 32K takes C3's warm tiles off the owner kernel's serialised
// LDS atomics, tile sweep 0.463-0.484 -> 0.443-0.466 ms (4 x / 64K before; 1 x / 16K and 2 x / 16K
// no better; no delta at all: 4.69 ms).
static uint64_t delta_mul() {
    static int v = env_int("LMR_DELTA_MUL", 2, 1, 1 << 20);
    return uint64_t(v);
}
static uint64_t delta_min() {
    static int v = env_int("LMR_DELTA_MIN", 32768, 1024, 1 << 30);
    return uint64_t(v);
}
static int tile_grid_cap() {
    static int v = env_int("LMR_DELTA_BLOCKS", 1024, 1, 1 << 24);
    return v;
}
// records per thread per round of the coarse / fine passes (LMR_COARSE_RPT,
// LMR_FINE_RPT: 4, 6, 8, 10, 12 or 16; capped to what fits the LDS). Bigger rounds
// amortise the per-round barriers and bucket scan and lengthen the output runs.
// Measured on one box (tools/r1h_cmd.sh): 8-byte values, coarse 1.71 -> 1.43 ms
// at 12K-record rounds, fine 1.75 -> 1.60 ms at 8K; 4-byte values (C5) are best
// at 4K-record rounds. Once a fine block streams its consecutive segments as one
// range (no partial round per segment), 12K fine rounds pay too (same box, C2:
// fine 1.59 -> 1.51 ms); the piece-based fine pass (kPiece = 16K records) stays
// at 8K rounds (C4 rehearsal: 12K = 1.5 rounds per piece, fine 2.52 -> 2.89 ms).
static int coarse_rpt(int vb) {
    static int v = env_int("LMR_COARSE_RPT", 0, 0, 16);
    return v ? v : (vb == 8 ? 12 : vb == 4 ? 8 : 4);      // 4-byte values: 8K rounds (C5 -0.03 ms)
}
static int fine_rpt(int vb) {
    static int v = env_int("LMR_FINE_RPT", 0, 0, 16);
    return v ? v : (vb == 8 ? 12 : 4);
}
static int piece_fine_rpt(int vb) {
    static int v = env_int("LMR_FINE_RPT", 0, 0, 16);
    return v ? v : (vb >= 4 ? 8 : 4);                      // 4-byte values: 8K rounds (C5 fine 0.91 -> 0.81 ms)
}
// f(vb, rpt) with rpt the largest supported value <= the request whose round
// (rpt * 1024 records of Extra + VB bytes in LDS) fits in 150 KiB
template <int Extra, typename F>
static void dispatch_vb_rpt(int vb, int rpt, F&& f) {
    using std::integral_constant;
    auto with_vb = [&](auto vbt) {
        constexpr int VB = decltype(vbt)::value;
        constexpr int kMaxR = (150 * 1024) / ((Extra + VB) * 1024);
        auto call = [&](auto r) {
            constexpr int R = decltype(r)::value;
            if constexpr (R <= kMaxR) f(vbt, r);
            else if constexpr (kMaxR >= 12) f(vbt, integral_constant<int, 12>{});
            else if constexpr (kMaxR >= 8) f(vbt, integral_constant<int, 8>{});
            else f(vbt, integral_constant<int, 4>{});
        };
        if (rpt >= 16) call(integral_constant<int, 16>{});
        else if (rpt >= 12) call(integral_constant<int, 12>{});
        else if (rpt >= 10) call(integral_constant<int, 10>{});
        else if (rpt >= 8) call(integral_constant<int, 8>{});
        else if (rpt >= 6) call(integral_constant<int, 6>{});
        else call(integral_constant<int, 4>{});
    };
    switch (vb) {
    case 1: with_vb(integral_constant<int, 1>{}); break;
    case 2: with_vb(integral_constant<int, 2>{}); break;
    case 4: with_vb(integral_constant<int, 4>{}); break;
    default: with_vb(integral_constant<int, 8>{}); break;
    }
}
static int fine_blocks_cap() {
    static int v = env_int("LMR_FINE_BLOCKS", 512, 1, 1 << 20);
    return v;
}
// k_fine_free's grid: 1024 blocks with XCD-grouped ranges (C2 fine 1.29 -> 1.26 ms vs 512)
static int free_fine_blocks() {
    static int v = env_int("LMR_FREE_FINE_BLOCKS", 1024, 8, 1 << 20);
    return v;
}
// LMR_FINE_XCD=0: k_fine_free's ranges dealt in plain block order (xcd_block off). The piece
// and counted fine passes keep plain order: with it, C5 fine 0.81 -> 0.89 ms, C3 +0.03 ms
static int fine_xcd() {
    static int v = env_int("LMR_FINE_XCD", 1, 0, 1);
    return v;
}

// dst[k] = src[map[k]] over G block-contiguous ranges of `chunk` records, each split into
// `split` sub-ranges (LMR_UNPART_SPLIT overrides); LMR_UNPART_NT threads per block,
// LMR_UNPART_U gathers in flight per thread (defaults 1024, and 4 for 8-byte values, 16 for
// narrower ones). The ranges (the one-shot path's forward chunks, one per CU; the staged
// regions' 64K-record ranges) are split into sub-ranges of 32 KB of values (split = 0): one
// block each, so the grid balances over the CUs. Measured per sub-range size (same box):
// C3 (8-byte) 8K records 0.68 ms, 4K 0.62, 2K 0.66; C5 (4-byte) 16K 0.60, 8K 0.57, 4K 0.61;
// C3 one-shot: 256K-record chunks unsplit 0.82 ms, 4K sub-ranges 0.64.
// Measured and not kept: 256 / 512-thread blocks, 2 or 8 gathers per thread for 8-byte
// values (C3 0.81 -> 0.82-0.90 ms), and (value, ok) packed into one u64 for Result ops
// on narrow types (C5: un-partition -0.01 ms, tile sweep +0.02 ms)
static hipError_t launch_unpartition(int vb, const uint32_t* map, uint64_t n, const uint32_t* n_dev, uint64_t chunk,
                                     uint64_t G, const uint8_t* src, uint8_t* dst, const uint8_t* oks, uint8_t* okd,
                                     hipStream_t s, int dflt_split = 0) {
    static const int split_env = env_int("LMR_UNPART_SPLIT", 0, 0, 64);
    static const int nt = env_int("LMR_UNPART_NT", 1024, 64, 1024);
    static const int uq = env_int("LMR_UNPART_U", 0, 0, 16);
    const uint64_t sub = 32768 / uint64_t(vb);
    const int split = split_env ? split_env
                    : dflt_split ? dflt_split
                                 : int(std::min<uint64_t>(64, std::max<uint64_t>(1, (chunk + sub - 1) / sub)));
    const uint64_t c2 = (chunk + split - 1) / split;
    const unsigned grid = unsigned(std::max<uint64_t>(1, G * uint64_t(split)));
    const int u = uq ? uq : (vb >= 8 ? 4 : 16);
    auto go = [&](auto vbt) {
        constexpr int VB = decltype(vbt)::value;
        auto with_u = [&](auto ut) {
            constexpr int UU = decltype(ut)::value;
            hipLaunchKernelGGL((k_unpartition<VB, UU>), dim3(grid), dim3(nt), 0, s, map, n, n_dev, c2, src, dst, oks, okd);
        };
        if (u >= 16) with_u(std::integral_constant<int, 16>{});
        else if (u >= 8) with_u(std::integral_constant<int, 8>{});
        else if (u >= 4) with_u(std::integral_constant<int, 4>{});
        else with_u(std::integral_constant<int, 2>{});
    };
    switch (vb) {
    case 1: go(std::integral_constant<int, 1>{}); break;
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 4: go(std::integral_constant<int, 4>{}); break;
    default: go(std::integral_constant<int, 8>{}); break;
    }
    return hipGetLastError();
}

// one k_unpartition_multi launch over the regions of t (block0 filled here); each region
// split as launch_unpartition splits a single range
static hipError_t launch_unpartition_multi(int vb, UnpartTable& t, hipStream_t s) {
    if (t.nr == 0) return hipSuccess;
    static const int sub_env = env_int("LMR_UNPART_SUB", 0, 0, 1 << 20);   // records per block (A/B knob)
    static const int uq = env_int("LMR_UNPART_U", 0, 0, 16);
    const uint64_t sub = sub_env ? uint64_t(sub_env) : 32768 / uint64_t(vb);
    uint32_t blocks = 0;
    for (uint32_t i = 0; i < t.nr; i++) {
        UnpartRegion& g = t.r[i];
        uint64_t Gu = (g.n + 65535) / 65536;
        Gu = std::max<uint64_t>(1, std::min<uint64_t>(Gu, 1024));
        const uint64_t chunk = (g.n + Gu - 1) / Gu;
        const uint64_t split = std::min<uint64_t>(64, std::max<uint64_t>(1, (chunk + sub - 1) / sub));
        g.chunk = (chunk + split - 1) / split;
        g.block0 = blocks;
        blocks += uint32_t(Gu * split);
    }
    const int u = uq ? uq : (vb >= 8 ? 4 : 16);
    auto go = [&](auto vbt) {
        constexpr int VB = decltype(vbt)::value;
        auto with_u = [&](auto ut) {
            hipLaunchKernelGGL((k_unpartition_multi<VB, decltype(ut)::value>), dim3(blocks), dim3(1024), 0, s, t);
        };
        if (u >= 16) with_u(std::integral_constant<int, 16>{});
        else if (u >= 8) with_u(std::integral_constant<int, 8>{});
        else with_u(std::integral_constant<int, 4>{});
    };
    switch (vb) {
    case 1: go(std::integral_constant<int, 1>{}); break;
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 4: go(std::integral_constant<int, 4>{}); break;
    default: go(std::integral_constant<int, 8>{}); break;
    }
    return hipGetLastError();
}

// Count-free partition (k_coarse_free / k_fine_free): order-insensitive ops with
// nothing returned, two-level shards, and >= 25 % headroom per coarse bucket region
// in the temp arrays for a uniform stream of n records (records past a full region
// are applied at once with device atomics, so a skewed stream stays correct).
// Returns its coarse round (records per thread), 0 when not used. LMR_FREE=0
// disables it (read per call: tests switch it in one process).
static int free_partition_rpt(int dtype, int op, int ret, uint64_t n, uint64_t num_tiles, uint64_t tmp_cap) {
    const char* e = getenv("LMR_FREE");
    if (e && e[0] == '0') return 0;
    if (ret != LMR_RET_NONE || dtype > LMR_I64) return 0;
    if (op != LMR_OP_ADD && op != LMR_OP_SUB && op != LMR_OP_MUL && op != LMR_OP_AND &&
        op != LMR_OP_OR && op != LMR_OP_XOR)
        return 0;
    if (num_tiles <= uint64_t(kFine) || num_tiles > uint64_t(kMaxTiles)) return 0;
    const uint64_t C = (num_tiles + kFine - 1) / kFine;
    const uint64_t capc = tmp_cap / C;
    if (n / C + n / (4 * C) + 8192 > capc) return 0;
    const int vb = dtype_bytes(dtype);
    if (capc * uint64_t(vb) >= (uint64_t(1) << 31)) return 0;   // k_fine_free's buffer descriptors
    // the largest round that fits next to the LDS tile counts (static + dynamic LDS
    // <= 160 KiB); 8-byte values: 10K-record rounds at 8192 tiles (12K with the
    // counted pass). 4-byte values take 8K rounds here (C5: coarse 0.80 -> 0.72 ms)
    const int cap_r = std::max(coarse_rpt(vb), 8);
    for (int r : {12, 10, 8, 4})
        if (r <= cap_r && size_t(4 + vb) * r * 1024 + num_tiles * 4 + 2048 <= size_t(158) * 1024) return r;
    return 0;
}

bool free_partition_applies(int dtype, int op, int ret, uint64_t shard_len, uint64_t n, uint64_t cap) {
    const int shift = tile_shift_for(dtype);
    const uint64_t num_tiles = (shard_len + (uint64_t(1) << shift) - 1) >> shift;
    return free_partition_rpt(dtype, op, ret, n, num_tiles, tmp_cap_for(cap)) > 0;
}

bool piece_partition_pays(int dtype, uint64_t shard_len, uint64_t n) {
    const int shift = tile_shift_for(dtype);
    const uint64_t num_tiles = (shard_len + (uint64_t(1) << shift) - 1) >> shift;
    if (num_tiles <= uint64_t(kFine) || num_tiles > uint64_t(kMaxTiles) || n == 0) return false;
    const int vb = dtype_bytes(dtype);
    uint64_t G = (n + 65535) / 65536;
    if (G > uint64_t(bin_blocks_cap(vb))) G = bin_blocks_cap(vb);
    const uint64_t C = (num_tiles + kFine - 1) / kFine;
    return n / (G * C) < 8192;
}

// count-free partition arguments shared by the one-shot path and the staged
// regions: bucket c's region is temp slots [c * capc, (c + 1) * capc); records that
// find it full are applied to the shard with device atomics (spill)
static PartArgs free_args(int dtype, const ApplyArgs& a, const TiledWs& w, uint32_t G) {
    const int shift = tile_shift_for(dtype);
    const uint32_t T = uint32_t((a.shard_len + (uint64_t(1) << shift) - 1) >> shift);
    PartArgs q{};
    q.shard_len = a.shard_len; q.tile_shift = shift; q.num_tiles = T;
    q.G = G; q.C = (T + kFine - 1) / kFine;
    q.tile_start = w.tile_start; q.counts = w.counts;
    q.tmp_idx = w.tmp_idx; q.tmp_val = w.tmp_val;          // values always materialised
    q.bin_lidx = w.bin_lidx; q.bin_val = w.bin_val;
    q.err = a.err;
    q.ff_fill = w.ff + 64; q.ff_tfill = w.ff + 64 + kMaxCoarse * kSegs;
    q.capc = uint32_t(w.tmp_cap / q.C); q.tmp_cap = w.tmp_cap;
    q.spill = 1; q.shard = a.shard; q.op = a.op;
    q.xcd_swz = fine_xcd();
    return q;
}

static hipError_t launch_coarse_free(int index_size, int vb, int frpt, const PartArgs& q, hipStream_t s) {
    return dispatch_iw(index_size, [&](auto iw) {
        constexpr int IW = decltype(iw)::value;
        dispatch_vb_rpt<4>(vb, frpt, [&](auto vbt, auto rpt) {
            constexpr int VBc = decltype(vbt)::value, R = decltype(rpt)::value;
            // (even chunks and an even n: every block's range is whole pairs, so no 16-B load
            // reaches past the caller's last record)
            const bool pairs = kCoarsePairs && IW == 8 && VBc == 8 && (R % 2) == 0 && q.idx_stride == 8 && q.val &&
                               q.val_stride == 8 && (q.chunk % 2) == 0 && (q.n % 2) == 0 &&
                               ((reinterpret_cast<uintptr_t>(q.idx) | reinterpret_cast<uintptr_t>(q.val)) & 15) == 0;
            if (pairs)
                hipLaunchKernelGGL((k_coarse_free<IW, VBc, R, (IW == 8 && VBc == 8 && R % 2 == 0)>), dim3(q.G), dim3(1024),
                                   size_t(q.num_tiles) * 4, s, q);
            else
                hipLaunchKernelGGL((k_coarse_free<IW, VBc, R, false>), dim3(q.G), dim3(1024), size_t(q.num_tiles) * 4, s, q);
        });
        return hipGetLastError();
    });
}

// exact tile starts from the coarse pass's tile-count rows, then the fine pass
static hipError_t launch_free_finish(int vb, const PartArgs& q, const TiledWs& w, uint64_t n, Prof* prof,
                                     hipStream_t s) {
    const uint32_t T = q.num_tiles;
    hipError_t e;
    {
        ProfScope ps(prof, LMR_STAGE_SCAN, s);
        hipLaunchKernelGGL(k_free_tile_totals, dim3((T + 63) / 64), dim3(1024), 0, s, w.counts, T, q.G, w.tile_start);
        e = scan_exclusive_u32(w.tile_start, T, w.partials, w.tile_start + T, s);
    }
    if (e != hipSuccess) return e;
    ProfScope ps(prof, LMR_STAGE_FINE_SCATTER, s, n);
    dispatch_vb_rpt<2>(vb, fine_rpt(vb), [&](auto vbt, auto rpt) {
        constexpr int VBc = decltype(vbt)::value, R = decltype(rpt)::value;
        hipLaunchKernelGGL((k_fine_free<VBc, R, 1024>), dim3(unsigned(free_fine_blocks())), dim3(1024), 0, s, q);
    });
    return hipGetLastError();
}

// work plan (owner items, delta pieces of hot tiles for combinable ops) and the tile
// sweep over the binned records [tile_start[t], tile_start[t + 1]) of every tile
static hipError_t launch_tile_sweep(int dtype, const ApplyArgs& a, const TiledWs& w, uint32_t T, uint64_t n,
                                    bool scalar, void* res_bin, uint8_t* ok_bin, hipStream_t s) {
    ProfScope ps(a.prof, LMR_STAGE_TILE_APPLY, s, n);
    const uint64_t avg = (n + T - 1) / T;
    const uint32_t thresh = uint32_t(std::min<uint64_t>(0xFFFFFFFFull, std::max<uint64_t>(delta_mul() * avg, delta_min())));
    TileItem* items = reinterpret_cast<TileItem*>(w.items);
    hipLaunchKernelGGL(k_tile_plan, dim3(1), dim3(1024), 0, s, w.tile_start, T, thresh, op_combines(a.op) ? 1 : 0,
                       items, items + kMaxTiles, w.item_count);
    TileArgs t;
    t.shard = a.shard; t.shard_len = a.shard_len; t.tile_shift = tile_shift_for(dtype);
    t.kind = a.kind; t.op = a.op; t.ret = res_bin ? a.ret : LMR_RET_NONE;
    t.cmp_bits = a.cmp_bits; t.eps_bits = a.eps_bits; t.val_bits = a.val_bits;
    t.scalar = scalar;
    t.items = items; t.delta = items + kMaxTiles; t.delta_count = w.item_count;
    t.num_tiles = T;
    t.bin_lidx = w.bin_lidx; t.bin_val = w.bin_val;
    t.results = res_bin; t.ok = ok_bin; t.err = a.err;
    t.rts = nullptr; t.nreg = 0; t.rstride = 0; t.mixed = 0;
    const bool delta = op_combines(a.op) && n > thresh;
    const unsigned dgrid = unsigned(std::min<uint64_t>(2 * ((n + kSplit - 1) / kSplit), uint64_t(tile_grid_cap())));
    return launch_tile_kernels(dtype, a.op, t, delta, dgrid, s, w.side);
}

// One tiled piece: a.n <= workspace capacity, a.n < 2^32.
hipError_t launch_apply_tiled(int dtype, int index_size, const ApplyArgs& a, const TiledWs& w,
                              hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const int shift = tile_shift_for(dtype);
    const uint64_t num_tiles = (a.shard_len + (uint64_t(1) << shift) - 1) >> shift;
    if (num_tiles == 0 || num_tiles > uint64_t(kMaxTiles)) return hipErrorNotSupported;
    const uint32_t T = uint32_t(num_tiles);
    const int vb = dtype_bytes(dtype);
    const bool has_res = a.ret != LMR_RET_NONE;
    hipError_t e;
    // ---- count-free partition: order-insensitive integer ops that return nothing
    if (const int frpt = free_partition_rpt(dtype, a.op, a.ret, a.n, num_tiles, w.tmp_cap)) {
        // one coarse block per CU once a round takes most of the LDS
        uint64_t Gf = (a.n + 65535) / 65536;
        Gf = std::max<uint64_t>(1, std::min<uint64_t>(Gf, frpt >= 8 ? 256 : 512));
        PartArgs q = free_args(dtype, a, w, uint32_t(Gf));
        q.idx = a.idx; q.idx_stride = a.idx_stride; q.val = a.val; q.val_stride = a.val_stride;
        q.val_bits = a.val_bits; q.n = a.n; q.chunk = (a.n + Gf - 1) / Gf;
        q.tmp_val = a.val ? w.tmp_val : nullptr;            // one scalar value: bins carry indices only
        e = hipMemsetAsync(w.ff, 0, ff_words() * 4, s);
        if (e != hipSuccess) return e;
        {
            ProfScope ps(a.prof, LMR_STAGE_BIN_SCATTER, s, a.n);
            e = launch_coarse_free(index_size, vb, frpt, q, s);
        }
        if (e == hipSuccess) e = launch_free_finish(vb, q, w, a.n, a.prof, s);
        if (e == hipSuccess) e = launch_tile_sweep(dtype, a, w, T, a.n, a.val == nullptr, nullptr, nullptr, s);
        return e;
    }
    // ---- counted partition: records keep input order within every tile
    // G blocks: >= 64K records each, at most kMaxBinBlocks
    uint64_t G = (a.n + 65535) / 65536;
    if (G > uint64_t(bin_blocks_cap(vb))) G = bin_blocks_cap(vb);
    if (G < 1) G = 1;
    BinArgs b{};
    b.idx = a.idx; b.idx_stride = a.idx_stride;
    b.val = a.val; b.val_stride = a.val_stride;
    b.n = a.n; b.shard_len = a.shard_len;
    b.chunk = (a.n + G - 1) / G;
    b.tile_shift = shift; b.num_tiles = T; b.G = uint32_t(G);
    b.counts = w.counts; b.bin_lidx = w.bin_lidx; b.bin_val = w.bin_val;
    b.rpos = has_res ? w.rpos : nullptr;
    b.err = a.err;
    const size_t hist_lds = size_t(num_tiles) * 4;
    {
        ProfScope ps(a.prof, LMR_STAGE_BIN_COUNT, s, a.n);
        e = dispatch_iw(index_size, [&](auto iw) {
            hipLaunchKernelGGL((k_bin_count<decltype(iw)::value>), dim3(unsigned(G)), dim3(kBinBlock),
                               hist_lds, s, b);
            return hipGetLastError();
        });
    }
    if (e != hipSuccess) return e;
    {
        ProfScope ps(a.prof, LMR_STAGE_SCAN, s);
        e = scan_exclusive_u32(w.counts, num_tiles * G, w.partials, w.total, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_tile_starts, dim3(unsigned((num_tiles + 1 + 255) / 256)), dim3(256), 0, s,
                           w.counts, T, uint32_t(G), w.total, w.tile_start);
    }
    if (num_tiles > uint64_t(kFine)) {
        // two-level LDS-staged partition: coarse buckets of kFine tiles, then tiles
        PartArgs q{};
        q.idx = a.idx; q.idx_stride = a.idx_stride; q.val = a.val; q.val_stride = a.val_stride;
        q.n = a.n; q.shard_len = a.shard_len; q.chunk = b.chunk; q.tile_shift = shift;
        q.num_tiles = T; q.G = uint32_t(G);
        q.C = uint32_t((num_tiles + kFine - 1) / kFine);
        q.fine_off = w.counts; q.tile_start = w.tile_start; q.coarse_off = w.coarse_off;
        q.tmp_idx = w.tmp_idx; q.tmp_val = a.val ? w.tmp_val : nullptr;
        q.qpos = has_res ? w.qpos : nullptr;
        q.bin_lidx = w.bin_lidx; q.bin_val = w.bin_val; q.rpos = b.rpos;
        {
            ProfScope ps(a.prof, LMR_STAGE_BIN_SCATTER, s, a.n);
            const uint64_t ncg = uint64_t(q.C) * G + 1;
            hipLaunchKernelGGL(k_coarse_offsets, dim3(unsigned((ncg + 255) / 256)), dim3(256), 0, s, q);
            e = dispatch_iw(index_size, [&](auto iw) {
                constexpr int IW = decltype(iw)::value;
                dispatch_vb_rpt<4>(vb, coarse_rpt(vb), [&](auto vbt, auto rpt) {
                    constexpr int VBc = decltype(vbt)::value, R = decltype(rpt)::value;
                    hipLaunchKernelGGL((k_coarse_scatter<IW, VBc, R>), dim3(unsigned(G)), dim3(1024), 0, s, q);
                });
                return hipGetLastError();
            });
        }
        if (e != hipSuccess) return e;
        ProfScope pf(a.prof, LMR_STAGE_FINE_SCATTER, s, a.n);
        const uint64_t nseg = uint64_t(q.C) * G;
        const unsigned fgrid = unsigned(std::min<uint64_t>(nseg, uint64_t(fine_blocks_cap())));
        dispatch_vb_rpt<2>(vb, fine_rpt(vb), [&](auto vbt, auto rpt) {
            constexpr int VBc = decltype(vbt)::value, R = decltype(rpt)::value;
            hipLaunchKernelGGL((k_fine_scatter<VBc, R>), dim3(fgrid ? fgrid : 1u), dim3(1024), 0, s, q);
        });
        e = hipGetLastError();
    } else {
        ProfScope ps(a.prof, LMR_STAGE_BIN_SCATTER, s, a.n);
        e = dispatch_iw(index_size, [&](auto iw) {
            constexpr int IW = decltype(iw)::value;
            switch (vb) {
            case 1: hipLaunchKernelGGL((k_bin_scatter<IW, 1>), dim3(unsigned(G)), dim3(kBinBlock), hist_lds, s, b); break;
            case 2: hipLaunchKernelGGL((k_bin_scatter<IW, 2>), dim3(unsigned(G)), dim3(kBinBlock), hist_lds, s, b); break;
            case 4: hipLaunchKernelGGL((k_bin_scatter<IW, 4>), dim3(unsigned(G)), dim3(kBinBlock), hist_lds, s, b); break;
            default: hipLaunchKernelGGL((k_bin_scatter<IW, 8>), dim3(unsigned(G)), dim3(kBinBlock), hist_lds, s, b); break;
            }
            return hipGetLastError();
        });
    }
    if (e != hipSuccess) return e;
    // results in binned order: reuse the temp buffers the partition is done with
    uint8_t* res_bin = w.tmp_val;
    uint8_t* ok_bin = reinterpret_cast<uint8_t*>(w.tmp_idx);
    e = launch_tile_sweep(dtype, a, w, T, a.n, a.val == nullptr, has_res ? res_bin : nullptr,
                          has_res ? ok_bin : nullptr, s);
    if (e != hipSuccess || !has_res) return e;
    // un-partition: binned -> (temp ->) input order, each a block-contiguous gather
    ProfScope pu(a.prof, LMR_STAGE_UNPARTITION, s, a.n);
    const uint8_t* ok_src = (a.ret == LMR_RET_RESULT) ? ok_bin : nullptr;
    auto gather = [&](const uint32_t* map, const uint32_t* n_dev, const uint8_t* src, uint8_t* dst,
                      const uint8_t* oks, uint8_t* okd) {
        (void)launch_unpartition(vb, map, a.n, n_dev, b.chunk, G, src, dst, oks, okd, s);
    };
    if (num_tiles > uint64_t(kFine)) {
        uint8_t* ok_tmp = ok_src ? reinterpret_cast<uint8_t*>(w.bin_lidx) : nullptr;
        gather(w.rpos, w.total, res_bin, w.bin_val, ok_src, ok_tmp);                                       // binned -> temp
        gather(w.qpos, nullptr, w.bin_val, reinterpret_cast<uint8_t*>(a.results), ok_tmp, a.ok);           // temp -> input
    } else {
        gather(w.rpos, nullptr, res_bin, reinterpret_cast<uint8_t*>(a.results), ok_src, a.ok);
    }
    return hipGetLastError();
}

// ============================================================ staged apply
// The owner side of the multi-PE exchange. A batch reaches its owner PE in
// chunks (one RCCL all-to-all-v per chunk, engine._distributed), as the
// reference's op AMs reach it one buffer at a time and are applied on arrival
// (registered_active_message.rs:443-497 -> impl/src/array_ops.rs:863-1408).
// Applying every chunk on arrival would sweep the whole shard once per chunk;
// instead each arriving record stream (a *region*) is partitioned into 64 KiB
// shard tiles on arrival, inside its own slice of the workspace, and one tile
// sweep at the end applies every region:
//   per region : k_ccount (coarse histogram per producer block, tile totals)
//                -> k_coarse_scatter (shared with the one-shot path; its blocks fold the
//                   raw counts into their cursors, block 0 stores the bucket starts and
//                   turns the tile totals into the region's tile starts)
//                -> k_fine_piece (each round reserves its tile runs with one atomic per
//                   tile; region now tile-sorted)
//   finish     : k_stage_plan -> k_tile_owner over every region's
//                range of its tile (+ k_tile_delta for hot tiles)
//                -> k_unpartition_multi x 2 (every region's results back to arrival order)
// The fine level works on fixed pieces of kPiece records of each coarse bucket
// (not on per-producer-block segments as k_fine_scatter does), so its LDS rounds
// stay full and its output runs long whatever the region size: a 2^25-record
// chunk partitions as efficiently as a 2^28-record batch.
#ifndef LMR_PIECE_RECORDS
#define LMR_PIECE_RECORDS 16384                  // (variant builds for measurements: -DLMR_PIECE_RECORDS=...)
#endif
constexpr uint32_t kPiece = LMR_PIECE_RECORDS;   // records per fine-level piece (2 LDS rounds of 8K)
constexpr int kStageInb = 320;                   //              in-bounds records per region
static_assert(kStageInb + kMaxRegions <= kStageInfoWords, "staged scratch");

// per-(coarse bucket, producer block) record counts: coarse_off[c * G + g]
// (16 lane-picked copies of the histogram, to spread the LDS atomics' address conflicts,
// measured 0.35 -> 0.36 ms per C5 step: the pass is not bound by them)
// Measured and dropped: per-thread private LDS counters instead of the shared histogram's
// atomics (C5 count 0.33 -> 0.38 ms: 128 KB of LDS per block, zeroing and folding); the bucket
// counts summed from the tile counts after the loop, one LDS atomic per record (0.371 -> 0.383 ms).
// Every block also counts its records per tile (LDS atomics over T bins, few conflicts) into
// its row of p.trows: k_coarse_scatter folds the rows into tile totals, k_fine_piece turns
// them into tile starts and reserves each round's tile runs inside them.
template <int IW>
__device__ __forceinline__ void ccount_body(const PartArgs& p, const uint32_t bid) {
    // loads in flight per thread (4: C5 count 0.347 -> 0.337 ms at 8; 16: 0.380 -> 0.398 ms)
    constexpr int U = 8;
    __shared__ uint32_t hist[kMaxCoarse];
    extern __shared__ uint32_t thist[];   // [num_tiles]
    for (uint32_t c = threadIdx.x; c < p.C; c += blockDim.x) hist[c] = 0;
    for (uint32_t t = threadIdx.x; t < p.num_tiles; t += blockDim.x) thist[t] = 0;
    __syncthreads();
    // block b counts the sub-range b % csub of producer block b / csub's chunk
    const uint32_t S = p.csub ? p.csub : 1u;
    const uint64_t sub = (p.chunk + S - 1) / S;
    const uint64_t g0 = uint64_t(bid / S) * p.chunk;
    const uint64_t lo = g0 + uint64_t(bid % S) * sub;
    const uint64_t hi = min(min(lo + sub, g0 + p.chunk), p.n);
    const int cshift = p.tile_shift + kFineShift;
    bool oob = false;
    // (measured and not kept: the next U indices loaded before the current ones are counted,
    // C5 count 0.371 -> 0.366-0.387 ms)
    for (uint64_t k0 = lo + threadIdx.x; k0 < hi; k0 += U * uint64_t(blockDim.x)) {
        uint64_t ix[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t k = k0 + uint64_t(j) * blockDim.x;
            ix[j] = k < hi ? load_idx<IW>(p.idx, p.idx_stride, k) : ~uint64_t(0);
        }
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t k = k0 + uint64_t(j) * blockDim.x;
            if (k >= hi) continue;
            if (ix[j] >= p.shard_len) { oob = true; continue; }
            atomicAdd(&hist[uint32_t(ix[j] >> cshift)], 1u);
            atomicAdd(&thist[uint32_t(ix[j] >> p.tile_shift)], 1u);
        }
    }
    if (oob) raise_err(p.err, LMR_ERRBIT_OOB);
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < p.C; c += blockDim.x)
        p.coarse_off[uint64_t(c) * p.G * S + bid] = hist[c];
    uint32_t* row = p.trows + uint64_t(bid) * p.num_tiles;
    for (uint32_t t = threadIdx.x; t < p.num_tiles; t += blockDim.x) row[t] = thist[t];
}

struct PieceArgs {
    const uint32_t* tmp_idx;    // the region's temp records (region-relative slots)
    const uint8_t* tmp_val;     // null: every record carries scalar_bits
    uint64_t scalar_bits;
    int tile_shift;
    uint32_t num_tiles;
    uint32_t C;
    uint32_t* bstart;           // [C + 1] first temp slot of bucket c; bstart[C] = in-bounds records
    uint16_t* bin_lidx;         // workspace bases (binned positions are absolute)
    uint8_t* bin_val;
    uint32_t* rpos;             // region temp slot -> binned position (null: nothing returned)
    uint32_t R;                 // the region's first workspace slot
    uint32_t* ts;               // out: the region's tile starts (absolute binned positions)
    const uint32_t* ttot;       // the region's tile totals (k_coarse_scatter)
    uint32_t* tfill;            // per-tile records placed so far (zeroed by k_coarse_scatter)
    // round-wise un-partition (rt non-null): rpos holds as u16 slot k's position in its round's LDS
    // staging, and each round's tile runs are recorded, rt[round][f] = {binned start, length}
    // (round = piece * rpp + the round within the piece), with the piece table in ptab
    // (pbase[C + 1], bstart[C + 1]): k_unpart_rounds reads each round's runs back whole
    uint32_t* rt;
    uint32_t* ptab;
    uint32_t rpp;               // rounds per piece
};

// bucket starts (k_coarse_scatter's) -> pieces of kPiece records, computed by every block
// of k_fine_piece into its LDS (C <= 128 loads)
__device__ void piece_table(const uint32_t* bstart, uint32_t C, uint32_t* pb_s, uint32_t* bs_s, uint32_t* np_s,
                            uint32_t* tot) {
    const uint32_t c = threadIdx.x;
    const uint32_t total = bstart[C];
    if (c < C) {
        const uint32_t s = bstart[c];
        const uint32_t e = bstart[c + 1];
        bs_s[c] = s;
        np_s[c] = (e - s + kPiece - 1) / kPiece;
    }
    __syncthreads();
    small_excl_scan(np_s, pb_s, C, tot);
    __syncthreads();
    if (c == 0) {
        pb_s[C] = *tot;
        bs_s[C] = total;
    }
    __syncthreads();
}

struct PieceLoc { uint32_t c, p, np, lo, hi; };

// piece pid -> its bucket (the largest c with pbase[c] <= pid) and record range;
// pbase / bstart are the piece table in global memory or a block's LDS copy of it
__device__ __forceinline__ PieceLoc piece_loc(const uint32_t* pbase, const uint32_t* bstart, uint32_t C,
                                              uint32_t pid) {
    uint32_t lo_c = 0, hi_c = C;
    while (hi_c - lo_c > 1) {
        const uint32_t m = (lo_c + hi_c) >> 1;
        if (pbase[m] <= pid) lo_c = m; else hi_c = m;
    }
    PieceLoc L;
    L.c = lo_c;
    L.p = pid - pbase[lo_c];
    L.np = pbase[lo_c + 1] - pbase[lo_c];
    L.lo = bstart[lo_c] + L.p * kPiece;
    L.hi = min(L.lo + kPiece, bstart[lo_c + 1]);
    return L;
}

// fine level: each piece counting-sorted by tile in LDS rounds, written at its
// final binned positions (persistent over pieces)
template <int VB, int RPT>
__device__ __forceinline__ void fine_piece_body(const PieceArgs& a, const uint32_t bid, const uint32_t nblk) {
    using V = typename idx_t<VB>::I;
    constexpr uint32_t kRound = RPT * 1024;
    static_assert(kRound < 0xFFFFu, "round staging positions are u16");
    __shared__ uint32_t hist[kFine], base[kFine], cursor[kFine], tot;
    __shared__ uint32_t s_pb[kMaxCoarse + 1], s_bs[kMaxCoarse + 1], s_np[kMaxCoarse], s_tot;   // piece table
    __shared__ uint16_t s_l[kRound];
    __shared__ V s_val[kRound];
    __shared__ uint32_t s_tt[kFine], s_start[kFine];
    piece_table(a.bstart, a.C, s_pb, s_bs, s_np, &s_tot);
    const uint32_t npieces = s_pb[a.C];
    if (a.rt && bid == 0)
        for (uint32_t c = threadIdx.x; c <= a.C; c += blockDim.x) {
            a.ptab[c] = s_pb[c];
            a.ptab[a.C + 1 + c] = s_bs[c];
        }
    // tile starts of buckets with no piece (all their tiles empty) and the region's end
    if (bid == 0) {
        for (uint32_t t = threadIdx.x; t < a.num_tiles; t += blockDim.x) {
            const uint32_t c = t >> kFineShift;
            if (s_pb[c + 1] == s_pb[c]) a.ts[t] = a.R + s_bs[c];
        }
        if (threadIdx.x == 0) a.ts[a.num_tiles] = a.R + s_bs[a.C];
    }
    const uint32_t lmask = (1u << a.tile_shift) - 1u;
    const V sv = V(a.scalar_bits);
    // the next round's records are loaded into registers while the current round is
    // ranked and written out; each round reserves its tile runs with one atomic per tile
    // (positions within a tile follow no input order: the tile sweep applies them with atomics)
    uint32_t m_idx[RPT];
    V m_val[RPT];
    auto load_round = [&](uint32_t r0, uint32_t hi) {
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint32_t k = r0 + uint32_t(j) * 1024 + threadIdx.x;
            const bool in = k < hi;
            m_idx[j] = in ? a.tmp_idx[k] : 0u;
            m_val[j] = in ? (a.tmp_val ? reinterpret_cast<const V*>(a.tmp_val)[k] : sv) : V(0);
        }
    };
    auto load_piece = [&](const PieceLoc& L) { load_round(L.lo, L.hi); };
    uint32_t pid = bid;
    PieceLoc L{};
    if (pid < npieces) {
        L = piece_loc(s_pb, s_bs, a.C, pid);
        load_piece(L);
    }
    for (; pid < npieces; pid += nblk) {
        const uint32_t t0 = L.c * kFine;
        const uint32_t nf = min(uint32_t(kFine), a.num_tiles - t0);
        // this bucket's tile starts: bucket start + the tile totals before each tile; the
        // bucket's first piece publishes them as the region's tile starts
        if (threadIdx.x < kFine) s_tt[threadIdx.x] = threadIdx.x < nf ? a.ttot[t0 + threadIdx.x] : 0u;
        __syncthreads();
        small_excl_scan(s_tt, s_start, nf, &tot);
        __syncthreads();
        if (threadIdx.x < nf) {
            s_start[threadIdx.x] += a.R + s_bs[L.c];
            if (L.p == 0) a.ts[t0 + threadIdx.x] = s_start[threadIdx.x];
        }
        const uint32_t nxt = pid + nblk;
        PieceLoc LN{};
        if (nxt < npieces) LN = piece_loc(s_pb, s_bs, a.C, nxt);
        for (uint32_t r0 = L.lo; r0 < L.hi; r0 += kRound) {
            for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x) hist[f] = 0;
            __syncthreads();
            uint32_t m_rank[RPT], m_f[RPT];
#pragma unroll
            for (int j = 0; j < RPT; j++) {
                m_f[j] = (m_idx[j] >> a.tile_shift) - t0;
                if (r0 + uint32_t(j) * 1024 + threadIdx.x < L.hi) m_rank[j] = atomicAdd(&hist[m_f[j]], 1u);
            }
            __syncthreads();
            // (measured and not kept: the reservations' results consumed after the LDS staging,
            // rpos written after a barrier: C5 fine 0.613 -> 0.63 ms, C3 0.443 -> 0.47 ms)
            if (threadIdx.x < nf) {
                const uint32_t h = hist[threadIdx.x];
                cursor[threadIdx.x] = h ? s_start[threadIdx.x] + atomicAdd(&a.tfill[t0 + threadIdx.x], h) : 0u;
            }
            small_excl_scan(hist, base, nf, &tot);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < RPT; j++) {
                const uint32_t k = r0 + uint32_t(j) * 1024 + threadIdx.x;
                if (k >= L.hi) continue;
                const uint32_t q = base[m_f[j]] + m_rank[j];
                s_l[q] = uint16_t(m_idx[j] & lmask);
                s_val[q] = m_val[j];
                if (a.rpos) {
                    if (a.rt) reinterpret_cast<uint16_t*>(a.rpos)[k] = uint16_t(q);   // u16 map
                    else a.rpos[k] = cursor[m_f[j]] + m_rank[j];
                }
            }
            if (a.rt && threadIdx.x < kFine) {
                uint32_t* rr = a.rt + (uint64_t(pid) * a.rpp + (r0 - L.lo) / kRound) * (2 * kFine) + 2 * threadIdx.x;
                const bool in = threadIdx.x < nf;
                rr[0] = in ? cursor[threadIdx.x] : 0u;
                rr[1] = in ? hist[threadIdx.x] : 0u;
            }
            if (r0 + kRound < L.hi) load_round(r0 + kRound, L.hi);
            else if (nxt < npieces) load_piece(LN);
            __syncthreads();
            bucket_writeout(hist, base, cursor, nf, [&](uint32_t q, uint32_t dst) {
                a.bin_lidx[dst] = s_l[q];
                reinterpret_cast<V*>(a.bin_val)[dst] = s_val[q];
            });
            __syncthreads();
        }
        __syncthreads();
        L = LN;
    }
}

// ---- fused staged partition. The regions a session has staged since its last partition are
// partitioned together: one launch per pass (count, coarse, fine) for up to kFuse regions, each
// region keeping its own block range, count rows, tile totals and tables. Separate launches per
// region left most of each short launch to ramp and tail (C5: five 27M-record regions per step,
// count 0.075 ms at ~2.9 TB/s per launch) and ran the coarse pass one block per CU.
constexpr int kFuse = 8;
struct CountRegion {
    const uint8_t* idx;
    uint64_t idx_stride, n, chunk;
    uint32_t* coarse_off;       // the region's [C][G * csub] raw counts
    uint32_t* trows;            // the region's [G * csub][num_tiles] tile-count rows
    uint32_t G, csub, block0;
};
struct CountTable {
    CountRegion r[kFuse];
    uint32_t nr, num_tiles, C;
    int tile_shift;
    uint64_t shard_len;
    uint32_t* err;
};
struct CoarseRegion {
    const uint8_t* idx;
    uint64_t idx_stride;
    const uint8_t* val;
    uint64_t val_stride, n, chunk;
    uint32_t *coarse_off, *bstart_out, *total_out, *trows, *ttot, *tfill, *tmp_idx;
    uint8_t* tmp_val;
    uint32_t *qpos, *crt;
    uint32_t G, csub, rpb, block0;
};
struct CoarseTable {
    CoarseRegion r[kFuse];
    uint32_t nr, num_tiles, C;
    int tile_shift;
    uint64_t shard_len;
    uint32_t* err;
};
struct FineRegion {
    PieceArgs a;
    uint32_t block0, nblk;
};
struct FineTable {
    FineRegion r[kFuse];
    uint32_t nr;
};

template <int IW>
__global__ __launch_bounds__(1024) void k_ccount_stage(CountTable t) {
    uint32_t i = 0;
    while (i + 1 < t.nr && t.r[i + 1].block0 <= blockIdx.x) i++;
    const CountRegion& g = t.r[i];
    PartArgs p{};
    p.idx = g.idx; p.idx_stride = g.idx_stride; p.n = g.n; p.chunk = g.chunk;
    p.shard_len = t.shard_len; p.tile_shift = t.tile_shift; p.num_tiles = t.num_tiles; p.C = t.C;
    p.G = g.G; p.csub = g.csub; p.coarse_off = g.coarse_off; p.trows = g.trows; p.err = t.err;
    ccount_body<IW>(p, blockIdx.x - g.block0);
}

template <int IW, int VB, int RPT>
__global__ __launch_bounds__(1024) void k_coarse_stage(CoarseTable t) {
    uint32_t i = 0;
    while (i + 1 < t.nr && t.r[i + 1].block0 <= blockIdx.x) i++;
    const CoarseRegion& g = t.r[i];
    PartArgs p{};
    p.idx = g.idx; p.idx_stride = g.idx_stride; p.val = g.val; p.val_stride = g.val_stride; p.n = g.n;
    p.chunk = g.chunk; p.shard_len = t.shard_len; p.tile_shift = t.tile_shift; p.num_tiles = t.num_tiles;
    p.C = t.C; p.G = g.G; p.csub = g.csub; p.coarse_off = g.coarse_off; p.bstart_out = g.bstart_out;
    p.total_out = g.total_out; p.trows = g.trows; p.ttot = g.ttot; p.tfill = g.tfill; p.tmp_idx = g.tmp_idx;
    p.tmp_val = g.tmp_val; p.qpos = g.qpos; p.crt = g.crt; p.rpb = g.rpb; p.err = t.err;
    coarse_scatter_body<IW, VB, RPT>(p, blockIdx.x - g.block0);
}

template <int VB, int RPT>
__global__ __launch_bounds__(1024) void k_fine_stage(FineTable t) {
    uint32_t i = 0;
    while (i + 1 < t.nr && t.r[i + 1].block0 <= blockIdx.x) i++;
    const FineRegion& g = t.r[i];
    fine_piece_body<VB, RPT>(g.a, blockIdx.x - g.block0, g.nblk);
}

// Round-wise first gather of a staged region's un-partition: one block per fine-pass round. The
// round's tile runs of binned results (recorded by k_fine_piece) are read whole into LDS in the
// round's staging order, then every slot of the round takes its value from its staging position
// (rpos). Each run is read once, contiguously; the per-slot gather of binned positions it
// replaces read 1.7-1.8x its bytes (a partial line at every run end, runs of ~2-4 records).
// runs[0..nr) of src (start s_cur[f], length s_len[f], staging base s_base[f], nr <= 128,
// total tot) copied into LDS in staging order: staging position x lies in the last run starting at
// or before it (empty runs start where the next one does); every thread takes consecutive
// positions, U loads in flight (a wave per run left Zipf-hot runs to one wave)
static_assert(kFine == 128 && kMaxCoarse == 128, "runs_to_lds searches 128 runs");
template <typename V>
__device__ __forceinline__ void runs_to_lds(const uint32_t* s_cur, const uint32_t* s_base, uint32_t tot,
                                            const V* __restrict__ src, const uint8_t* __restrict__ oks, V* s_v,
                                            uint8_t* s_ok) {
    constexpr int U = 4;
    for (uint32_t x0 = threadIdx.x; x0 < tot; x0 += U * 1024) {
        uint32_t sp[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t x = min(x0 + uint32_t(u) * 1024, tot - 1);
            uint32_t lo_f = 0, hi_f = 128;
#pragma unroll
            for (int it = 0; it < 7; it++) {
                const uint32_t m = (lo_f + hi_f) >> 1;
                if (s_base[m] <= x) lo_f = m; else hi_f = m;
            }
            sp[u] = s_cur[lo_f] + (x - s_base[lo_f]);
        }
        V v[U];
        uint8_t o[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            v[u] = src[sp[u]];
            o[u] = oks ? oks[sp[u]] : uint8_t(0);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t x = x0 + uint32_t(u) * 1024;
            if (x < tot) {
                s_v[x] = v[u];
                s_ok[x] = o[u];
            }
        }
    }
}

struct RoundRegion {
    const uint32_t* rt;         // the region's run tables
    const uint32_t* ptab;       // pbase[C + 1], bstart[C + 1]
    const uint16_t* lpos;       // slot -> staging position in its round (u16)
    const uint8_t* src;         // binned results
    uint8_t* dst;               // results by slot
    const uint8_t* oks;
    uint8_t* okd;
    uint32_t C, rpp, block0;
};
struct RoundTable {
    RoundRegion r[kMaxRegions];
    uint32_t nr;
};

template <int VB, int RPT>
__global__ __launch_bounds__(1024) void k_unpart_rounds(RoundTable t) {
    using V = typename idx_t<VB>::I;
    constexpr uint32_t kRound = RPT * 1024;
    __shared__ V s_v[kRound];
    __shared__ uint8_t s_ok[kRound];
    __shared__ uint32_t s_cur[kFine], s_len[kFine], s_base[kFine], s_tot;
    uint32_t i = 0;
    while (i + 1 < t.nr && t.r[i + 1].block0 <= blockIdx.x) i++;
    const RoundRegion& g = t.r[i];
    const uint32_t b = blockIdx.x - g.block0;
    const uint32_t pid = b / g.rpp, j = b % g.rpp;
    const uint32_t* pbase = g.ptab;
    const uint32_t* bstart = g.ptab + g.C + 1;
    if (pid >= pbase[g.C]) return;                        // block-uniform
    const PieceLoc L = piece_loc(pbase, bstart, g.C, pid);
    const uint32_t lo = L.lo + j * kRound;
    if (lo >= L.hi) return;
    const uint32_t hi = min(lo + kRound, L.hi);
    if (threadIdx.x < kFine) {
        const uint32_t* rr = g.rt + uint64_t(b) * (2 * kFine) + 2 * threadIdx.x;
        s_cur[threadIdx.x] = rr[0];
        s_len[threadIdx.x] = rr[1];
    }
    __syncthreads();
    small_excl_scan(s_len, s_base, kFine, &s_tot);
    __syncthreads();
    runs_to_lds(s_cur, s_base, s_tot, reinterpret_cast<const V*>(g.src), g.oks, s_v, s_ok);
    __syncthreads();
    V* dst = reinterpret_cast<V*>(g.dst);
    for (uint32_t k = lo + threadIdx.x; k < hi; k += blockDim.x) {
        const uint32_t q = g.lpos[k];                     // (u16 map)
        dst[k] = s_v[q];
        if (g.oks) g.okd[k] = s_ok[q];
    }
}

// Round-wise second gather: one block per (region, producer block, coarse round). The round's
// bucket runs of temp-slot results are read whole into LDS in the round's staging order, then
// every record of the round takes its value from its staging position (qpos; ~0 = out of bounds).
struct CRoundRegion {
    const uint32_t* crt;        // the region's coarse run tables
    const uint16_t* qpos;       // record -> staging position in its round (u16, 0xFFFF: out of bounds)
    const uint8_t* src;         // results by temp slot
    uint8_t* dst;               // caller's results (arrival order)
    const uint8_t* oks;
    uint8_t* okd;
    uint64_t n, chunk;
    uint32_t rpb, block0;
};
struct CRoundTable {
    CRoundRegion r[kMaxRegions];
    uint32_t nr;
};

template <int VB, int RPT>
__global__ __launch_bounds__(1024) void k_unpart_crounds(CRoundTable t) {
    using V = typename idx_t<VB>::I;
    constexpr uint32_t kRound = RPT * 1024;
    __shared__ V s_v[kRound];
    __shared__ uint8_t s_ok[kRound];
    __shared__ uint32_t s_cur[kMaxCoarse], s_len[kMaxCoarse], s_base[kMaxCoarse], s_tot;
    uint32_t i = 0;
    while (i + 1 < t.nr && t.r[i + 1].block0 <= blockIdx.x) i++;
    const CRoundRegion& g = t.r[i];
    const uint32_t b = blockIdx.x - g.block0;
    const uint64_t lo = uint64_t(b / g.rpb) * g.chunk + uint64_t(b % g.rpb) * kRound;
    const uint64_t hi = min(min(uint64_t(b / g.rpb) * g.chunk + g.chunk, g.n), lo + kRound);
    if (lo >= hi) return;                                 // block-uniform
    if (threadIdx.x < kMaxCoarse) {
        const uint32_t* rr = g.crt + uint64_t(b) * (2 * kMaxCoarse) + 2 * threadIdx.x;
        s_cur[threadIdx.x] = rr[0];
        s_len[threadIdx.x] = rr[1];
    }
    __syncthreads();
    small_excl_scan(s_len, s_base, kMaxCoarse, &s_tot);
    __syncthreads();
    runs_to_lds(s_cur, s_base, s_tot, reinterpret_cast<const V*>(g.src), g.oks, s_v, s_ok);
    __syncthreads();
    V* dst = reinterpret_cast<V*>(g.dst);
    for (uint64_t k = lo + threadIdx.x; k < hi; k += blockDim.x) {
        const uint32_t q = g.qpos[k];
        if (q == 0xFFFFu) continue;
        dst[k] = s_v[q];
        if (g.okd) g.okd[k] = s_ok[q];
    }
}

// work plan when no tile splits (mixed sessions, ops that do not combine): an owner item per
// touched tile, one thread per tile over the whole grid (the one-block plan below took 14 us
// for C5's 4096 tiles x 5 regions)
__global__ void k_stage_plan_owner(const uint32_t* rts, uint32_t nreg, uint32_t stride, uint32_t num_tiles,
                                   TileItem* items, uint32_t* delta_count) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) *delta_count = 0;
    if (t >= num_tiles) return;
    uint32_t all = 0;
    for (uint32_t r = 0; r < nreg; r++) all += rts[uint64_t(r) * stride + t + 1] - rts[uint64_t(r) * stride + t];
    items[t] = TileItem{t, 0u, 0u, all ? 0u : 2u};
}

// work plan over all regions, one block: owner item per touched tile; a hot tile of a
// combinable op becomes delta pieces of <= kSplit records over each region's range
__global__ __launch_bounds__(1024) void k_stage_plan(const uint32_t* rts, uint32_t nreg, uint32_t stride,
                                                     uint32_t num_tiles, uint32_t thresh, int combinable,
                                                     TileItem* items, TileItem* delta, uint32_t* delta_count) {
    __shared__ uint32_t tot;
    uint32_t carry = 0;
    for (uint32_t t0 = 0; t0 < num_tiles; t0 += 1024) {
        const uint32_t t = t0 + threadIdx.x;
        uint32_t m = 0;
        if (t < num_tiles) {
            uint32_t all = 0, pieces = 0;
            for (uint32_t r = 0; r < nreg; r++) {
                const uint32_t c = rts[uint64_t(r) * stride + t + 1] - rts[uint64_t(r) * stride + t];
                all += c;
                pieces += (c + kSplit - 1) / kSplit;
            }
            m = (all == 0) ? 0u : ((combinable && all > thresh && pieces > 1) ? pieces : 1u);
        }
        const uint32_t x = m > 1 ? m : 0u;
        uint32_t j = carry + block_excl_scan(x, &tot);
        if (t < num_tiles) {
            items[t] = TileItem{t, 0u, 0u, m == 1 ? 0u : 2u};
            if (x)
                for (uint32_t r = 0; r < nreg; r++) {
                    const uint32_t lo = rts[uint64_t(r) * stride + t], hi = rts[uint64_t(r) * stride + t + 1];
                    for (uint32_t l = lo; l < hi; l += kSplit) delta[j++] = TileItem{t, l, min(hi, l + kSplit), 1u};
                }
        }
        carry += tot;
    }
    if (threadIdx.x == 0) *delta_count = carry;
}

// ---- count-free staged regions (order-insensitive integer ops, nothing returned)
// Every region's records go through k_coarse_free into the same per-bucket regions
// of the temp arrays (fill counters and per-block tile-count rows accumulate over the
// session); records that find their bucket region full are applied to the shard at
// once with device atomics (spill). The finish runs the tile totals, one k_fine_free
// over all buckets and one tile sweep: no per-region counting and no piece tables.
constexpr uint32_t kStageFreeBlocks = 256;
// blocks of one grouped k_coarse_free_stage launch, shared by its regions (LMR_FREE_GROUP_BLOCKS).
// One block per CU in all (the pass holds 144 KB of LDS per block): every block zeroes and writes
// a tile-count row and the tile totals read them all, so more blocks cost rows, not bandwidth.
// Two C2 batches in one session, same box (profiles/r4/ab/r4v_*, r4w_*): 1024 blocks 3.40-3.42 ms,
// 512 3.40, 256 3.06-3.21, 128 4.18-4.20; a lone region: 256 3.62, 128 4.42, 64 6.42 ms.
static uint32_t free_group_blocks() {
    static int v = env_int("LMR_FREE_GROUP_BLOCKS", kStageFreeBlocks, 32, kMaxBinBlocks);
    return uint32_t(v);
}
// Counted regions partitioned together share a block budget per pass (split over the group's
// regions; LMR_COUNT_GROUP_BLOCKS overrides, 0 = each region its own count): as with the count-free
// pass, every block adds count rows and a partial round per bucket, so a group of four to eight
// regions runs best with few blocks each. Same box (profiles/r4/ab/r4x_count_groups.log), two
// steps per session: C3 (8-byte values) 1.83 -> 1.68 ms at 512, 1.71 at 256; C5 (4-byte) 2.04 ->
// 1.93 at 512, 1.81 at 256.
static uint32_t count_group_blocks(int vb) {
    static int v = env_int("LMR_COUNT_GROUP_BLOCKS", -1, -1, 8 * kMaxBinBlocks);
    return v >= 0 ? uint32_t(v) : (vb == 8 ? 512u : 256u);
}
// blocks of a lone region's k_coarse_free_stage launch (LMR_FREE_BLOCKS)
static uint32_t free_single_blocks() {
    static int v = env_int("LMR_FREE_BLOCKS", kStageFreeBlocks, 16, kMaxBinBlocks);
    return uint32_t(v);
}
// paired loads in the staged count-free pass (LMR_FREE_STAGE_PAIRS=0: one record per load)
static bool free_stage_pairs() {
    static int v = env_int("LMR_FREE_STAGE_PAIRS", 1, 0, 1);
    return v != 0;
}

bool stage_free_applies(int dtype, int op, int ret, uint64_t shard_len, uint64_t cap) {
    return free_partition_applies(dtype, op, ret, shard_len, 0, cap);
}

static hipError_t stage_region_free(int dtype, int index_size, const ApplyArgs& a, const TiledWs& w,
                                    StageSession& s, hipStream_t st, const int64_t* n_dev = nullptr,
                                    uint64_t expect = 0) {
    (void)w; (void)st;
    if (s.nreg >= kMaxRegions) return hipErrorInvalidValue;
    // recorded; partitioned with the session's other pending regions (stage_partition_free)
    s.reg[s.nreg] = StageRegion{0, a.n, nullptr, nullptr, a.op, LMR_RET_NONE, a.cmp_bits, a.eps_bits};
    s.pend[s.nreg] = PendingRegion{a, index_size, n_dev};
    s.nreg += 1;
    // a device-count region counts its expected records (its capacity is an upper bound; the
    // session's bucket regions spill to device atomics if a stream brings more than expected)
    s.staged += n_dev ? std::min(expect, a.n) : a.n;
    return hipSuccess;
}

hipError_t launch_stage_region_dev(int dtype, int index_size, const ApplyArgs& a, const int64_t* n_dev,
                                   uint64_t expect, const TiledWs& w, StageSession& s, hipStream_t st) {
    if (a.n == 0) return hipSuccess;
    if (!s.free || !n_dev) return hipErrorInvalidValue;
    return stage_region_free(dtype, index_size, a, w, s, st, n_dev, expect);
}

// the pending count-free regions, k_coarse_free over groups of up to kFuseFree regions of one
// index width: a lone region keeps kStageFreeBlocks blocks, a group shares kMaxBinBlocks rows
static hipError_t stage_partition_free(const TiledWs& w, StageSession& s, hipStream_t st) {
    const int dtype = s.dtype, vb = dtype_bytes(dtype);
    while (s.parted < s.nreg) {
        const ApplyArgs& a0 = s.pend[s.parted].a;
        const int iw = s.pend[s.parted].iw;
        PartArgs q = free_args(dtype, a0, w, kStageFreeBlocks);
        q.accumulate = 1;                                  // tile-count rows add up over the session
        const int frpt = free_partition_rpt(dtype, a0.op, a0.ret, 0, q.num_tiles, w.tmp_cap);
        if (frpt == 0) return hipErrorInvalidValue;
        if (!s.free_armed) {                               // fill counters, tile-count rows
            hipError_t e = hipMemsetAsync(w.ff, 0, ff_words() * 4, st);
            if (e == hipSuccess) e = hipMemsetAsync(w.counts, 0, size_t(kMaxBinBlocks) * q.num_tiles * 4, st);
            if (e != hipSuccess) return e;
            s.free_armed = true;
        }
        int r1 = s.parted;
        while (r1 < s.nreg && r1 - s.parted < kFuseFree && s.pend[r1].iw == iw) r1++;
        const uint32_t nr = uint32_t(r1 - s.parted);
        const uint32_t gcap = nr == 1 ? free_single_blocks() : std::max<uint32_t>(32, free_group_blocks() / nr);
        FreeTable t{};
        uint32_t rows = 0;
        uint64_t n_all = 0;
        bool pairs = kCoarsePairs && iw == 8 && vb == 8 && (frpt % 2) == 0;
        for (uint32_t k = 0; k < nr; k++) {
            const ApplyArgs& a = s.pend[s.parted + int(k)].a;
            const uint32_t G = uint32_t(std::max<uint64_t>(1, std::min<uint64_t>((a.n + 16383) / 16384, gcap)));
            const uint64_t chunk = (a.n + G - 1) / G;
            const int64_t* nd = s.pend[s.parted + int(k)].n_dev;
            t.r[k] = FreeRegion{a.idx, a.idx_stride, a.val, a.val_stride, a.val_bits, a.n, chunk, G, rows, rows, nd};
            // paired 16-B loads (as the one-shot pass): contiguous, 16-B aligned u64 indices and
            // values, and every block's range whole pairs (even chunks, even n; a device-count
            // region's last pair may read one record past its count, inside its capacity + 1)
            pairs = pairs && a.idx_stride == 8 && a.val && a.val_stride == 8 && chunk % 2 == 0 && a.n % 2 == 0 &&
                    ((reinterpret_cast<uintptr_t>(a.idx) | reinterpret_cast<uintptr_t>(a.val)) & 15) == 0;
            rows += G;
            n_all += a.n;
        }
        t.nr = nr;
        s.free_rows = std::max(s.free_rows, rows);
        hipError_t e;
        {
            ProfScope ps(a0.prof, LMR_STAGE_BIN_SCATTER, st, n_all);
            e = dispatch_iw(iw, [&](auto iwt) {
                constexpr int IW = decltype(iwt)::value;
                dispatch_vb_rpt<4>(vb, frpt, [&](auto vbt, auto rpt) {
                    constexpr int VBc = decltype(vbt)::value, R = decltype(rpt)::value;
                    constexpr bool kP = IW == 8 && VBc == 8 && R % 2 == 0;
                    if (kP && pairs && free_stage_pairs())
                        hipLaunchKernelGGL((k_coarse_free_stage<IW, VBc, R, kP>), dim3(rows), dim3(1024),
                                           size_t(q.num_tiles) * 4, st, q, t);
                    else
                        hipLaunchKernelGGL((k_coarse_free_stage<IW, VBc, R, false>), dim3(rows), dim3(1024),
                                           size_t(q.num_tiles) * 4, st, q, t);
                });
                return hipGetLastError();
            });
        }
        if (e != hipSuccess) return e;
        s.parted = r1;
    }
    // partitioned count-free regions need nothing more (the sweep reads the shared bucket
    // regions): one entry stands for them all, so a session can take any number of streams
    if (s.nreg > 1) {
        s.reg[0] = s.reg[s.nreg - 1];
        s.nreg = s.parted = 1;
    }
    return hipSuccess;
}

static hipError_t stage_finish_free(const TiledWs& w, StageSession& s, hipStream_t st) {
    const ApplyArgs& a = s.a;
    const int dtype = s.dtype, vb = dtype_bytes(dtype);
    hipError_t e = stage_partition_free(w, s, st);
    PartArgs q = free_args(dtype, a, w, std::max<uint32_t>(s.free_rows, 1));
    if (e == hipSuccess) e = launch_free_finish(vb, q, w, s.staged, a.prof, st);
    // values are materialised in the bins (regions may mix array and scalar values)
    if (e == hipSuccess) e = launch_tile_sweep(dtype, a, w, q.num_tiles, s.staged, false, nullptr, nullptr, st);
    s.nreg = 0;
    s.parted = 0;
    s.staged = 0;
    s.free_armed = false;
    s.free_rows = 0;
    return e;
}

hipError_t launch_stage_region(int dtype, int index_size, const ApplyArgs& a, const TiledWs& w,
                               StageSession& s, hipStream_t st) {
    if (a.n == 0) return hipSuccess;
    if (s.free) return stage_region_free(dtype, index_size, a, w, s, st);
    const int shift = tile_shift_for(dtype);
    const uint64_t num_tiles = (a.shard_len + (uint64_t(1) << shift) - 1) >> shift;
    if (num_tiles == 0 || num_tiles > uint64_t(kMaxTiles) || a.n > kStageMaxRegion || s.nreg >= kMaxRegions)
        return hipErrorInvalidValue;
    // the region takes workspace slots [staged, staged + n) now; its records are partitioned
    // with the session's other pending regions (launch_stage_partition): the caller's record
    // buffers must stay valid until then
    const int r = s.nreg;
    s.reg[r] = StageRegion{s.staged, a.n, a.results, a.ok, a.op, a.ret, a.cmp_bits, a.eps_bits};
    s.pend[r] = PendingRegion{a, index_size};
    s.nreg = r + 1;
    s.staged += a.n;
    return hipSuccess;
}

// the regions [s.parted, s.nreg): count, coarse and fine passes, fused over groups of up to kFuse
// regions of one index width whose count rows fit the workspace
hipError_t launch_stage_partition(const TiledWs& w, StageSession& s, hipStream_t st) {
    if (s.free) return stage_partition_free(w, s, st);
    if (!s.wide_set && s.parted < s.nreg) {               // one partition layout per session
        s.wide = s.parted == 0 && wide_applies(s.dtype, s.pend[0].a.shard_len, w.cap);
        s.wide_set = true;
    }
    if (s.wide) return wide_partition(w, s, st);
    const int dtype = s.dtype, vb = dtype_bytes(dtype);
    const int shift = tile_shift_for(dtype);
    while (s.parted < s.nreg) {
        const ApplyArgs& a0 = s.pend[s.parted].a;
        const int iw = s.pend[s.parted].iw;
        const uint32_t T = uint32_t((a0.shard_len + (uint64_t(1) << shift) - 1) >> shift);
        const uint32_t C = (T + kFine - 1) / kFine;
        uint32_t kcround = 0, kround = 0;
        dispatch_vb_rpt<4>(vb, coarse_rpt(vb), [&](auto, auto rpt) { kcround = uint32_t(decltype(rpt)::value) * 1024; });
        dispatch_vb_rpt<2>(vb, piece_fine_rpt(vb), [&](auto, auto rpt) { kround = uint32_t(decltype(rpt)::value) * 1024; });
        const uint32_t rpp = (kPiece + kround - 1) / kround;
        CountTable ct{};
        CoarseTable cs{};
        FineTable ft{};
        uint64_t rows = 0;                                  // count rows of the group so far
        uint32_t cb = 0, gb = 0, fb = 0;
        uint64_t n_all = 0;
        int r = s.parted;
        // a group's regions share a block budget (LMR_COUNT_GROUP_BLOCKS; 0: each region its own)
        const uint32_t in_group = uint32_t(std::min<int>(kFuse, s.nreg - s.parted));
        const uint64_t gbudget = count_group_blocks(vb) && in_group > 1
                                     ? std::max<uint64_t>(32, count_group_blocks(vb) / in_group) : 0;
        for (; r < s.nreg && r - s.parted < kFuse && s.pend[r].iw == iw; r++) {
            const ApplyArgs& a = s.pend[r].a;
            StageRegion& g = s.reg[r];
            const bool has_res = a.ret != LMR_RET_NONE;
            uint64_t G = (a.n + 65535) / 65536;
            if (G > uint64_t(bin_blocks_cap(vb))) G = bin_blocks_cap(vb);
            if (gbudget && G > gbudget) G = gbudget;
            if (G < 1) G = 1;
            // count blocks per producer block: one 1024-thread block per CU leaves a lone
            // region's read-only count pass at half occupancy (LMR_CCOUNT_SPLIT)
            const uint64_t csub = std::max<uint64_t>(1, std::min<uint64_t>(ccount_split(), uint64_t(kMaxBinBlocks) / G));
            const uint64_t GS = G * csub;
            if (r > s.parted && ((rows + GS) * T > uint64_t(kMaxTiles) * kMaxBinBlocks ||
                                 (rows + GS) * C > uint64_t(kMaxCoarse) * kMaxBinBlocks))
                break;                                      // the next group takes it
            const uint64_t chunk = (a.n + G - 1) / G;
            const uint32_t R = uint32_t(g.base);
            const uint32_t k = uint32_t(r - s.parted);
            uint32_t* coarse_off = w.coarse_off + rows * C;
            uint32_t* trows = w.counts + rows * T;
            uint32_t* ptab = w.ptab + size_t(r) * 2 * (kMaxCoarse + 1);
            uint32_t* bstart = ptab + C + 1;                // the piece table's bucket starts
            uint32_t* ttot = w.rtot + size_t(r) * kMaxTiles;
            uint32_t* tfill = w.rfill + size_t(r) * kMaxTiles;
            ct.r[k] = CountRegion{a.idx, a.idx_stride, a.n, chunk, coarse_off, trows, uint32_t(G), uint32_t(csub), cb};
            cb += uint32_t(GS);
            // coarse run tables for the round-wise second un-partition gather
            const uint32_t rpb = uint32_t((chunk + kcround - 1) / kcround);
            const uint64_t ncr = G * rpb;
            const bool crounds = has_res && (unpart_rounds() & (vb == 8 ? 4 : 2)) && s.crounds + ncr <= w.crt_rounds;
            cs.r[k] = CoarseRegion{a.idx, a.idx_stride, a.val, a.val_stride, a.n, chunk, coarse_off, bstart,
                                   w.sinfo + kStageInb + r, trows, ttot, tfill, w.tmp_idx + R,
                                   a.val ? w.tmp_val + uint64_t(R) * vb : nullptr, has_res ? w.qpos + R : nullptr,
                                   crounds ? w.crtab + s.crounds * (2 * kMaxCoarse) : nullptr, uint32_t(G),
                                   uint32_t(csub), rpb, gb};
            gb += uint32_t(G);
            // run tables for the round-wise first gather: rpp rounds per piece
            const uint64_t max_pieces = (a.n + kPiece - 1) / kPiece + C;
            const uint64_t nrounds = max_pieces * rpp;
            const bool rounds = has_res && (unpart_rounds() & 1) && s.rounds + nrounds <= w.rt_rounds;
            PieceArgs pa;
            pa.tmp_idx = w.tmp_idx + R; pa.tmp_val = cs.r[k].tmp_val; pa.scalar_bits = a.val_bits;
            pa.tile_shift = shift; pa.num_tiles = T; pa.C = C; pa.bstart = bstart;
            pa.bin_lidx = w.bin_lidx; pa.bin_val = w.bin_val;
            pa.rpos = has_res ? w.rpos + R : nullptr; pa.R = R;
            pa.ts = w.rts + uint64_t(r) * (kMaxTiles + 1); pa.ttot = ttot; pa.tfill = tfill;
            pa.rt = rounds ? w.runtab + s.rounds * (2 * kFine) : nullptr;
            pa.ptab = ptab;
            pa.rpp = rpp;
            // (a group budget for the fine pass as for count / coarse measured no better: the fine
            // blocks are persistent over pieces, profiles/r4/ab/r4fa_*)
            const uint32_t fgrid = uint32_t(std::min<uint64_t>(max_pieces, uint64_t(fine_blocks_cap())));
            ft.r[k] = FineRegion{pa, fb, fgrid};
            fb += fgrid;
            g.round_base = uint32_t(s.rounds);
            g.kround = kround;
            g.nrounds = rounds ? uint32_t(nrounds) : 0u;
            g.cround_base = uint32_t(s.crounds);
            g.ncrounds = crounds ? uint32_t(ncr) : 0u;
            g.rpb = rpb;
            g.kcround = kcround;
            g.chunk = chunk;
            if (rounds) s.rounds += nrounds;
            if (crounds) s.crounds += ncr;
            rows += GS;
            n_all += a.n;
        }
        const uint32_t nr = uint32_t(r - s.parted);
        ct.nr = cs.nr = ft.nr = nr;
        ct.num_tiles = cs.num_tiles = T;
        ct.C = cs.C = C;
        ct.tile_shift = cs.tile_shift = shift;
        ct.shard_len = cs.shard_len = a0.shard_len;
        ct.err = cs.err = a0.err;
        hipError_t e;
        {
            ProfScope ps(a0.prof, LMR_STAGE_BIN_COUNT, st, n_all);
            e = dispatch_iw(iw, [&](auto iwt) {
                constexpr int IW = decltype(iwt)::value;
                hipLaunchKernelGGL((k_ccount_stage<IW>), dim3(cb), dim3(1024), size_t(T) * 4, st, ct);
                return hipGetLastError();
            });
        }
        if (e != hipSuccess) return e;
        {
            ProfScope ps(a0.prof, LMR_STAGE_BIN_SCATTER, st, n_all);
            e = dispatch_iw(iw, [&](auto iwt) {
                constexpr int IW = decltype(iwt)::value;
                dispatch_vb_rpt<4>(vb, coarse_rpt(vb), [&](auto vbt, auto rpt) {
                    constexpr int VBc = decltype(vbt)::value, RP = decltype(rpt)::value;
                    hipLaunchKernelGGL((k_coarse_stage<IW, VBc, RP>), dim3(gb), dim3(1024), 0, st, cs);
                });
                return hipGetLastError();
            });
        }
        if (e != hipSuccess) return e;
        {
            ProfScope ps(a0.prof, LMR_STAGE_FINE_SCATTER, st, n_all);
            dispatch_vb_rpt<2>(vb, piece_fine_rpt(vb), [&](auto vbt, auto rpt) {
                constexpr int VBc = decltype(vbt)::value, RP = decltype(rpt)::value;
                hipLaunchKernelGGL((k_fine_stage<VBc, RP>), dim3(fb), dim3(1024), 0, st, ft);
            });
            e = hipGetLastError();
        }
        if (e != hipSuccess) return e;
        s.parted = r;
    }
    return hipSuccess;
}

hipError_t launch_stage_finish(const TiledWs& w, StageSession& s, hipStream_t st) {
    if (s.nreg == 0) return hipSuccess;
    if (s.free) return stage_finish_free(w, s, st);
    {
        const hipError_t ep = launch_stage_partition(w, s, st);
        if (ep != hipSuccess) {
            s.nreg = s.parted = 0;
            s.staged = s.rounds = s.crounds = 0;
            s.wide = s.wide_set = false;
            s.wcnt = s.wrh = 0;
            return ep;
        }
    }
    const bool wide = s.wide;
    // the regions' op: every region's, or per region (mixed: op phases in staging order)
    ApplyArgs a = s.a;
    a.op = s.reg[0].op; a.ret = s.reg[0].ret; a.cmp_bits = s.reg[0].cmp_bits; a.eps_bits = s.reg[0].eps_bits;
    bool mixed = false;
    for (int r = 1; r < s.nreg; r++)
        mixed = mixed || s.reg[r].op != a.op || s.reg[r].cmp_bits != a.cmp_bits || s.reg[r].eps_bits != a.eps_bits;
    for (int r = 1; r < s.nreg; r++)
        if (s.reg[r].ret != LMR_RET_NONE && (a.ret == LMR_RET_NONE || s.reg[r].ret == LMR_RET_RESULT))
            a.ret = s.reg[r].ret;                                 // maps kept if any region returns
    const int dtype = s.dtype;
    const int shift = wide ? wide_shift(dtype_bytes(dtype)) : tile_shift_for(dtype);
    const uint32_t T = uint32_t((a.shard_len + (uint64_t(1) << shift) - 1) >> shift);
    const int vb = dtype_bytes(dtype);
    const uint32_t stride = uint32_t(kMaxTiles + 1);
    const bool has_res = a.ret != LMR_RET_NONE;
    // temps are free after the fine passes (the wide path's packed 16-B records live in tmp_val:
    // results then go to bin_val)
    uint8_t* const recs = wide ? wide_records(w, s) : w.bin_val;
    uint8_t* res_bin = recs == w.tmp_val ? w.bin_val : w.tmp_val;
    uint8_t* ok_bin = reinterpret_cast<uint8_t*>(w.tmp_idx);
    hipError_t e;
    {
        ProfScope ps(a.prof, LMR_STAGE_TILE_APPLY, st, s.staged);
        const uint64_t avg = (s.staged + T - 1) / T;
        const uint32_t thresh = uint32_t(std::min<uint64_t>(0xFFFFFFFFull, std::max<uint64_t>(delta_mul() * avg, delta_min())));
        TileItem* items = reinterpret_cast<TileItem*>(w.items);
        if (!mixed && op_combines(a.op))
            hipLaunchKernelGGL(k_stage_plan, dim3(1), dim3(1024), 0, st, w.rts, uint32_t(s.nreg), stride, T, thresh,
                               1, items, items + kMaxTiles, w.item_count);
        else
            hipLaunchKernelGGL(k_stage_plan_owner, dim3((T + 255) / 256), dim3(256), 0, st, w.rts, uint32_t(s.nreg),
                               stride, T, items, w.item_count);
        TileArgs t;
        t.shard = a.shard; t.shard_len = a.shard_len; t.tile_shift = shift;
        t.kind = a.kind; t.op = a.op; t.ret = a.ret;
        t.cmp_bits = a.cmp_bits; t.eps_bits = a.eps_bits; t.val_bits = 0;
        t.scalar = false;                                         // values are materialised in the bins
        t.items = items; t.delta = items + kMaxTiles; t.delta_count = w.item_count;
        t.num_tiles = T;
        t.bin_lidx = w.bin_lidx; t.bin_val = recs;
        t.results = res_bin; t.ok = ok_bin; t.err = a.err;
        t.rts = w.rts; t.nreg = uint32_t(s.nreg); t.rstride = stride;
        t.mixed = mixed ? 1 : 0;
        t.packed = wide && s.wpack ? 1 : 0;
        for (int r = 0; r < s.nreg; r++)
            t.rop[r] = RegionOp{s.reg[r].op, s.reg[r].ret, s.reg[r].cmp_bits, s.reg[r].eps_bits};
        // delta mode needs one combinable op; a mixed session's hot tiles stay with their owner
        const bool delta = !mixed && op_combines(a.op) && s.staged > thresh;
        const unsigned dgrid = unsigned(std::min<uint64_t>(2 * ((s.staged + kSplit - 1) / kSplit) + 2 * uint64_t(s.nreg),
                                                           uint64_t(tile_grid_cap())));
        e = launch_tile_kernels(dtype, mixed ? -1 : a.op, t, delta, dgrid, st, w.side, wide ? kWideBytes : kTileBytes);
    }
    if (e == hipSuccess && has_res && wide) {
        uint64_t n_ret = 0;
        for (int r = 0; r < s.nreg; r++)
            if (s.reg[r].results && s.reg[r].ret != LMR_RET_NONE) n_ret += s.reg[r].n;
        ProfScope pu(a.prof, LMR_STAGE_UNPARTITION, st, n_ret);
        e = wide_unpartition(w, s, res_bin, ok_bin, T, st);
    } else if (e == hipSuccess && has_res) {
        // binned -> temp slot (in-bounds slots of each region) -> arrival order
        uint64_t n_ret = 0;                                       // records whose op returns a value
        for (int r = 0; r < s.nreg; r++)
            if (s.reg[r].results && s.reg[r].ret != LMR_RET_NONE) n_ret += s.reg[r].n;
        ProfScope pu(a.prof, LMR_STAGE_UNPARTITION, st, n_ret);
        uint8_t* tmpres = w.bin_val;                              // bins are free after the tile sweep
        uint8_t* ok_tmp_all = (a.ret == LMR_RET_RESULT) ? reinterpret_cast<uint8_t*>(w.bin_lidx) : nullptr;
        const uint8_t* ok_src_all = (a.ret == LMR_RET_RESULT) ? ok_bin : nullptr;
        // every returning region's first gather in one launch (round-wise for the regions with run
        // tables, per slot for the rest), then every second gather
        UnpartTable t1{}, t2{};
        RoundTable tr{};
        CRoundTable tc{};
        uint32_t rblocks = 0, kround = 0, cblocks = 0, kcround = 0;
        for (int r = 0; r < s.nreg; r++) {
            const StageRegion& g = s.reg[r];
            if (!g.results || g.ret == LMR_RET_NONE) continue;
            uint8_t* ok_tmp = g.ret == LMR_RET_RESULT ? ok_tmp_all : nullptr;
            const uint8_t* ok_src = g.ret == LMR_RET_RESULT ? ok_src_all : nullptr;
            const bool want_ok = ok_tmp && g.ok;
            if (g.nrounds) {
                const uint32_t C = (T + kFine - 1) / kFine;
                tr.r[tr.nr++] = RoundRegion{w.runtab + uint64_t(g.round_base) * (2 * kFine),
                                            w.ptab + size_t(r) * 2 * (kMaxCoarse + 1),
                                            reinterpret_cast<const uint16_t*>(w.rpos + g.base), res_bin,
                                            tmpres + g.base * vb, ok_src, ok_tmp ? ok_tmp + g.base : nullptr, C,
                                            (kPiece + g.kround - 1) / g.kround, rblocks};
                rblocks += g.nrounds;
                kround = g.kround;
            } else
                t1.r[t1.nr++] = UnpartRegion{w.rpos + g.base, w.sinfo + kStageInb + r, g.n, 0, res_bin,
                                             tmpres + g.base * vb, ok_src, ok_tmp ? ok_tmp + g.base : nullptr, 0};
            if (g.ncrounds) {
                tc.r[tc.nr++] = CRoundRegion{w.crtab + uint64_t(g.cround_base) * (2 * kMaxCoarse),
                                             reinterpret_cast<const uint16_t*>(w.qpos + g.base),
                                             tmpres + g.base * vb, reinterpret_cast<uint8_t*>(g.results),
                                             want_ok ? ok_tmp + g.base : nullptr, want_ok ? g.ok : nullptr, g.n,
                                             g.chunk, g.rpb, cblocks};
                cblocks += g.ncrounds;
                kcround = g.kcround;
            } else
                t2.r[t2.nr++] = UnpartRegion{w.qpos + g.base, nullptr, g.n, 0, tmpres + g.base * vb,
                                             reinterpret_cast<uint8_t*>(g.results), want_ok ? ok_tmp + g.base : nullptr,
                                             want_ok ? g.ok : nullptr, 0};
        }
        if (tr.nr) {
            dispatch_vb_rpt<2>(vb, int(kround / 1024), [&](auto vbt, auto rpt) {
                constexpr int VBc = decltype(vbt)::value, RP = decltype(rpt)::value;
                hipLaunchKernelGGL((k_unpart_rounds<VBc, RP>), dim3(rblocks), dim3(1024), 0, st, tr);
            });
            e = hipGetLastError();
        }
        if (e == hipSuccess && t1.nr) e = launch_unpartition_multi(vb, t1, st);
        if (e == hipSuccess && tc.nr) {
            dispatch_vb_rpt<4>(vb, int(kcround / 1024), [&](auto vbt, auto rpt) {
                constexpr int VBc = decltype(vbt)::value, RP = decltype(rpt)::value;
                hipLaunchKernelGGL((k_unpart_crounds<VBc, RP>), dim3(cblocks), dim3(1024), 0, st, tc);
            });
            e = hipGetLastError();
        }
        if (e == hipSuccess && t2.nr) e = launch_unpartition_multi(vb, t2, st);
    }
    s.nreg = 0;
    s.parted = 0;
    s.staged = 0;
    s.rounds = 0;
    s.crounds = 0;
    s.wide = s.wide_set = false;
    s.wcnt = s.wrh = 0;
    return e;
}

}  // namespace lmr
