// lmr_wide.hip — the one-level ("wide") staged partition for 8-byte element shards of at most
// kWideMaxTiles 128 KiB tiles (2^24 elements: C3's 128 MiB f64 shard).
//
// The two-level staged path (lmr_apply.hip: count -> coarse -> fine -> tile sweep -> two
// un-partition gathers) moves ~116 B per fetch_add record for C3: each level costs a pass on the
// way in and a gather of the olds on the way back. Here every region is partitioned straight into
// its wide tiles, and its olds come back in one gather:
//   k_wcount_stage   per-(tile, producer block) counts, tile-major           idx 8 B
//   scan             one exclusive scan over the group's counts -> each (tile, block)'s binned
//                    slice; k_wide_starts turns them into the regions' tile starts
//   k_wide_stage     LDS rounds of kWideRound records ranked by tile and written as runs of each
//                    tile's slice (u16 offset in the tile + the value); per record its staging
//                    position (qpos, u16) and per round the tile counts (rhist, u16)
//                                                                            16 r + 12 w
//   tile sweep       k_tile_owner / k_tile_delta on 128 KiB tiles            10 r + 8 w (+ shard)
//   k_unpart_wide    the same blocks replay their rounds from rhist: each round's tile runs of
//                    olds read into LDS in staging order, every record takes its old at qpos
//                                                                            10 r + 8 w
// = 72 B per record against 116: an LDS round of 8K records over up to 1024 tiles writes runs of
// ~8 records (measured: tools/onelevel_probe.hip), so the scatter runs below the two-level
// passes' bandwidth but moves 40 B per record less, and one gather replaces two.
#include "lmr_tile.hpp"
#include "lmr_device.hpp"
#include <algorithm>
#include <cstdlib>

namespace lmr {

namespace {

#ifndef LMR_WIDE_RPT
#define LMR_WIDE_RPT 8
#endif
#ifndef LMR_WIDE_GATHER_U
#define LMR_WIDE_GATHER_U 4          // olds loads in flight per thread in k_unpart_wide
#endif
#ifndef LMR_WIDE_BLOCKS
#define LMR_WIDE_BLOCKS 256
#endif
constexpr uint32_t kWT = 1024;                        // threads per block
constexpr int kWideRpt = LMR_WIDE_RPT;                // records per thread per round
constexpr uint32_t kWideRound = kWideRpt * kWT;       // 8K records: 96 KB of LDS staging
static_assert(kWideRound <= 0xFFFFu, "staging positions and round counts are u16");
static_assert(kWideMaxTiles <= kWT, "one tile counter per thread");

template <int IW>
__device__ __forceinline__ uint64_t wload_idx(const uint8_t* base, uint64_t stride, uint64_t k) {
    using I = typename idx_t<IW>::I;
    return uint64_t(*reinterpret_cast<const I*>(base + k * stride));
}

// ---- per-region launch tables (block0: the region's first block of the fused launch)
struct WCountRegion {
    const uint8_t* idx;
    uint64_t idx_stride, n, chunk;
    uint32_t* cnt;              // [T][G] tile-major
    uint32_t G, block0;
};
struct WCountTable {
    WCountRegion r[kMaxRegions];
    uint32_t nr, T;
    int shift;
    uint64_t shard_len;
    uint32_t* err;
};

struct WStageRegion {
    const uint8_t* idx;
    uint64_t idx_stride;
    const uint8_t* val;         // null: every record carries val_bits
    uint64_t val_stride, val_bits, n, chunk;
    const uint32_t* cnt;        // scanned [T][G]: each (tile, block)'s slice, relative to gbase
    uint16_t* qpos;             // region slot -> staging position in its round (null: no results)
    uint16_t* rhist;            // [G * rpb][T] per-round tile counts (null: no results)
    uint32_t G, rpb, block0, gbase;
};
struct WStageTable {
    WStageRegion r[kMaxRegions];
    uint32_t nr, T;
    int shift;
    uint64_t shard_len;
    uint16_t* bin_lidx;
    uint64_t* bin_val;
};

struct WUnpartRegion {
    const uint32_t* cnt;
    const uint16_t* qpos;
    const uint16_t* rhist;
    uint8_t* dst;               // caller's results (arrival order)
    uint8_t* okd;               // caller's ok flags (RESULT ops), may be null
    uint64_t n, chunk;
    uint32_t G, rpb, block0, gbase;
};
struct WUnpartTable {
    WUnpartRegion r[kMaxRegions];
    uint32_t nr, T;
    const uint64_t* src;        // binned results
    const uint8_t* oks;         // binned ok flags, may be null
};

template <typename Tab>
__device__ __forceinline__ uint32_t region_of(const Tab& t) {
    uint32_t i = 0;
    while (i + 1 < t.nr && t.r[i + 1].block0 <= blockIdx.x) i++;
    return i;
}

template <int IW>
__global__ __launch_bounds__(1024) void k_wcount_stage(WCountTable t) {
    __shared__ uint32_t h[kWideMaxTiles];
    const WCountRegion& g = t.r[region_of(t)];
    const uint32_t b = blockIdx.x - g.block0;
    for (uint32_t x = threadIdx.x; x < t.T; x += kWT) h[x] = 0;
    __syncthreads();
    const uint64_t lo = uint64_t(b) * g.chunk, hi = min(lo + g.chunk, g.n);
    constexpr int U = 8;
    bool oob = false;
    for (uint64_t k0 = lo + threadIdx.x; k0 < hi; k0 += U * uint64_t(kWT)) {
        uint64_t ix[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t k = k0 + uint64_t(j) * kWT;
            ix[j] = k < hi ? wload_idx<IW>(g.idx, g.idx_stride, k) : ~uint64_t(0);
        }
#pragma unroll
        for (int j = 0; j < U; j++) {
            if (k0 + uint64_t(j) * kWT >= hi) continue;
            if (ix[j] >= t.shard_len) { oob = true; continue; }
            atomicAdd(&h[uint32_t(ix[j] >> t.shift)], 1u);
        }
    }
    if (oob) raise_err(t.err, LMR_ERRBIT_OOB);
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < t.T; x += kWT) g.cnt[uint64_t(x) * g.G + b] = h[x];
}

// tile starts of every region of the group: rts[r][x] = gbase + the first slice of tile x,
// rts[r][T] = the next region's first slice (the group total for the last)
struct WStartsTable {
    const uint32_t* cnt[kMaxRegions];
    uint32_t G[kMaxRegions];
    uint32_t* rts[kMaxRegions];
    uint32_t nr, T, gbase;
    const uint32_t* total;
};
__global__ __launch_bounds__(1024) void k_wide_starts(WStartsTable t) {
    const uint32_t k = blockIdx.x;
    for (uint32_t x = threadIdx.x; x <= t.T; x += kWT) {
        uint32_t v;
        if (x < t.T) v = t.cnt[k][uint64_t(x) * t.G[k]];
        else v = k + 1 < t.nr ? t.cnt[k + 1][0] : *t.total;
        t.rts[k][x] = t.gbase + v;
    }
}

template <int IW>
__global__ __launch_bounds__(1024) void k_wide_stage(WStageTable t) {
    __shared__ uint32_t hist[kWideMaxTiles], base[kWideMaxTiles], cursor[kWideMaxTiles], s_tot;
    __shared__ uint16_t s_l[kWideRound], s_b[kWideRound];
    __shared__ uint64_t s_v[kWideRound];
    const WStageRegion& g = t.r[region_of(t)];
    const uint32_t b = blockIdx.x - g.block0;
    const uint32_t T = t.T;
    for (uint32_t x = threadIdx.x; x < T; x += kWT) cursor[x] = g.gbase + g.cnt[uint64_t(x) * g.G + b];
    const uint64_t lo = uint64_t(b) * g.chunk, hi = min(lo + g.chunk, g.n);
    const uint32_t lmask = (1u << t.shift) - 1u;
    uint64_t m_raw[kWideRpt], m_val[kWideRpt];
    auto load_round = [&](uint64_t r0) {
#pragma unroll
        for (int j = 0; j < kWideRpt; j++) {
            const uint64_t k = r0 + uint64_t(j) * kWT + threadIdx.x;
            const bool in = k < hi;
            m_raw[j] = in ? wload_idx<IW>(g.idx, g.idx_stride, k) : ~uint64_t(0);
            m_val[j] = g.val ? (in ? *reinterpret_cast<const uint64_t*>(g.val + k * g.val_stride) : 0ull) : g.val_bits;
        }
    };
    if (lo < hi) load_round(lo);
    uint32_t rid = b * g.rpb;
    for (uint64_t r0 = lo; r0 < hi; r0 += kWideRound, rid++) {
        for (uint32_t x = threadIdx.x; x < T; x += kWT) hist[x] = 0;
        __syncthreads();
        uint32_t m_rank[kWideRpt], m_t[kWideRpt];
        bool m_ok[kWideRpt];
#pragma unroll
        for (int j = 0; j < kWideRpt; j++) {
            m_ok[j] = m_raw[j] < t.shard_len;
            m_t[j] = m_ok[j] ? uint32_t(m_raw[j] >> t.shift) : 0u;
            if (m_ok[j]) m_rank[j] = atomicAdd(&hist[m_t[j]], 1u);
        }
        __syncthreads();
        {
            const uint32_t h = threadIdx.x < T ? hist[threadIdx.x] : 0u;
            const uint32_t e = block_excl_scan(h, &s_tot);
            if (threadIdx.x < T) {
                base[threadIdx.x] = e;
                if (g.rhist) g.rhist[uint64_t(rid) * T + threadIdx.x] = uint16_t(h);
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kWideRpt; j++) {
            const uint64_t k = r0 + uint64_t(j) * kWT + threadIdx.x;
            if (!m_ok[j]) {
                if (g.qpos && k < hi) g.qpos[k] = 0xFFFFu;
                continue;
            }
            const uint32_t q = base[m_t[j]] + m_rank[j];
            s_l[q] = uint16_t(m_raw[j] & lmask);
            s_b[q] = uint16_t(m_t[j]);
            s_v[q] = m_val[j];
            if (g.qpos) g.qpos[k] = uint16_t(q);                   // coalesced in k
        }
        if (r0 + kWideRound < hi) load_round(r0 + kWideRound);    // next round in flight
        __syncthreads();
        const uint32_t tot = s_tot;
        for (uint32_t q = threadIdx.x; q < tot; q += kWT) {
            const uint32_t x = s_b[q];
            const uint32_t dst = cursor[x] + (q - base[x]);
            t.bin_lidx[dst] = s_l[q];
            t.bin_val[dst] = s_v[q];
        }
        __syncthreads();
        for (uint32_t x = threadIdx.x; x < T; x += kWT) cursor[x] += hist[x];
    }
}

// the olds of one round (tile runs at cursor[x], length hist[x], staging base base[x]) into LDS in
// staging order: position p lies in the last run starting at or before it; U loads in flight
template <bool OK>
__device__ __forceinline__ void wruns_to_lds(const uint32_t* cursor, const uint32_t* base, uint32_t T,
                                             uint32_t tot, const uint64_t* __restrict__ src,
                                             const uint8_t* __restrict__ oks, uint64_t* s_v, uint8_t* s_ok) {
    constexpr int U = LMR_WIDE_GATHER_U;
    for (uint32_t p0 = threadIdx.x; p0 < tot; p0 += U * kWT) {
        uint32_t sp[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t p = min(p0 + uint32_t(u) * kWT, tot - 1);
            uint32_t lo_x = 0, hi_x = T;
            while (hi_x - lo_x > 1) {
                const uint32_t m = (lo_x + hi_x) >> 1;
                if (base[m] <= p) lo_x = m; else hi_x = m;
            }
            // (an empty run starts where the next one does, so the last run starting at or
            // before p is never an empty one)
            sp[u] = cursor[lo_x] + (p - base[lo_x]);
        }
        uint64_t v[U];
        uint8_t o[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            v[u] = src[sp[u]];
            if constexpr (OK) o[u] = oks[sp[u]];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t p = p0 + uint32_t(u) * kWT;
            if (p < tot) {
                s_v[p] = v[u];
                if constexpr (OK) s_ok[p] = o[u];
            }
        }
    }
}

template <bool OK>
__global__ __launch_bounds__(1024) void k_unpart_wide(WUnpartTable t) {
    __shared__ uint32_t hist[kWideMaxTiles], base[kWideMaxTiles], cursor[kWideMaxTiles], s_tot;
    __shared__ uint64_t s_v[kWideRound];
    __shared__ uint8_t s_ok[OK ? kWideRound : 1];
    const WUnpartRegion& g = t.r[region_of(t)];
    const uint32_t b = blockIdx.x - g.block0;
    const uint32_t T = t.T;
    for (uint32_t x = threadIdx.x; x < T; x += kWT) cursor[x] = g.gbase + g.cnt[uint64_t(x) * g.G + b];
    const uint64_t lo = uint64_t(b) * g.chunk, hi = min(lo + g.chunk, g.n);
    uint32_t rid = b * g.rpb;
    for (uint64_t r0 = lo; r0 < hi; r0 += kWideRound, rid++) {
        const uint32_t h = threadIdx.x < T ? uint32_t(g.rhist[uint64_t(rid) * T + threadIdx.x]) : 0u;
        const uint32_t e = block_excl_scan(h, &s_tot);
        if (threadIdx.x < T) {
            hist[threadIdx.x] = h;
            base[threadIdx.x] = e;
        }
        __syncthreads();
        wruns_to_lds<OK>(cursor, base, T, s_tot, t.src, t.oks, s_v, s_ok);
        __syncthreads();
        const uint64_t rhi = min(r0 + kWideRound, hi);
        for (uint64_t k = r0 + threadIdx.x; k < rhi; k += kWT) {
            const uint32_t q = g.qpos[k];
            if (q == 0xFFFFu) continue;
            reinterpret_cast<uint64_t*>(g.dst)[k] = s_v[q];
            if constexpr (OK) if (g.okd) g.okd[k] = s_ok[q];
        }
        __syncthreads();
        for (uint32_t x = threadIdx.x; x < T; x += kWT) cursor[x] += hist[x];
    }
}

template <typename F>
hipError_t wdispatch_iw(int iw, F&& f) {
    switch (iw) {
    case 1: return f(std::integral_constant<int, 1>{});
    case 2: return f(std::integral_constant<int, 2>{});
    case 4: return f(std::integral_constant<int, 4>{});
    case 8: return f(std::integral_constant<int, 8>{});
    default: return hipErrorInvalidValue;
    }
}

int wide_env() {
    static const int v = [] {
        const char* e = getenv("LMR_WIDE");
        return e && *e ? atoi(e) : 1;
    }();
    return v;
}

// producer blocks of a region: one per 64K records (at least), at most kWideBlocks
constexpr uint32_t kWideBlocks = LMR_WIDE_BLOCKS;
uint32_t wide_blocks(uint64_t n) {
    return uint32_t(std::max<uint64_t>(1, std::min<uint64_t>((n + 65535) / 65536, kWideBlocks)));
}

}  // namespace

bool wide_applies(int dtype, uint64_t shard_len, uint64_t cap) {
    if (!wide_env() || dtype_bytes(dtype) != 8) return false;
    const uint64_t tiles = (shard_len + (uint64_t(1) << kWideShift8) - 1) >> kWideShift8;
    // the per-round tile counts live in the position map rpos (4 B per slot, unused by this path).
    // A region of n records has G <= ceil(n / 64K) blocks of whole rounds: <= n / R + n / 64K + 1
    // rounds of R records, so a session's counts fit when (cap / R + cap / 64K + kMaxRegions)
    // rounds of `tiles` u16 do
    const uint64_t rh_entries = (cap / kWideRound + cap / 65536 + kMaxRegions) * tiles;
    return tiles >= 1 && tiles <= kWideMaxTiles && rh_entries <= cap * 2;
}

hipError_t wide_partition(const TiledWs& w, StageSession& s, hipStream_t st) {
    const int shift = kWideShift8;
    while (s.parted < s.nreg) {
        const ApplyArgs& a0 = s.pend[s.parted].a;
        const int iw = s.pend[s.parted].iw;
        const uint32_t T = uint32_t((a0.shard_len + (uint64_t(1) << shift) - 1) >> shift);
        WCountTable ct{};
        WStageTable sc{};
        WStartsTable ws{};
        const uint64_t cnt0 = s.wcnt;
        uint32_t blocks = 0;
        uint64_t n_all = 0;
        int r = s.parted;
        const uint32_t gbase = uint32_t(s.reg[r].base);
        for (; r < s.nreg && s.pend[r].iw == iw; r++) {
            const ApplyArgs& a = s.pend[r].a;
            StageRegion& g = s.reg[r];
            const uint32_t G = wide_blocks(a.n);
            if (s.wcnt + uint64_t(G) * T > uint64_t(kMaxTiles) * kMaxBinBlocks) {
                if (r == s.parted) return hipErrorInvalidValue;
                break;                                             // the next group takes it
            }
            const uint64_t chunk = ((a.n + G - 1) / G + kWideRound - 1) / kWideRound * kWideRound;
            const uint32_t rpb = uint32_t(chunk / kWideRound);
            const bool has_res = a.ret != LMR_RET_NONE && g.results;
            const uint64_t nrh = has_res ? uint64_t(G) * rpb * T : 0;
            if (s.wrh + nrh > w.cap * 2) return hipErrorInvalidValue;     // (wide_applies sized it)
            uint32_t* cnt = w.counts + s.wcnt;
            uint16_t* rh = has_res ? reinterpret_cast<uint16_t*>(w.rpos) + s.wrh : nullptr;
            const uint32_t k = uint32_t(r - s.parted);
            ct.r[k] = WCountRegion{a.idx, a.idx_stride, a.n, chunk, cnt, G, blocks};
            sc.r[k] = WStageRegion{a.idx, a.idx_stride, a.val, a.val_stride, a.val_bits, a.n, chunk, cnt,
                                   has_res ? reinterpret_cast<uint16_t*>(w.qpos) + g.base : nullptr, rh, G, rpb,
                                   blocks, gbase};
            ws.cnt[k] = cnt;
            ws.G[k] = G;
            ws.rts[k] = w.rts + uint64_t(r) * (kMaxTiles + 1);
            g.wcnt = s.wcnt;
            g.wrh = s.wrh;
            g.wg = G;
            g.rpb = rpb;
            g.chunk = chunk;
            g.wbase = gbase;
            g.wres = has_res;
            s.wcnt += uint64_t(G) * T;
            s.wrh += nrh;
            blocks += G;
            n_all += a.n;
        }
        const uint32_t nr = uint32_t(r - s.parted);
        ct.nr = sc.nr = ws.nr = nr;
        ct.T = sc.T = ws.T = T;
        ct.shift = sc.shift = shift;
        ct.shard_len = sc.shard_len = a0.shard_len;
        ct.err = a0.err;
        sc.bin_lidx = w.bin_lidx;
        sc.bin_val = reinterpret_cast<uint64_t*>(w.bin_val);
        ws.gbase = gbase;
        ws.total = w.total;
        hipError_t e;
        {
            ProfScope ps(a0.prof, LMR_STAGE_BIN_COUNT, st, n_all);
            e = wdispatch_iw(iw, [&](auto iwt) {
                hipLaunchKernelGGL((k_wcount_stage<decltype(iwt)::value>), dim3(blocks), dim3(kWT), 0, st, ct);
                return hipGetLastError();
            });
            if (e == hipSuccess) e = scan_exclusive_u32(w.counts + cnt0, s.wcnt - cnt0, w.partials, w.total, st);
            if (e == hipSuccess) {
                hipLaunchKernelGGL(k_wide_starts, dim3(nr), dim3(kWT), 0, st, ws);
                e = hipGetLastError();
            }
        }
        if (e != hipSuccess) return e;
        {
            ProfScope ps(a0.prof, LMR_STAGE_BIN_SCATTER, st, n_all);
            e = wdispatch_iw(iw, [&](auto iwt) {
                hipLaunchKernelGGL((k_wide_stage<decltype(iwt)::value>), dim3(blocks), dim3(kWT), 0, st, sc);
                return hipGetLastError();
            });
        }
        if (e != hipSuccess) return e;
        s.parted = r;
    }
    return hipSuccess;
}

hipError_t wide_unpartition(const TiledWs& w, const StageSession& s, const uint8_t* res_bin, const uint8_t* ok_bin,
                            uint32_t T, hipStream_t st) {
    WUnpartTable t{};
    t.T = T;
    t.src = reinterpret_cast<const uint64_t*>(res_bin);
    bool ok = false;
    uint32_t blocks = 0;
    for (int r = 0; r < s.nreg; r++) {
        const StageRegion& g = s.reg[r];
        if (!g.wres || !g.results || g.ret == LMR_RET_NONE) continue;
        const bool want_ok = g.ret == LMR_RET_RESULT && g.ok;
        ok = ok || want_ok;
        t.r[t.nr++] = WUnpartRegion{w.counts + g.wcnt, reinterpret_cast<const uint16_t*>(w.qpos) + g.base,
                                    reinterpret_cast<const uint16_t*>(w.rpos) + g.wrh,
                                    reinterpret_cast<uint8_t*>(g.results), want_ok ? g.ok : nullptr, g.n, g.chunk,
                                    g.wg, g.rpb, blocks, g.wbase};
        blocks += g.wg;
    }
    if (!t.nr) return hipSuccess;
    if (ok) {
        t.oks = ok_bin;
        hipLaunchKernelGGL(k_unpart_wide<true>, dim3(blocks), dim3(kWT), 0, st, t);
    } else {
        hipLaunchKernelGGL(k_unpart_wide<false>, dim3(blocks), dim3(kWT), 0, st, t);
    }
    return hipGetLastError();
}

}  // namespace lmr
