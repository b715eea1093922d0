// lmr_wide.hip — the one-level ("wide") staged partition into 128 KiB tiles: 8-byte element
// shards of at most kWideMaxTiles tiles (2^24 elements: C3's 128 MiB f64 shard), and 1/2/4-byte
// element shards of at most kWideMaxTiles4 tiles of 32-bit LDS words (2^26 elements: C5's 256 MiB
// u32 shard).
//
// The two-level staged path (lmr_apply.hip: count -> coarse -> fine -> tile sweep -> two
// un-partition gathers) moves ~116 B per fetch_add record for C3: each level costs a pass on the
// way in and a gather of the olds on the way back. Here every region is partitioned straight into
// its wide tiles, and its olds come back in one gather (8-byte values; 4-byte values in brackets):
//   k_wcount_stage   per-(tile, producer block) counts, tile-major           idx 8 B
//   scan             one exclusive scan over the group's counts -> each (tile, block)'s binned
//                    slice; k_wide_starts turns them into the regions' tile starts
//   k_wide_stage     LDS rounds of R records (8K; [16K]) ranked by tile and written as runs of each
//                    tile's slice (u16 offset in the tile + the value); per record its staging
//                    position (qpos, u16) and per round the tile counts (rhist, u16)
//                                                                            16 r + 12 w  [12 r + 6 w]
//   tile sweep       k_tile_owner / k_tile_delta on 128 KiB tiles            10 r + 8 w   [6 r + 4 w] (+ shard)
//   k_unpart_wide    the same blocks replay their rounds from rhist: each round's tile runs of
//                    olds read into LDS in staging order, every record takes its old at qpos
//                                                                            10 r + 8 w   [6 r + 4 w]
// = 72 B per record against 116 (C3): an LDS round of R records over up to 1024 [2048] tiles writes
// runs of ~8 records (measured: tools/onelevel_probe.hip), so the scatter runs below the two-level
// passes' bandwidth but moves fewer bytes per record, and one gather replaces two. For 4-byte values
// a 16K-record round stages 8 B per record (u16 offset, u16 tile, u32 value: 128 KB of gfx950's
// 160 KiB LDS), so runs over 2048 tiles keep C3's length.
#include "lmr_tile.hpp"
#include "lmr_device.hpp"
#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace lmr {

namespace {

#ifndef LMR_WIDE_RPT
#define LMR_WIDE_RPT 8
#endif
#ifndef LMR_WIDE4_RPT
#define LMR_WIDE4_RPT 16
#endif
#ifndef LMR_WIDE_GATHER_U
#define LMR_WIDE_GATHER_U 4          // olds loads in flight per thread in k_unpart_wide
#endif
#ifndef LMR_WIDE_BLOCKS
#define LMR_WIDE_BLOCKS 256
#endif
constexpr uint32_t kWT = 1024;                        // threads per block

// the geometry of a value width: records per thread and round, tiles, LDS staging word
template <int VB>
struct WGeom {
    static constexpr int kRpt = VB == 8 ? LMR_WIDE_RPT : LMR_WIDE4_RPT;
    static constexpr uint32_t kRound = uint32_t(kRpt) * kWT;        // 8K (8-byte) / 16K records
    static constexpr uint32_t kMaxT = VB == 8 ? kWideMaxTiles : kWideMaxTiles4;
    static constexpr uint32_t kPer = kMaxT / kWT;                   // tile counters per thread
    using S = std::conditional_t<VB == 8, uint64_t, uint32_t>;     // LDS staging word of a value
    using V = std::conditional_t<VB == 8, uint64_t, std::conditional_t<VB == 4, uint32_t,
                                 std::conditional_t<VB == 2, uint16_t, uint8_t>>>;
    static_assert(kRound <= 0xFFFFu, "staging positions and round counts are u16");
    static_assert(kMaxT % kWT == 0, "whole tile counters per thread");
};
static_assert(WGeom<8>::kRound * (2 + 2 + 8) + 3 * 4 * WGeom<8>::kMaxT <= 160 * 1024, "8-byte stage LDS");
static_assert(WGeom<4>::kRound * (2 + 2 + 4) + 3 * 4 * WGeom<4>::kMaxT + 256 <= 160 * 1024, "4-byte stage LDS");

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
    uint8_t* bin_val;           // values of VB bytes
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
    const uint8_t* src;         // binned results (VB bytes each)
    const uint8_t* oks;         // binned ok flags, may be null
};

template <typename Tab>
__device__ __forceinline__ uint32_t region_of(const Tab& t) {
    uint32_t i = 0;
    while (i + 1 < t.nr && t.r[i + 1].block0 <= blockIdx.x) i++;
    return i;
}

// exclusive scan of the round's tile counts (kPer consecutive counters per thread): base[x],
// and the counts themselves to rhist (a returning region) and hist_out (when not null)
template <uint32_t PER>
__device__ __forceinline__ void wscan_tiles(const uint32_t* hist, uint32_t* base, uint32_t T, uint32_t* s_tot,
                                            uint16_t* rhist_row, uint32_t* hist_out) {
    uint32_t hv[PER];
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t p = 0; p < PER; p++) {
        const uint32_t x = threadIdx.x * PER + p;
        hv[p] = x < T ? hist[x] : 0u;
        sum += hv[p];
    }
    uint32_t e = block_excl_scan(sum, s_tot);
#pragma unroll
    for (uint32_t p = 0; p < PER; p++) {
        const uint32_t x = threadIdx.x * PER + p;
        if (x < T) {
            base[x] = e;
            if (rhist_row) rhist_row[x] = uint16_t(hv[p]);
            if (hist_out) hist_out[x] = hv[p];
        }
        e += hv[p];
    }
}

template <int IW, int MT>
__global__ __launch_bounds__(1024) void k_wcount_stage(WCountTable t) {
    __shared__ uint32_t h[MT];
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

// PK: packed records (VB <= 4): one uint2 {tile-local index, value bits} per record in bin_val,
// one 8-B store per record (a run of ~8 records is 64 contiguous bytes) instead of a u16 offset
// and a value in two arrays (runs of 16 and 32 bytes: two partial-line writes per run)
template <int IW, int VB, bool PK>
__global__ __launch_bounds__(1024) void k_wide_stage(WStageTable t) {
    using Gm = WGeom<VB>;
    using S = typename Gm::S;
    using V = typename Gm::V;
    constexpr int kRpt = Gm::kRpt;
    constexpr uint32_t kRound = Gm::kRound;
    __shared__ uint32_t hist[Gm::kMaxT], base[Gm::kMaxT], cursor[Gm::kMaxT], s_tot;
    __shared__ uint16_t s_l[kRound], s_b[kRound];
    __shared__ S s_v[kRound];
    const WStageRegion& g = t.r[region_of(t)];
    const uint32_t b = blockIdx.x - g.block0;
    const uint32_t T = t.T;
    V* bin_val = reinterpret_cast<V*>(t.bin_val);
    for (uint32_t x = threadIdx.x; x < T; x += kWT) cursor[x] = g.gbase + g.cnt[uint64_t(x) * g.G + b];
    const uint64_t lo = uint64_t(b) * g.chunk, hi = min(lo + g.chunk, g.n);
    const uint32_t lmask = (1u << t.shift) - 1u;
    uint64_t m_raw[kRpt];
    S m_val[kRpt];
    auto load_round = [&](uint64_t r0) {
#pragma unroll
        for (int j = 0; j < kRpt; j++) {
            const uint64_t k = r0 + uint64_t(j) * kWT + threadIdx.x;
            const bool in = k < hi;
            m_raw[j] = in ? wload_idx<IW>(g.idx, g.idx_stride, k) : ~uint64_t(0);
            m_val[j] = g.val ? (in ? S(*reinterpret_cast<const V*>(g.val + k * g.val_stride)) : S(0)) : S(g.val_bits);
        }
    };
    if (lo < hi) load_round(lo);
    uint32_t rid = b * g.rpb;
    for (uint64_t r0 = lo; r0 < hi; r0 += kRound, rid++) {
        for (uint32_t x = threadIdx.x; x < T; x += kWT) hist[x] = 0;
        __syncthreads();
        // (tile << 16 | rank in the round's tile run), all ones out of bounds: one register a record
        uint32_t m_key[kRpt];
#pragma unroll
        for (int j = 0; j < kRpt; j++) {
            const bool ok = m_raw[j] < t.shard_len;
            const uint32_t x = uint32_t(m_raw[j] >> t.shift);
            m_key[j] = ok ? (x << 16) | atomicAdd(&hist[x], 1u) : ~0u;
        }
        __syncthreads();
        wscan_tiles<Gm::kPer>(hist, base, T, &s_tot, g.rhist ? g.rhist + uint64_t(rid) * T : nullptr, nullptr);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kRpt; j++) {
            const uint64_t k = r0 + uint64_t(j) * kWT + threadIdx.x;
            if (m_key[j] == ~0u) {
                if (g.qpos && k < hi) g.qpos[k] = 0xFFFFu;
                continue;
            }
            const uint32_t x = m_key[j] >> 16;
            const uint32_t q = base[x] + (m_key[j] & 0xFFFFu);
            s_l[q] = uint16_t(m_raw[j] & lmask);
            s_b[q] = uint16_t(x);
            s_v[q] = m_val[j];
            if (g.qpos) g.qpos[k] = uint16_t(q);                   // coalesced in k
        }
        if (r0 + kRound < hi) load_round(r0 + kRound);            // next round in flight
        __syncthreads();
        const uint32_t tot = s_tot;
        for (uint32_t q = threadIdx.x; q < tot; q += kWT) {
            const uint32_t x = s_b[q];
            const uint32_t dst = cursor[x] + (q - base[x]);
            if constexpr (PK && VB == 8) {
                const uint64_t v = uint64_t(s_v[q]);
                reinterpret_cast<uint4*>(t.bin_val)[dst] = make_uint4(s_l[q], 0u, uint32_t(v), uint32_t(v >> 32));
            } else if constexpr (PK) {
                reinterpret_cast<uint2*>(t.bin_val)[dst] = make_uint2(s_l[q], uint32_t(s_v[q]));
            } else {
                t.bin_lidx[dst] = s_l[q];
                bin_val[dst] = V(s_v[q]);
            }
        }
        __syncthreads();
        for (uint32_t x = threadIdx.x; x < T; x += kWT) cursor[x] += hist[x];
    }
}

// the olds of staging positions [p_lo, p_hi) of one round (tile runs at cursor[x], length hist[x],
// staging base base[x]) into LDS at p - p_lo: position p lies in the last run starting at or before
// it; U loads in flight
template <bool OK, typename V, typename S>
__device__ __forceinline__ void wruns_to_lds(const uint32_t* cursor, const uint32_t* base, uint32_t T,
                                             uint32_t p_lo, uint32_t p_hi, const V* __restrict__ src,
                                             const uint8_t* __restrict__ oks, S* s_v, uint8_t* s_ok) {
    constexpr int U = LMR_WIDE_GATHER_U;
    for (uint32_t p0 = p_lo + threadIdx.x; p0 < p_hi; p0 += U * kWT) {
        uint32_t sp[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t p = min(p0 + uint32_t(u) * kWT, p_hi - 1);
            uint32_t lo_x = 0, hi_x = T;
            while (hi_x - lo_x > 1) {
                const uint32_t m = (lo_x + hi_x) >> 1;
                if (base[m] <= p) lo_x = m; else hi_x = m;
            }
            // (an empty run starts where the next one does, so the last run starting at or
            // before p is never an empty one)
            sp[u] = cursor[lo_x] + (p - base[lo_x]);
        }
        V v[U];
        uint8_t o[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            v[u] = src[sp[u]];
            if constexpr (OK) o[u] = oks[sp[u]];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t p = p0 + uint32_t(u) * kWT;
            if (p < p_hi) {
                s_v[p - p_lo] = S(v[u]);
                if constexpr (OK) s_ok[p - p_lo] = o[u];
            }
        }
    }
}

// NH sub-rounds: a round's olds are read into LDS kRound / NH positions at a time, so the block's
// LDS fits two blocks per CU for values of <= 4 bytes (32 waves: twice the loads in flight of one
// 104 KB block); each thread keeps its records' staging positions in registers across them
template <bool OK, int VB>
__global__ __launch_bounds__(1024) void k_unpart_wide(WUnpartTable t) {
    using Gm = WGeom<VB>;
    using S = typename Gm::S;
    using V = typename Gm::V;
    constexpr uint32_t kRound = Gm::kRound;
    constexpr uint32_t NH = VB == 8 ? 1 : 2;
    constexpr uint32_t kSub = kRound / NH;
    constexpr int kRpt = Gm::kRpt;
    __shared__ uint32_t hist[Gm::kMaxT], base[Gm::kMaxT], cursor[Gm::kMaxT], s_tot;
    __shared__ S s_v[kSub];
    __shared__ uint8_t s_ok[OK ? kSub : 1];
    const WUnpartRegion& g = t.r[region_of(t)];
    const uint32_t b = blockIdx.x - g.block0;
    const uint32_t T = t.T;
    for (uint32_t x = threadIdx.x; x < T; x += kWT) cursor[x] = g.gbase + g.cnt[uint64_t(x) * g.G + b];
    const uint64_t lo = uint64_t(b) * g.chunk, hi = min(lo + g.chunk, g.n);
    uint32_t rid = b * g.rpb;
    for (uint64_t r0 = lo; r0 < hi; r0 += kRound, rid++) {
        {   // the round's tile counts (rhist) -> hist, base
            uint32_t hv[Gm::kPer];
            uint32_t sum = 0;
#pragma unroll
            for (uint32_t p = 0; p < Gm::kPer; p++) {
                const uint32_t x = threadIdx.x * Gm::kPer + p;
                hv[p] = x < T ? uint32_t(g.rhist[uint64_t(rid) * T + x]) : 0u;
                sum += hv[p];
            }
            uint32_t e = block_excl_scan(sum, &s_tot);
#pragma unroll
            for (uint32_t p = 0; p < Gm::kPer; p++) {
                const uint32_t x = threadIdx.x * Gm::kPer + p;
                if (x < T) {
                    hist[x] = hv[p];
                    base[x] = e;
                }
                e += hv[p];
            }
        }
        uint16_t qv[kRpt];                                     // this thread's records' positions
#pragma unroll
        for (int j = 0; j < kRpt; j++) {
            const uint64_t k = r0 + threadIdx.x + uint64_t(j) * kWT;
            qv[j] = k < hi ? g.qpos[k] : uint16_t(0xFFFFu);
        }
        __syncthreads();
        const uint32_t tot = s_tot;
#pragma unroll
        for (uint32_t h = 0; h < NH; h++) {
            const uint32_t p_lo = h * kSub, p_hi = min(tot, p_lo + kSub);
            if (h) __syncthreads();                            // the previous sub-round's reads done
            if (p_lo < p_hi)
                wruns_to_lds<OK>(cursor, base, T, p_lo, p_hi, reinterpret_cast<const V*>(t.src), t.oks, s_v, s_ok);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kRpt; j++) {
                const uint32_t q = qv[j];
                if (q == 0xFFFFu || q < p_lo || q >= p_lo + kSub) continue;
                const uint64_t k = r0 + threadIdx.x + uint64_t(j) * kWT;
                reinterpret_cast<V*>(g.dst)[k] = V(s_v[q - p_lo]);
                if constexpr (OK) if (g.okd) g.okd[k] = s_ok[q - p_lo];
            }
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
template <typename F>
hipError_t wdispatch_vb(int vb, F&& f) {
    switch (vb) {
    case 1: return f(std::integral_constant<int, 1>{});
    case 2: return f(std::integral_constant<int, 2>{});
    case 4: return f(std::integral_constant<int, 4>{});
    case 8: return f(std::integral_constant<int, 8>{});
    default: return hipErrorInvalidValue;
    }
}

// LMR_WIDE=0: no wide sessions; LMR_WIDE4=0: none below 8-byte elements. Read per session, so a
// process (a test) can switch them.
// packed records: 1/2/4-byte values by default (LMR_WIDE_PACK=0: split offset / value arrays), 8-byte
// values on request (LMR_WIDE_PACK=8 or =1: 16-B records {index, 0, value} in the temp array)
bool wide_pack_env(int vb) {
    const char* e = getenv("LMR_WIDE_PACK");
    if (vb == 8) return e && *e && (atoi(e) == 8 || atoi(e) == 1) && e[0] != '4';
    return !(e && *e && atoi(e) == 0);
}
// LMR_WIDE4=0 / 1: no / wide sessions below 8-byte elements (default kWide4Default)
constexpr bool kWide4Default = false;   // C5 same box, alternating: 2.06 ms wide vs 1.96 two-level (r6b)
bool wide_env(int vb) {
    const char* e = getenv("LMR_WIDE");
    if (e && *e && atoi(e) == 0) return false;
    if (vb < 8) {
        const char* e4 = getenv("LMR_WIDE4");
        return e4 && *e4 ? atoi(e4) != 0 : kWide4Default;
    }
    return true;
}

uint32_t wide_round(int vb) { return vb == 8 ? WGeom<8>::kRound : WGeom<4>::kRound; }
uint32_t wide_max_tiles(int vb) { return vb == 8 ? kWideMaxTiles : kWideMaxTiles4; }

// producer blocks of a region: one per LMR_WIDE_CHUNK records (default 64K), at most kWideBlocks
constexpr uint32_t kWideBlocks = LMR_WIDE_BLOCKS;
uint32_t wide_blocks(uint64_t n) {
    static const uint64_t per = [] {
        const char* e = getenv("LMR_WIDE_CHUNK");
        const long v = e && *e ? atol(e) : 65536;
        return uint64_t(std::max<long>(4096, v));
    }();
    return uint32_t(std::max<uint64_t>(1, std::min<uint64_t>((n + per - 1) / per, kWideBlocks)));
}

}  // namespace

// the wide session's binned records: bin_val (split arrays, or packed 8-B records), or the temp
// array for packed 16-B records of 8-byte values (cap x 16 B; the results then go to bin_val)
uint8_t* wide_records(const TiledWs& w, const StageSession& s) {
    return s.wpack && dtype_bytes(s.dtype) == 8 ? w.tmp_val : w.bin_val;
}

bool wide_applies(int dtype, uint64_t shard_len, uint64_t cap) {
    const int vb = dtype_bytes(dtype);
    if (vb == 0 || !wide_env(vb)) return false;
    const int shift = wide_shift(vb);
    const uint64_t tiles = (shard_len + (uint64_t(1) << shift) - 1) >> shift;
    // the per-round tile counts live in the position map rpos (4 B per slot, unused by this path).
    // A region of n records has G <= ceil(n / 4K) blocks of whole rounds: <= n / R + n / 4K + 1
    // rounds of R records, so a session's counts fit when (cap / R + cap / 4K + kMaxRegions)
    // rounds of `tiles` u16 do
    const uint64_t rh_entries = (cap / wide_round(vb) + cap / 4096 + kMaxRegions) * tiles;
    return tiles >= 1 && tiles <= wide_max_tiles(vb) && rh_entries <= cap * 2;
}

hipError_t wide_partition(const TiledWs& w, StageSession& s, hipStream_t st) {
    const int vb = dtype_bytes(s.dtype);
    if (s.parted == 0) s.wpack = wide_pack_env(vb);              // one record layout per session
    const int shift = wide_shift(vb);
    const uint32_t R = wide_round(vb);
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
            const uint64_t chunk = ((a.n + G - 1) / G + R - 1) / R * R;
            const uint32_t rpb = uint32_t(chunk / R);
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
        sc.bin_val = wide_records(w, s);
        ws.gbase = gbase;
        ws.total = w.total;
        hipError_t e;
        {
            ProfScope ps(a0.prof, LMR_STAGE_BIN_COUNT, st, n_all);
            e = wdispatch_iw(iw, [&](auto iwt) {
                constexpr int IW = decltype(iwt)::value;
                if (vb == 8)
                    hipLaunchKernelGGL((k_wcount_stage<IW, int(kWideMaxTiles)>), dim3(blocks), dim3(kWT), 0, st, ct);
                else
                    hipLaunchKernelGGL((k_wcount_stage<IW, int(kWideMaxTiles4)>), dim3(blocks), dim3(kWT), 0, st, ct);
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
                return wdispatch_vb(vb, [&](auto vbt) {
                    constexpr int IW = decltype(iwt)::value, VB = decltype(vbt)::value;
                    if (s.wpack) {
                        hipLaunchKernelGGL((k_wide_stage<IW, VB, true>), dim3(blocks), dim3(kWT), 0, st, sc);
                        return hipGetLastError();
                    }
                    hipLaunchKernelGGL((k_wide_stage<IW, VB, false>), dim3(blocks), dim3(kWT), 0, st, sc);
                    return hipGetLastError();
                });
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
    t.src = res_bin;
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
    if (ok) t.oks = ok_bin;
    return wdispatch_vb(dtype_bytes(s.dtype), [&](auto vbt) {
        constexpr int VB = decltype(vbt)::value;
        if (ok)
            hipLaunchKernelGGL((k_unpart_wide<true, VB>), dim3(blocks), dim3(kWT), 0, st, t);
        else
            hipLaunchKernelGGL((k_unpart_wide<false, VB>), dim3(blocks), dim3(kWT), 0, st, t);
        return hipGetLastError();
    });
}

}  // namespace lmr
