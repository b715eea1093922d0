// lmr_pack.hip — device pack of a batched op into per-destination op buffers.
//
// Restates the pack loops of the reference (src/array/unsafe/operations.rs:
// multi_val_multi_index :709-778, one_val_multi_indices :518-552): every global
// index is mapped to (destination PE, local offset) with the array's Block /
// Cyclic / sub-array math (src/array/unsafe.rs:1207-1223, 1610-1736), narrowed
// to the array's IndexSize, and appended to that PE's buffer together with its
// input position j (the reference's res_buffs, used to put fetch results back
// in input order, operations/handle.rs:315-317).
//
// The device version is a counting sort by PE: per-block PE counts -> exclusive
// scan over (PE, block) -> scatter. lmr_pack's scatter ranks with wave ballots
// and is stable, so each PE's buffer holds its records in input order (the
// concatenation, in order, of the reference's per-PE op buffers);
// lmr_pack_unordered's stages rounds in LDS and writes long per-PE runs.
// Output is structure-of-arrays (indices, values, positions): coalesced for the
// apply kernels and for RCCL.
#include "lmr_internal.hpp"
#include "lmr_device.hpp"
#include <stdlib.h>
#include <type_traits>

namespace lmr {

struct PackK {
    lmr_layout_t L;
    FastLayout F;
    const uint64_t* gidx;
    const uint8_t* vals;
    uint32_t vb;
    uint64_t n;
    uint32_t iw;
    uint64_t chunk;
    uint32_t G;
    uint32_t npes;
    uint32_t* counts;       // [npes * G], pe-major
    uint8_t* out_idx;
    uint8_t* out_vals;
    uint32_t* out_pos;
    uint32_t* err;
    uint32_t* fill;         // count-free pack: records reserved in each destination's region
    uint32_t cap;           // count-free pack: records per destination region
    // count-free pack with an overflow list (the exchange's fixed-region mode): a record past its
    // destination's region goes to ovf_gidx / ovf_vals[*ovf_count] (global index, value), not lost
    uint64_t* ovf_gidx;
    uint8_t* ovf_vals;
    uint32_t* ovf_count;
    uint64_t ovf_cap;
    // count-free pack into other PEs' memory (the peer transport's push): destination i's region
    // starts at out_idx_tab[i] / out_vals_tab[i] (device arrays of npes pointers, IPC-mapped peer
    // regions), and every wave ends with a system-scope release so the owners see the records
    uint8_t* const* out_idx_tab;
    uint8_t* const* out_vals_tab;
};

// Wave-aggregated LDS counting: one atomic per distinct key in the wave instead
// of one per lane (a batch spreads over few PEs, so per-lane atomics on
// hist[pe] serialise 64/npes-deep). Returns each active lane's rank among the
// records counted so far under its key. Wave-uniform loop: every lane takes part
// in the ballots.
__device__ __forceinline__ uint32_t wave_agg_rank(uint32_t* hist, uint32_t key, bool active) {
    const int lane = threadIdx.x & 63;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint64_t todo = __ballot(active);
    uint32_t rank = 0;
    while (todo) {
        const int leader = __ffsll((unsigned long long)todo) - 1;
        const uint32_t x = __shfl(key, leader, 64);
        const uint64_t m = __ballot(active && key == x);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&hist[x], uint32_t(__popcll(m)));
        base = __shfl(base, leader, 64);
        if (active && key == x) rank = base + uint32_t(__popcll(m & lt));
        todo &= ~m;
    }
    return rank;
}

// count-only form: no rank, no return value needed from the LDS atomic
__device__ __forceinline__ void wave_agg_count(uint32_t* hist, uint32_t key, bool active) {
    const int lane = threadIdx.x & 63;
    uint64_t todo = __ballot(active);
    while (todo) {
        const int leader = __ffsll((unsigned long long)todo) - 1;
        const uint32_t x = __shfl(key, leader, 64);
        const uint64_t m = __ballot(active && key == x);
        if (lane == leader) atomicAdd(&hist[x], uint32_t(__popcll(m)));
        todo &= ~m;
    }
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_pack_count(PackK p) {
    extern __shared__ uint32_t cnt[];
    for (uint32_t i = threadIdx.x; i < p.npes; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    const uint64_t lo = uint64_t(blockIdx.x) * p.chunk;
    const uint64_t hi = min(lo + p.chunk, p.n);
    const int bits = key_bits(p.npes);
    bool oob = false;
#ifndef LMR_PACK_COUNT_U
#define LMR_PACK_COUNT_U 4
#endif
    constexpr int U = LMR_PACK_COUNT_U;
    for (uint64_t b0 = lo; b0 < hi; b0 += U * 1024) {       // block-uniform: ballots need every lane
        const uint64_t k0 = b0 + threadIdx.x;
        uint64_t g[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t k = k0 + uint64_t(j) * 1024;
            g[j] = k < hi ? p.gidx[k] : ~uint64_t(0);
        }
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t k = k0 + uint64_t(j) * 1024;
            uint64_t pe = 0, off;
            const bool in = k < hi;
            const bool ok = in && pe_and_offset_mode<MODE>(p.F, g[j], pe, off);
            oob |= in && !ok;
            wave_match_count(cnt, ok ? uint32_t(pe) : 0u, ok, bits);
        }
    }
    if (oob) raise_err(p.err, LMR_ERRBIT_OOB);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < p.npes; i += blockDim.x)
        p.counts[uint64_t(i) * p.G + blockIdx.x] = cnt[i];
}

__device__ __forceinline__ void store_idx(uint8_t* base, uint32_t iw, uint64_t pos, uint64_t v) {
    switch (iw) {
    case 1: base[pos] = uint8_t(v); break;
    case 2: reinterpret_cast<uint16_t*>(base)[pos] = uint16_t(v); break;
    case 4: reinterpret_cast<uint32_t*>(base)[pos] = uint32_t(v); break;
    default: reinterpret_cast<uint64_t*>(base)[pos] = v; break;
    }
}

__device__ __forceinline__ void copy_val(uint8_t* dst, const uint8_t* src, uint32_t vb, uint64_t dpos,
                                         uint64_t spos) {
    switch (vb) {
    case 1: dst[dpos] = src[spos]; break;
    case 2: reinterpret_cast<uint16_t*>(dst)[dpos] = reinterpret_cast<const uint16_t*>(src)[spos]; break;
    case 4: reinterpret_cast<uint32_t*>(dst)[dpos] = reinterpret_cast<const uint32_t*>(src)[spos]; break;
    default: reinterpret_cast<uint64_t*>(dst)[dpos] = reinterpret_cast<const uint64_t*>(src)[spos]; break;
    }
}

// Stable scatter. The block walks its chunk in rounds of 1024 records (in
// order); inside a round, wave w holds records [64w, 64w+64). Rank of a record
// = records of the same PE in earlier rounds (cursor) + in earlier waves of
// this round (wave_base) + in earlier lanes of this wave (ballot popcount).
template <int MODE>
__global__ __launch_bounds__(1024) void k_pack_scatter(PackK p) {
    extern __shared__ uint32_t sm[];
    uint32_t* cursor = sm;                     // [npes]
    uint32_t* wcnt = sm + p.npes;              // [16][npes]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t i = threadIdx.x; i < p.npes; i += blockDim.x)
        cursor[i] = p.counts[uint64_t(i) * p.G + blockIdx.x];
    const uint64_t lo = uint64_t(blockIdx.x) * p.chunk;
    const uint64_t hi = min(lo + p.chunk, p.n);
    for (uint64_t r0 = lo; r0 < hi; r0 += 1024) {
        for (uint32_t i = threadIdx.x; i < 16 * p.npes; i += blockDim.x) wcnt[i] = 0;
        __syncthreads();
        const uint64_t k = r0 + threadIdx.x;
        uint64_t pe = 0, off = 0;
        bool valid = (k < hi) && pe_and_offset_mode<MODE>(p.F, p.gidx[k], pe, off);
        const uint32_t mype = valid ? uint32_t(pe) : 0xFFFFFFFFu;
        // group lanes by PE (match-any by repeated ballot over distinct values)
        uint64_t remaining = __ballot(true);
        uint64_t mine = 0;
        while (remaining) {
            int leader = __ffsll((unsigned long long)remaining) - 1;
            uint32_t x = __shfl(mype, leader, 64);
            uint64_t m = __ballot(mype == x);
            if (mype == x) mine = m;
            remaining &= ~m;
        }
        const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
        const uint32_t rank = __popcll(mine & lt);
        const bool first = (mine & lt) == 0;
        if (valid && first) wcnt[w * p.npes + mype] = __popcll(mine);
        __syncthreads();
        // per PE: exclusive scan over the 16 waves, advance the cursor
        for (uint32_t i = threadIdx.x; i < p.npes; i += blockDim.x) {
            uint32_t run = cursor[i];
            for (int ww = 0; ww < 16; ww++) {
                uint32_t c = wcnt[ww * p.npes + i];
                wcnt[ww * p.npes + i] = run;
                run += c;
            }
            cursor[i] = run;
        }
        __syncthreads();
        if (valid) {
            uint64_t pos = uint64_t(wcnt[w * p.npes + mype]) + rank;
            store_idx(p.out_idx, p.iw, pos, off);
            if (p.vals) copy_val(p.out_vals, p.vals, p.vb, pos, k);
            if (p.out_pos) p.out_pos[pos] = uint32_t(k);
        }
        __syncthreads();
    }
}

// LDS-staged scatter for npes <= kStageMaxPes (the common case): rounds of
// RPT * 1024 records are ranked per PE with LDS atomics, staged in LDS in PE
// order and written out as long per-PE runs (~round/npes records), like the
// apply's coarse pass. Not stable within a PE: no caller depends on the order of
// records inside one destination's buffer (the apply is a parallel, per-element
// atomic application, as the reference's concurrent AMs are).
constexpr uint32_t kStageMaxPes = 512;

// exclusive scan of hist[0..m) (m <= kStageMaxPes <= blockDim.x) into base[], total
// into base[kStageMaxPes]; every thread of the block takes part
__device__ __forceinline__ void stage_scan(const uint32_t* hist, uint32_t* base, uint32_t m) {
    __shared__ uint32_t wsum[16];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t x = t < m ? hist[t] : 0u;
    uint32_t inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (int(lane) >= d) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    if (w == 0) {
        const uint32_t nw = blockDim.x >> 6;
        const uint32_t v = lane < nw ? wsum[lane] : 0u;
        uint32_t vi = v;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const uint32_t y = __shfl_up(vi, d, 64);
            if (int(lane) >= d) vi += y;
        }
        if (lane < nw) wsum[lane] = vi - v;
        if (lane == nw - 1) base[kStageMaxPes] = vi;
    }
    __syncthreads();
    if (t < m) base[t] = inc - x + wsum[w];
}

// FREE: no count pass. Destination i owns the region [i * cap, (i + 1) * cap) of the output;
// each round reserves its run per destination with one atomicAdd on fill[i]. A round that
// would overflow a region writes nothing (fill[i] still counts every record, so the caller
// sees a count above cap and packs the chunk again with the counted pack).
template <int IW, int VB, int RPT, int MODE, bool FREE, bool PAIRS = false>
__global__ __launch_bounds__(1024) void k_pack_stage(PackK p) {
    using I = typename idx_t<IW>::I;
    using V = typename idx_t<VB>::I;
    constexpr uint32_t kRound = RPT * 1024;
    __shared__ uint32_t hist[kStageMaxPes], base[kStageMaxPes + 1], cursor[kStageMaxPes];
    __shared__ I s_off[kRound];
    __shared__ V s_val[kRound];
    __shared__ uint32_t s_pos[FREE ? 1 : kRound];   // FREE packs return nothing: no positions, and
                                                    // the smaller LDS footprint fits 2 blocks per CU
    const uint32_t np = p.npes;
    const int bits = key_bits(np);
    __shared__ uint32_t s_over;
    __shared__ uint32_t s_room[FREE ? kStageMaxPes : 1], s_obase[FREE ? kStageMaxPes : 1];
    const bool ovf = FREE && p.ovf_count != nullptr;
    if constexpr (!FREE)
        for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) cursor[i] = p.counts[uint64_t(i) * p.G + blockIdx.x];
    const uint64_t lo = uint64_t(blockIdx.x) * p.chunk;
    const uint64_t hi = min(lo + p.chunk, p.n);
    const V* vals = reinterpret_cast<const V*>(p.vals);
    uint64_t m_g[RPT];
    V m_v[RPT];
    bool m_in[RPT];
    auto load_round = [&](uint64_t r0) {
        if constexpr (PAIRS) {
            // two consecutive records per thread: one 16-B load of their global indices and one
            // of their values (the round's order inside a destination is free: nothing returned)
#pragma unroll
            for (int j = 0; j < RPT; j += 2) {
                const uint64_t k = r0 + uint64_t(j) * 1024 + 2 * uint64_t(threadIdx.x);
                if (k + 1 < hi) {
                    const uint4 gq = *reinterpret_cast<const uint4*>(p.gidx + k);
                    const uint4 vq = *reinterpret_cast<const uint4*>(vals + k);
                    m_g[j] = uint64_t(gq.x) | (uint64_t(gq.y) << 32);
                    m_g[j + 1] = uint64_t(gq.z) | (uint64_t(gq.w) << 32);
                    m_v[j] = V(uint64_t(vq.x) | (uint64_t(vq.y) << 32));
                    m_v[j + 1] = V(uint64_t(vq.z) | (uint64_t(vq.w) << 32));
                    m_in[j] = m_in[j + 1] = true;
                } else {
                    m_in[j] = k < hi;
                    m_in[j + 1] = false;
                    m_g[j] = m_in[j] ? p.gidx[k] : ~uint64_t(0);
                    m_v[j] = m_in[j] ? vals[k] : V(0);
                    m_g[j + 1] = ~uint64_t(0);
                    m_v[j + 1] = V(0);
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < RPT; j++) {
                const uint64_t k = r0 + uint64_t(j) * 1024 + threadIdx.x;
                m_in[j] = k < hi;
                m_g[j] = m_in[j] ? p.gidx[k] : ~uint64_t(0);
                m_v[j] = (m_in[j] && vals) ? vals[k] : V(0);
            }
        }
    };
    load_round(lo);
    for (uint64_t r0 = lo; r0 < hi; r0 += kRound) {
        for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) hist[i] = 0;
        if (FREE && threadIdx.x == 0) s_over = 0;
        __syncthreads();
        uint32_t m_rank[RPT], m_pe[RPT];
        uint64_t m_off[RPT];
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            uint64_t pe = 0, off = 0;
            const bool ok = m_in[j] && pe_and_offset_mode<MODE>(p.F, m_g[j], pe, off);
            m_pe[j] = ok ? uint32_t(pe) : 0xFFFFFFFFu;
            m_off[j] = off;
            m_rank[j] = wave_match_rank(hist, ok ? uint32_t(pe) : 0u, ok, bits);
        }
        __syncthreads();
        stage_scan(hist, base, np);
        if constexpr (FREE) {
            for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) {
                const uint32_t h = hist[i];
                const uint32_t r = h ? atomicAdd(&p.fill[i], h) : 0u;
                if (uint64_t(r) + h > p.cap) s_over = 1;
                cursor[i] = i * p.cap + r;
                if (ovf) {                                 // the part past the region: the overflow list
                    const uint32_t room = r >= p.cap ? 0u : min(h, p.cap - r);
                    s_room[i] = room;
                    s_obase[i] = h > room ? atomicAdd(p.ovf_count, h - room) : 0u;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            if (m_pe[j] == 0xFFFFFFFFu) continue;
            const uint32_t q = base[m_pe[j]] + m_rank[j];
            if (ovf && s_over && m_rank[j] >= s_room[m_pe[j]]) {
                const uint64_t o = uint64_t(s_obase[m_pe[j]]) + (m_rank[j] - s_room[m_pe[j]]);
                if (o < p.ovf_cap) {
                    p.ovf_gidx[o] = m_g[j];
                    if (vals) reinterpret_cast<V*>(p.ovf_vals)[o] = m_v[j];
                }
                continue;
            }
            s_off[q] = I(m_off[j]);
            s_val[q] = m_v[j];
            if (!FREE && p.out_pos) s_pos[q] = uint32_t(r0 + uint64_t(j) * 1024 + threadIdx.x);
        }
        if (r0 + kRound < hi) load_round(r0 + kRound);
        __syncthreads();
        auto put = [&](uint32_t q, uint32_t dst) {
            reinterpret_cast<I*>(p.out_idx)[dst] = s_off[q];
            if (vals) reinterpret_cast<V*>(p.out_vals)[dst] = s_val[q];
            if (!FREE && p.out_pos) p.out_pos[dst] = s_pos[q];
        };
        if (FREE && p.out_idx_tab) {                       // per-destination regions elsewhere
            const uint32_t nw = blockDim.x >> 6, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
            const uint32_t wpb = np >= nw ? 1u : nw / np, bstep = nw / wpb;
            for (uint32_t c = wave / wpb; c < np; c += bstep) {
                const uint32_t len = ovf ? s_room[c] : (s_over ? 0u : hist[c]), b = base[c];
                const uint32_t d = cursor[c] - c * p.cap;   // offset in destination c's region
                I* oi = reinterpret_cast<I*>(p.out_idx_tab[c]);
                V* ov = vals ? reinterpret_cast<V*>(p.out_vals_tab[c]) : nullptr;
                for (uint32_t i = (wave % wpb) * 64 + lane; i < len; i += wpb * 64) {
                    as_global(oi)[d + i] = s_off[b + i];
                    if (ov) as_global(ov)[d + i] = s_val[b + i];
                }
            }
        } else if (!FREE || !s_over) {
            bucket_writeout(hist, base, cursor, np, put);
        } else if (ovf) {                                  // each destination's run up to its room
            const uint32_t nw = blockDim.x >> 6, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
            const uint32_t wpb = np >= nw ? 1u : nw / np, bstep = nw / wpb;
            for (uint32_t c = wave / wpb; c < np; c += bstep) {
                const uint32_t len = s_room[c], b = base[c], d = cursor[c];
                for (uint32_t i = (wave % wpb) * 64 + lane; i < len; i += wpb * 64) put(b + i, d + i);
            }
        }
        __syncthreads();
        if constexpr (!FREE)
            for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) cursor[i] += hist[i];
    }
    if (FREE && p.out_idx_tab) {                          // the owners read the regions next:
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's stores done,
        __syncthreads();                                  // then one system-scope release per block
        if (threadIdx.x == 0) __threadfence_system();
    }
}

__global__ void k_fill_counts(uint32_t* fill, uint32_t npes, uint64_t* dest_counts, int clear) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < npes) {
        dest_counts[i] = fill[i];
        if (clear) fill[i] = 0;             // zero again for the next pack (PackArgs::fill_zeroed)
    }
}

__global__ void k_dest_offsets(const uint32_t* counts, uint32_t npes, uint32_t G, const uint32_t* total,
                               uint64_t* dest_offsets, uint64_t* dest_counts) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= npes) {
        uint64_t o = (i < npes) ? counts[uint64_t(i) * G] : *total;
        dest_offsets[i] = o;
    }
    if (i < npes && dest_counts) {
        uint64_t nx = (i + 1 < npes) ? counts[uint64_t(i + 1) * G] : *total;
        dest_counts[i] = nx - counts[uint64_t(i) * G];
    }
}

template <typename F>
static void dispatch_pack_stage(int iw, int vb, F&& f) {
    using std::integral_constant;
    auto with_iw = [&](auto iwt) {
        switch (vb) {
        case 1: f(iwt, integral_constant<int, 1>{}); break;
        case 2: f(iwt, integral_constant<int, 2>{}); break;
        case 4: f(iwt, integral_constant<int, 4>{}); break;
        default: f(iwt, integral_constant<int, 8>{}); break;
        }
    };
    switch (iw) {
    case 1: with_iw(integral_constant<int, 1>{}); break;
    case 2: with_iw(integral_constant<int, 2>{}); break;
    case 4: with_iw(integral_constant<int, 4>{}); break;
    default: with_iw(integral_constant<int, 8>{}); break;
    }
}

hipError_t launch_pack(const PackArgs& a, uint32_t* counts, uint32_t* partials, uint32_t* total,
                       hipStream_t s) {
    const uint32_t npes = a.layout.num_pes;
    if (npes == 0 || npes > uint32_t(kMaxPackPes)) return hipErrorInvalidValue;
    uint64_t G = (a.n + 65535) / 65536;
    if (G > uint64_t(kMaxBinBlocks)) G = kMaxBinBlocks;
    if (G < 1) G = 1;
    PackK p;
    p.L = a.layout; p.F = make_fast_layout(a.layout); p.gidx = a.gidx; p.vals = a.vals; p.vb = a.val_bytes; p.n = a.n;
    p.iw = a.index_size; p.chunk = (a.n + G - 1) / G; if (p.chunk == 0) p.chunk = 1;
    p.G = uint32_t(G); p.npes = npes; p.counts = counts;
    p.out_idx = a.out_idx; p.out_vals = a.out_vals; p.out_pos = a.out_pos; p.err = a.err;
    p.fill = nullptr; p.cap = 0;
    p.ovf_gidx = nullptr; p.ovf_vals = nullptr; p.ovf_count = nullptr; p.ovf_cap = 0;
    p.out_idx_tab = nullptr; p.out_vals_tab = nullptr;
    ProfScope ps(a.prof, LMR_STAGE_PACK, s, a.n);
    const int mode = layout_map_mode(a.layout);
    auto by_mode = [&](auto f) {
        using std::integral_constant;
        if (mode == LMR_MAP_BLOCK) f(integral_constant<int, LMR_MAP_BLOCK>{});
        else if (mode == LMR_MAP_CYCLIC) f(integral_constant<int, LMR_MAP_CYCLIC>{});
        else f(integral_constant<int, LMR_MAP_GENERIC>{});
    };
    if (a.n > 0) {
        by_mode([&](auto m) {
            hipLaunchKernelGGL((k_pack_count<decltype(m)::value>), dim3(unsigned(G)), dim3(1024), size_t(npes) * 4,
                               s, p);
        });
    } else {
        hipError_t e0 = hipMemsetAsync(counts, 0, size_t(npes) * G * 4, s);
        if (e0 != hipSuccess) return e0;
    }
    hipError_t e = scan_exclusive_u32(counts, uint64_t(npes) * G, partials, total, s);
    if (e != hipSuccess) return e;
    if (a.n > 0) {
        if (!a.stable && npes <= kStageMaxPes) {
            const int vbk = a.vals ? int(a.val_bytes) : 1;
            dispatch_pack_stage(int(a.index_size), vbk, [&](auto iw, auto vb) {
                by_mode([&](auto m) {
                    constexpr int IWc = decltype(iw)::value, VBc = decltype(vb)::value;
                    constexpr int RP = (IWc + VBc + 4) * 8 <= 150 ? 8 : 4;      // rounds of RP * 1024 records in LDS
                    hipLaunchKernelGGL((k_pack_stage<IWc, VBc, RP, decltype(m)::value, false>),
                                       dim3(unsigned(G)), dim3(1024), 0, s, p);
                });
            });
        } else {
            by_mode([&](auto m) {
                hipLaunchKernelGGL((k_pack_scatter<decltype(m)::value>), dim3(unsigned(G)), dim3(1024),
                                   size_t(npes) * 17 * 4, s, p);
            });
        }
    }
    hipLaunchKernelGGL(k_dest_offsets, dim3((npes + 1 + 255) / 256), dim3(256),
                       0, s, counts, npes, uint32_t(G), total, a.dest_offsets, a.dest_counts);
    return hipGetLastError();
}

#ifndef LMR_PACK_FREE_LDS
#define LMR_PACK_FREE_LDS 100  // KB of LDS per round buffer: 8K-record rounds of 12-B records, one block per CU
                               // (72: 4K rounds, 2 blocks per CU; alone 0.511 -> 0.460 ms per 2^26 records at 8
                               // PEs, the one-rank rehearsal unchanged, profiles/r5/pack/ab_round.log)
#endif

// Count-free unordered pack (nothing returned): destination i's records land in
// [i * cap, i * cap + dest_counts[i]) of out_idx / out_vals. dest_counts[i] > cap means
// the region overflowed and the output is incomplete (pack again with launch_pack).
hipError_t launch_pack_free(const PackArgs& a, uint32_t* fill, uint32_t cap, hipStream_t s) {
    const uint32_t npes = a.layout.num_pes;
    if (npes == 0 || npes > kStageMaxPes || a.out_pos || a.stable) return hipErrorInvalidValue;
    uint64_t G = (a.n + 65535) / 65536;
    if (G > uint64_t(kMaxBinBlocks)) G = kMaxBinBlocks;
    if (G < 1) G = 1;
    PackK p;
    p.L = a.layout; p.F = make_fast_layout(a.layout); p.gidx = a.gidx; p.vals = a.vals; p.vb = a.val_bytes; p.n = a.n;
    p.iw = a.index_size; p.chunk = (a.n + G - 1) / G; if (p.chunk == 0) p.chunk = 1;
    p.G = uint32_t(G); p.npes = npes; p.counts = nullptr;
    p.out_idx = a.out_idx; p.out_vals = a.out_vals; p.out_pos = nullptr; p.err = a.err;
    p.fill = fill; p.cap = cap;
    p.ovf_gidx = a.ovf_gidx; p.ovf_vals = a.ovf_vals; p.ovf_count = a.ovf_count; p.ovf_cap = a.ovf_cap;
    p.out_idx_tab = a.out_idx_tab; p.out_vals_tab = a.out_vals_tab;
    // paired 16-B loads: 8-byte values, 16-B aligned index and value arrays, even block ranges
    // (LMR_PACK_PAIRS=0: one record per load)
    static const bool pairs_on = [] { const char* v = getenv("LMR_PACK_PAIRS"); return !(v && v[0] == '0'); }();
    if (pairs_on && (p.chunk & 1)) p.chunk += 1;
    const bool pairs = pairs_on && a.vals && a.val_bytes == 8 &&
                       ((reinterpret_cast<uintptr_t>(a.gidx) | reinterpret_cast<uintptr_t>(a.vals)) & 15) == 0;
    ProfScope ps(a.prof, LMR_STAGE_PACK, s, a.n);
    if (!a.fill_zeroed) {
        const hipError_t e = hipMemsetAsync(fill, 0, size_t(npes) * 4, s);
        if (e != hipSuccess) return e;
    }
    if (a.n > 0) {
        const int mode = layout_map_mode(a.layout);
        const int vbk = a.vals ? int(a.val_bytes) : 1;
        dispatch_pack_stage(int(a.index_size), vbk, [&](auto iw, auto vb) {
            constexpr int IWc = decltype(iw)::value, VBc = decltype(vb)::value;
            constexpr int RP = (IWc + VBc) * 8 <= LMR_PACK_FREE_LDS ? 8 : 4;   // rounds of RP * 1024 records
            constexpr bool kP = VBc == 8;
            if (kP && pairs && mode == LMR_MAP_BLOCK)
                hipLaunchKernelGGL((k_pack_stage<IWc, VBc, RP, LMR_MAP_BLOCK, true, kP>), dim3(unsigned(G)), dim3(1024), 0, s, p);
            else if (kP && pairs && mode == LMR_MAP_CYCLIC)
                hipLaunchKernelGGL((k_pack_stage<IWc, VBc, RP, LMR_MAP_CYCLIC, true, kP>), dim3(unsigned(G)), dim3(1024), 0, s, p);
            else if (mode == LMR_MAP_BLOCK)
                hipLaunchKernelGGL((k_pack_stage<IWc, VBc, RP, LMR_MAP_BLOCK, true>), dim3(unsigned(G)), dim3(1024), 0, s, p);
            else if (mode == LMR_MAP_CYCLIC)
                hipLaunchKernelGGL((k_pack_stage<IWc, VBc, RP, LMR_MAP_CYCLIC, true>), dim3(unsigned(G)), dim3(1024), 0, s, p);
            else
                hipLaunchKernelGGL((k_pack_stage<IWc, VBc, RP, LMR_MAP_GENERIC, true>), dim3(unsigned(G)), dim3(1024), 0, s,
                                   p);
        });
    }
    hipLaunchKernelGGL(k_fill_counts, dim3((npes + 255) / 256), dim3(256), 0, s, fill, npes, a.dest_counts,
                       a.fill_zeroed ? 1 : 0);
    return hipGetLastError();
}

// ------------------------------------------------------------------ results
template <typename V>
__global__ void k_scatter_results(const V* __restrict__ in, const uint32_t* __restrict__ pos, uint64_t n,
                                  V* __restrict__ out, const uint8_t* ok_in, uint8_t* ok_out) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < n; k += stride) {
        uint32_t p = pos[k];
        out[p] = in[k];
        if (ok_in) ok_out[p] = ok_in[k];
    }
}

hipError_t launch_scatter_results(const uint8_t* in, const uint32_t* pos, uint64_t n,
                                  uint32_t elem_bytes, uint8_t* out, const uint8_t* ok_in,
                                  uint8_t* ok_out, Prof* prof, hipStream_t s) {
    if (n == 0) return hipSuccess;
    ProfScope ps(prof, LMR_STAGE_SCATTER_RESULTS, s, n);
    uint64_t g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    switch (elem_bytes) {
    case 1: hipLaunchKernelGGL((k_scatter_results<uint8_t>), dim3(unsigned(g)), dim3(256), 0, s,
                               in, pos, n, out, ok_in, ok_out); break;
    case 2: hipLaunchKernelGGL((k_scatter_results<uint16_t>), dim3(unsigned(g)), dim3(256), 0, s,
                               reinterpret_cast<const uint16_t*>(in), pos, n,
                               reinterpret_cast<uint16_t*>(out), ok_in, ok_out); break;
    case 4: hipLaunchKernelGGL((k_scatter_results<uint32_t>), dim3(unsigned(g)), dim3(256), 0, s,
                               reinterpret_cast<const uint32_t*>(in), pos, n,
                               reinterpret_cast<uint32_t*>(out), ok_in, ok_out); break;
    case 8: hipLaunchKernelGGL((k_scatter_results<uint64_t>), dim3(unsigned(g)), dim3(256), 0, s,
                               reinterpret_cast<const uint64_t*>(in), pos, n,
                               reinterpret_cast<uint64_t*>(out), ok_in, ok_out); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace lmr
