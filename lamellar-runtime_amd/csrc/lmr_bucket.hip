// lmr_bucket.hip — the exchange's bucketed regions: the sender's pack
// groups a chunk's records by (owner PE, owner bucket of 256 tiles) into a region per owner laid
// out by bucket -- a header of slice counts, then the slices -- so the owner skips its coarse pass.
// Over the peer transport the pack writes straight into the owners' IPC-mapped receive regions;
// over a collective transport (RCCL, host callbacks) into the send buffer, whose regions the
// all-to-all-v moves whole.
//
// The plain exchange: sender pack by owner (8 keys) -> owner stages every source's region -> owner
// coarse pass (24 B per record) -> fine pass (22 B) -> tile sweep. Here:
//   k_pack_bucket   sender, LDS rounds of 8K records ranked by (owner, bucket) -- up to
//                   kBucketMaxKeys keys: 8 PEs x 32 buckets of 256 tiles at 2^26-element u64 shards --
//                   each round's run of every key reserved with one atomicAdd on the key's fill
//                   counter and written into the owner's region at bucket b's slice
//                   [b * cap_b, (b + 1) * cap_b); records past a slice go to the overflow list (the
//                   exchange's overflow round)
//   k_bucket_hdr    sender, per owner: the slices' record counts into the region's header (the
//                   first kBucketHdr bytes of the index area), the fill counters cleared, one
//                   system-scope release (a peer owner reads the header after the chunk's publish)
//   k_fine_bucket   owner, per chunk: every source's slices of a bucket are one virtual record
//                   stream (record-balanced block ranges, as the count-free fine pass reads its
//                   bucket segments), ranked by tile in LDS and appended to fixed tile regions of
//                   the session (tile t at [t * cap_t, (t + 1) * cap_t) of the workspace's temp
//                   arrays, one atomicAdd per tile and round on its fill counter); a record past
//                   its tile region is applied to the shard at once with a device atomic (the op is
//                   order-insensitive: any split is exact)
//   k_bucket_plan   owner, at the session's sweep: one tile item per tile from the fills (and the
//                   fills cleared), then k_tile_owner over the items
//   k_bucket_direct an owner without a session workspace: the slices applied with device atomics
// Only ops whose records commute take it (add / sub / mul / and / or / xor on integers, nothing
// returned). The session stays open across deferred batches like the staged one
// (lmr_exchange_flush sweeps it).
#include "lmr_tile.hpp"
#include "lmr_device.hpp"
#include <algorithm>

namespace lmr {

namespace {

constexpr uint32_t kBT = 1024;
constexpr uint32_t kBTilesPerBucket = 512;            // tiles per bucket at most (LMR_BUCKET_TPB)

// ---------------------------------------------------------------- sender
struct BPackK {
    FastLayout F;
    const uint64_t* gidx;
    const uint8_t* vals;         // null: scalar value val_bits
    uint64_t val_bits;
    uint64_t n, chunk;
    uint32_t npes, C, cap_b;
    int cshift;                  // bucket of a local offset = off >> cshift
    uint8_t* const* idx_tab;     // device: owner q's index area (header + C x cap_b u32 offsets in bucket)
    uint8_t* const* val_tab;     // device: owner q's value area (C x cap_b values)
    // idx_tab null: owner q's areas at idx_base + q * idx_stride / val_base + q * val_stride (a send
    // buffer of the collective exchange; val_base null: scalar value)
    uint8_t* idx_base;
    uint8_t* val_base;
    uint64_t idx_stride, val_stride;
    uint32_t* fill;              // [npes * C] records reserved in each slice this chunk
    uint64_t* ovf_gidx;
    uint8_t* ovf_vals;
    uint32_t* ovf_count;
    uint64_t ovf_cap;
    uint32_t* err;
};

// RPT records per thread and round: 8 (8K-record rounds, 132 KB of LDS, one block per CU) or 4
// (4K, 76 KB, two blocks per CU: one block's round-trip latencies overlap the other's)
// PAIRS: two consecutive records per 16-B load of indices and of values (8-byte values, both arrays
// 16-B aligned, even block ranges); record j of a round is then 2 * ((j / 2) * 1024 + thread) + j % 2
template <int VB, int MODE, int RPT, bool PAIRS>
__global__ __launch_bounds__(1024) void k_pack_bucket(BPackK p) {
    using V = typename idx_t<VB>::I;
    constexpr uint32_t kPRound = RPT * kBT;
    __shared__ uint32_t hist[kBucketMaxKeys], base[kBucketMaxKeys], cur[kBucketMaxKeys], room[kBucketMaxKeys],
        obase[kBucketMaxKeys], s_tot;
    __shared__ uint16_t s_k[kPRound];
    __shared__ uint32_t s_i[kPRound];
    __shared__ V s_v[kPRound];
    __shared__ uint8_t s_dq[kBucketMaxKeys];
    __shared__ uint8_t* s_itab[kBucketMaxSrc];
    __shared__ uint8_t* s_vtab[kBucketMaxSrc];
    const uint32_t nkeys = p.npes * p.C;
    // the owners' region pointers in LDS (a per-record load from the device table would put a
    // dependent global load in front of every store of the write-out)
    if (threadIdx.x < p.npes) {
        const uint64_t q = threadIdx.x;
        s_itab[q] = (p.idx_tab ? p.idx_tab[q] : p.idx_base + q * p.idx_stride) + kBucketHdr;
        s_vtab[q] = p.idx_tab ? (p.val_tab ? p.val_tab[q] : nullptr) : (p.val_base ? p.val_base + q * p.val_stride : nullptr);
    }
    const bool has_vals = p.idx_tab ? p.val_tab != nullptr : p.val_base != nullptr;
    const uint64_t lo = uint64_t(blockIdx.x) * p.chunk, hi = min(lo + p.chunk, p.n);
    const uint64_t bmask = (uint64_t(1) << p.cshift) - 1;
    const V* vals = reinterpret_cast<const V*>(p.vals);
    bool oob = false;
    uint64_t g[RPT];
    V v[RPT];
    auto kof = [&](uint64_t r0, int j) -> uint64_t {
        return PAIRS ? r0 + 2 * (uint64_t(j >> 1) * kBT + threadIdx.x) + (j & 1) : r0 + uint64_t(j) * kBT + threadIdx.x;
    };
    // (pairs: every pair is loaded from an even offset <= kl, the block range's last pair, and the
    // records past hi are masked by the round)
    const uint64_t kl = lo < hi ? lo + ((hi - 1 - lo) & ~uint64_t(1)) : lo;
    auto load_round = [&](uint64_t r0) {
        if constexpr (PAIRS) {
#pragma unroll
            for (int j = 0; j < RPT; j += 2) {
                const uint64_t k = kof(r0, j);
                const uint64_t kc = k <= kl ? k : kl;
                const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(p.gidx + kc);
                const ulonglong2 y = *reinterpret_cast<const ulonglong2*>(vals + kc);
                g[j] = k < hi ? x.x : ~uint64_t(0);
                g[j + 1] = k + 1 < hi ? x.y : ~uint64_t(0);
                v[j] = V(y.x);
                v[j + 1] = V(y.y);
            }
        } else {
#pragma unroll
            for (int j = 0; j < RPT; j++) {
                const uint64_t k = kof(r0, j);
                g[j] = k < hi ? p.gidx[k] : ~uint64_t(0);
                v[j] = k < hi ? (vals ? vals[k] : V(p.val_bits)) : V(0);
            }
        }
    };
    if (lo < hi) load_round(lo);
    for (uint64_t r0 = lo; r0 < hi; r0 += kPRound) {
        for (uint32_t x = threadIdx.x; x < nkeys; x += kBT) hist[x] = 0;
        __syncthreads();
        uint32_t key[RPT];                          // (key << 16) | rank, all ones: no record
        uint32_t lof[RPT];                          // offset in the bucket
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint64_t k = kof(r0, j);
            uint64_t pe = 0, off = 0;
            const bool ok = k < hi && pe_and_offset_mode<MODE>(p.F, g[j], pe, off);
            oob |= k < hi && !ok;
            const uint32_t kk = ok ? uint32_t(pe) * p.C + uint32_t(off >> p.cshift) : 0u;
            key[j] = ok ? (kk << 16) | atomicAdd(&hist[kk], 1u) : ~0u;
            lof[j] = uint32_t(off & bmask);
        }
        __syncthreads();
        {   // exclusive scan of the keys' counts (one per thread: nkeys <= 1024)
            const uint32_t h = threadIdx.x < nkeys ? hist[threadIdx.x] : 0u;
            const uint32_t e = block_excl_scan(h, &s_tot);
            if (threadIdx.x < nkeys) {
                base[threadIdx.x] = e;
                // this round's run of the key: one reservation; the part past the slice goes to the
                // overflow list
                const uint32_t r = h ? atomicAdd(&p.fill[threadIdx.x], h) : 0u;
                const uint32_t rm = r >= p.cap_b ? 0u : min(h, p.cap_b - r);
                const uint32_t dq = threadIdx.x / p.C;
                cur[threadIdx.x] = (threadIdx.x - dq * p.C) * p.cap_b + r;   // the run's first slot in the region
                s_dq[threadIdx.x] = uint8_t(dq);
                room[threadIdx.x] = rm;
                obase[threadIdx.x] = h > rm ? atomicAdd(p.ovf_count, h - rm) : 0u;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            if (key[j] == ~0u) continue;
            const uint32_t kk = key[j] >> 16, rk = key[j] & 0xFFFFu;
            const uint32_t q = base[kk] + rk;
            s_k[q] = uint16_t(kk);                    // (also for a hole: the write-out skips it by its key)
            if (rk >= room[kk]) {                     // past its slice: the overflow list
                const uint64_t o = uint64_t(obase[kk]) + (rk - room[kk]);
                if (o < p.ovf_cap) {
                    p.ovf_gidx[o] = g[j];
                    if (p.ovf_vals) reinterpret_cast<V*>(p.ovf_vals)[o] = v[j];
                }
                continue;
            }
            s_i[q] = lof[j];
            s_v[q] = v[j];
        }
        if (r0 + kPRound < hi) load_round(r0 + kPRound);   // the next round's loads under the write-out
        __syncthreads();
        const uint32_t tot = s_tot;
        // (a static trip count: the compiler can then wait for the prefetched loads alone, not for
        // the write-out's stores after them, at the next round's first use)
#pragma unroll
        for (int it = 0; it < RPT; it++) {
            const uint32_t q = uint32_t(it) * kBT + threadIdx.x;
            if (q >= tot) continue;
            const uint32_t kk = s_k[q];
            const uint32_t jj = q - base[kk];
            if (jj >= room[kk]) continue;             // (a hole: its record went to the overflow list)
            const uint32_t dq = s_dq[kk];
            const uint32_t slot = cur[kk] + jj;
            as_global(reinterpret_cast<uint32_t*>(s_itab[dq]))[slot] = s_i[q];
            if (has_vals) as_global(reinterpret_cast<V*>(s_vtab[dq]))[slot] = s_v[q];
        }
        __syncthreads();
    }
    if (oob) raise_err(p.err, LMR_ERRBIT_OOB);
    // the owners read the regions after the chunk's publish: every wave's stores done, then one
    // system-scope release per block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __threadfence_system();
}

// one block per owner q: the slices' counts into q's region header, their sum into tot[q] (the
// mailbox count), the fill counters cleared for the next chunk, then a system-scope release
__global__ __launch_bounds__(256) void k_bucket_hdr(uint32_t* fill, uint32_t C, uint32_t cap_b,
                                                    uint8_t* const* idx_tab, uint8_t* idx_base, uint64_t idx_stride,
                                                    uint32_t* tot) {
    const uint32_t q = blockIdx.x;
    __shared__ uint32_t s;
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    uint32_t* hdr = reinterpret_cast<uint32_t*>(idx_tab ? idx_tab[q] : idx_base + uint64_t(q) * idx_stride);
    for (uint32_t b = threadIdx.x; b < C; b += blockDim.x) {
        const uint32_t c = min(fill[q * C + b], cap_b);
        __hip_atomic_store(hdr + b, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        atomicAdd(&s, c);
        fill[q * C + b] = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        tot[q] = s;
        __threadfence_system();
    }
}

// ---------------------------------------------------------------- owner
struct BFineK {
    const uint8_t* idx[kBucketMaxSrc];   // source s's index area (header + slices), this chunk's parity
    const uint8_t* val[kBucketMaxSrc];   // null: the source's scalar sbits[s]
    uint64_t sbits[kBucketMaxSrc];
    uint32_t cap_b[kBucketMaxSrc];       // source s's slice capacity (records)
    uint32_t S, C, T;
    int cshift;                          // bucket b's elements start at b << cshift (k_bucket_direct)
    uint64_t shard_len;
    uint32_t tpb;                        // tiles per bucket (a power of two, <= kBTilesPerBucket)
    int tile_shift;
    uint64_t cap_t;                      // records per fixed tile region
    uint16_t* bin_lidx;                  // [T * cap_t]
    uint8_t* bin_val;
    uint32_t* tfill;                     // [T] the session's tile fills
    void* shard;
    int op;
    uint32_t* err;
};

// RPT records per thread and round: 8 (8K-record rounds, one block per CU) or 4 (4K, ~64 KB of LDS:
// two blocks per CU, or one beside a pack block)
template <int VB, int RPT>
__global__ __launch_bounds__(1024) void k_fine_bucket(BFineK p) {
    using V = typename idx_t<VB>::I;
    constexpr uint32_t kFRound = RPT * kBT;
    constexpr uint32_t kSegMax = kBucketMaxKeys * 2;   // (bucket, source) segments: C x S
    __shared__ uint32_t s_vs[kSegMax + 1];
    __shared__ uint32_t hist[kBTilesPerBucket], base[kBTilesPerBucket], cur[kBTilesPerBucket],
        room[kBTilesPerBucket], s_tot, s_part[16], s_spill;
    __shared__ uint16_t s_l[kFRound];
    __shared__ uint16_t s_f[kFRound];
    __shared__ V s_v[kFRound];
    __shared__ const uint8_t* s_ib[kBucketMaxSrc];
    __shared__ const uint8_t* s_vb[kBucketMaxSrc];
    __shared__ uint64_t s_sb[kBucketMaxSrc];
    __shared__ uint32_t s_cb[kBucketMaxSrc];
    const uint32_t S = p.S, C = p.C, nseg = C * S;
    // the sources' areas in LDS: indexing the kernel-argument arrays by a per-lane source put two
    // dependent global loads (the pointers) in front of every record's loads
    if (threadIdx.x < S) {
        s_ib[threadIdx.x] = p.idx[threadIdx.x] ? p.idx[threadIdx.x] + kBucketHdr : nullptr;
        s_vb[threadIdx.x] = p.val[threadIdx.x];
        s_sb[threadIdx.x] = p.sbits[threadIdx.x];
        s_cb[threadIdx.x] = p.cap_b[threadIdx.x];
    }
    __syncthreads();
    // segment (b, s) = virtual records [s_vs[b * S + s], s_vs[b * S + s + 1])
    for (uint32_t x = threadIdx.x; x < nseg; x += kBT) {
        const uint32_t b = x / S, s = x - b * S;
        s_vs[x] = p.idx[s] ? min(reinterpret_cast<const uint32_t*>(p.idx[s])[b], s_cb[s]) : 0u;
    }
    __syncthreads();
    {   // in-place exclusive scan (one thread per up-to-two entries)
        const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
        const uint32_t a = 2 * t < nseg ? s_vs[2 * t] : 0u, c = 2 * t + 1 < nseg ? s_vs[2 * t + 1] : 0u;
        uint32_t inc = a + c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d, 64);
            if (int(lane) >= d) inc += y;
        }
        if (lane == 63) s_part[w] = inc;
        __syncthreads();
        if (t == 0) {
            uint32_t run = 0;
            for (int i = 0; i < 16; i++) { const uint32_t x = s_part[i]; s_part[i] = run; run += x; }
            s_vs[nseg] = run;
        }
        __syncthreads();
        const uint32_t ex = s_part[w] + inc - (a + c);
        if (2 * t < nseg) s_vs[2 * t] = ex;
        if (2 * t + 1 < nseg) s_vs[2 * t + 1] = ex + a;
        __syncthreads();
    }
    const uint32_t total = s_vs[nseg];
    const uint32_t nb = gridDim.x, lb = xcd_block(true);
    const uint32_t v_lo = uint32_t(uint64_t(total) * lb / nb), v_hi = uint32_t(uint64_t(total) * (lb + 1) / nb);
    const uint32_t lmask = (1u << p.tile_shift) - 1u;
    const uint64_t tile_elems = uint64_t(1) << p.tile_shift;
    auto bstart = [&](uint32_t b) { return s_vs[b * S]; };   // bucket b = virtual [bstart(b), bstart(b + 1))
    uint32_t li[RPT];
    V vv[RPT];
    // round [v0, min(v0 + kFRound, e)) of bucket b's virtual records (its sources' slices in order)
    auto load_round = [&](uint32_t b, uint32_t v0, uint32_t e) {
        uint32_t k = b * S;
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint32_t v = v0 + uint32_t(j) * kBT + threadIdx.x;
            li[j] = 0;
            vv[j] = V(0);
            if (v < e) {
                while (v >= s_vs[k + 1]) k++;
                const uint32_t s = k - b * S;
                const uint64_t slot = uint64_t(b) * s_cb[s] + (v - s_vs[k]);
                li[j] = as_global(reinterpret_cast<const uint32_t*>(s_ib[s]))[slot];
                const V* vb = reinterpret_cast<const V*>(s_vb[s]);
                vv[j] = vb ? as_global(vb)[slot] : V(s_sb[s]);
            }
        }
    };
    // the next bucket at or after bb with records in [v_lo, v_hi)
    auto next_bucket = [&](uint32_t bb) {
        while (bb < C && bstart(bb) < v_hi && max(v_lo, bstart(bb)) >= min(v_hi, bstart(bb + 1))) bb++;
        return bb;
    };
    uint32_t b = 0;
    while (b + 1 < C && bstart(b + 1) <= v_lo) b++;
    b = next_bucket(b);
    if (b < C && bstart(b) < v_hi) load_round(b, max(v_lo, bstart(b)), min(v_hi, bstart(b + 1)));
    bool oob = false;
    V* shard = reinterpret_cast<V*>(p.shard);
    while (b < C && bstart(b) < v_hi) {
        const uint32_t a = max(v_lo, bstart(b)), e = min(v_hi, bstart(b + 1));
        const uint32_t bn = next_bucket(b + 1);
        const bool has_next = bn < C && bstart(bn) < v_hi;
        const uint32_t t0 = b * p.tpb;
        const uint32_t nf = t0 < p.T ? min(p.tpb, p.T - t0) : 0u;
        for (uint32_t v0 = a; v0 < e; v0 += kFRound) {
            for (uint32_t f = threadIdx.x; f < p.tpb; f += kBT) hist[f] = 0;
            if (threadIdx.x == 0) s_spill = 0;
            __syncthreads();
            uint32_t key[RPT];                     // (tile in bucket << 16) | rank, all ones: none
#pragma unroll
            for (int j = 0; j < RPT; j++) {
                const uint32_t v = v0 + uint32_t(j) * kBT + threadIdx.x;
                const uint32_t f = li[j] >> p.tile_shift;
                const bool ok = v < e && f < nf;
                oob |= v < e && !ok;
                key[j] = ok ? (f << 16) | atomicAdd(&hist[f], 1u) : ~0u;
            }
            __syncthreads();
            {
                const uint32_t h = threadIdx.x < p.tpb ? hist[threadIdx.x] : 0u;
                const uint32_t ex = block_excl_scan(h, &s_tot);
                if (threadIdx.x < nf) {
                    base[threadIdx.x] = ex;
                    const uint32_t r = h ? atomicAdd(&p.tfill[t0 + threadIdx.x], h) : 0u;
                    const uint32_t rm = uint64_t(r) >= p.cap_t ? 0u : uint32_t(min<uint64_t>(h, p.cap_t - r));
                    cur[threadIdx.x] = r;
                    room[threadIdx.x] = rm;
                    if (rm < h) s_spill = 1;
                }
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < RPT; j++) {
                if (key[j] == ~0u) continue;
                const uint32_t f = key[j] >> 16;
                const uint32_t q = base[f] + (key[j] & 0xFFFFu);
                s_l[q] = uint16_t(li[j] & lmask);
                s_f[q] = uint16_t(f);
                s_v[q] = vv[j];
            }
            {   // one prefetch site: this bucket's next round, else the next bucket's first
                const bool more = v0 + kFRound < e;
                const uint32_t nbk = more ? b : (has_next ? bn : b);
                load_round(nbk, more ? v0 + kFRound : (has_next ? max(v_lo, bstart(bn)) : e),
                           more ? e : (has_next ? min(v_hi, bstart(bn + 1)) : e));
            }
            __syncthreads();
            const uint32_t tot = s_tot;
            // the write-out holds no device atomic (a returned value would make the compiler wait for
            // the prefetch); the records past their tile's region go in the loop after it
#pragma unroll
            for (int it = 0; it < RPT; it++) {       // (a static trip count, as in the pack)
                const uint32_t q = uint32_t(it) * kBT + threadIdx.x;
                if (q >= tot) continue;
                const uint32_t f = s_f[q], jj = q - base[f];
                if (jj < room[f]) {
                    const uint64_t dst = uint64_t(t0 + f) * p.cap_t + cur[f] + jj;
                    p.bin_lidx[dst] = s_l[q];
                    reinterpret_cast<V*>(p.bin_val)[dst] = s_v[q];
                }
            }
            if (s_spill) {                           // past the tile's region: applied now (exact: the
                for (uint32_t q = threadIdx.x; q < tot; q += kBT) {   // op is order-insensitive)
                    const uint32_t f = s_f[q], jj = q - base[f];
                    if (jj < room[f]) continue;
                    uint8_t okf;
                    rmw_global<V>(shard + uint64_t(t0 + f) * tile_elems + s_l[q], p.op, LMR_KIND_NATIVE_ATOMIC, s_v[q],
                                  V(0), V(0), okf, p.err);
                }
            }
            __syncthreads();
        }
        b = bn;
    }
    if (oob) raise_err(p.err, LMR_ERRBIT_OOB);
}

// an owner without a session workspace: every source's slices applied with device atomics (the
// mode's ops are order-insensitive); one (source, bucket) slice per block iteration
template <int VB>
__global__ __launch_bounds__(256) void k_bucket_direct(BFineK p) {
    using V = typename idx_t<VB>::I;
    bool oob = false;
    for (uint32_t sb = blockIdx.x; sb < p.S * p.C; sb += gridDim.x) {
        const uint32_t s = sb % p.S, b = sb / p.S;
        if (!p.idx[s]) continue;
        const uint32_t cnt = min(reinterpret_cast<const uint32_t*>(p.idx[s])[b], p.cap_b[s]);
        const uint32_t* off = reinterpret_cast<const uint32_t*>(p.idx[s] + kBucketHdr) + uint64_t(b) * p.cap_b[s];
        const V* val = p.val[s] ? reinterpret_cast<const V*>(p.val[s]) + uint64_t(b) * p.cap_b[s] : nullptr;
        for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
            const uint64_t e = (uint64_t(b) << p.cshift) + off[i];
            if (e >= p.shard_len) { oob = true; continue; }
            uint8_t okf;
            rmw_global<V>(reinterpret_cast<V*>(p.shard) + e, p.op, LMR_KIND_NATIVE_ATOMIC, val ? val[i] : V(p.sbits[s]),
                          V(0), V(0), okf, p.err);
        }
    }
    if (oob) raise_err(p.err, LMR_ERRBIT_OOB);
}

__global__ void k_bucket_plan(uint32_t* tfill, uint32_t T, uint64_t cap_t, TileItem* items) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const uint32_t f = tfill[t];
    const uint32_t lo = uint32_t(uint64_t(t) * cap_t);
    items[t] = TileItem{t, lo, lo + uint32_t(min<uint64_t>(f, cap_t)), f ? 0u : 2u};
    tfill[t] = 0;
}

template <typename F>
hipError_t bdispatch_vb(int vb, F&& f) {
    switch (vb) {
    case 1: return f(std::integral_constant<int, 1>{});
    case 2: return f(std::integral_constant<int, 2>{});
    case 4: return f(std::integral_constant<int, 4>{});
    case 8: return f(std::integral_constant<int, 8>{});
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

// LMR_BUCKET_TPB: log2 of the tiles per bucket (default 8: 256 tiles of 64 KiB). The sender's keys
// are PEs x buckets: at 8 PEs x 2^26-element u64 shards, 256 keys. Measured on one GPU at that
// geometry (tools/bucket_bench, per 2^26-record chunk, pack + owner fine pass on two streams):
// 128 tiles (512 keys) 1.13-1.17 ms, 256 tiles 1.02-1.06, 512 tiles 1.04; 64 tiles (1024 keys) 1.22
int bucket_tpb_log2() {
    static const int v = [] {
        const char* e = getenv("LMR_BUCKET_TPB");
        const int x = (e && *e) ? atoi(e) : 8;
        return x < 0 ? 0 : (x > 9 ? 9 : x);
    }();
    return v;
}

bool bucket_geometry(const lmr_layout_t& L, int dtype, uint32_t& C, int& cshift) {
    const int vb = dtype_bytes(dtype);
    if (vb == 0 || L.num_pes == 0 || L.num_pes > kBucketMaxSrc) return false;
    uint64_t maxlen = 0;
    for (uint32_t p = 0; p < L.num_pes; p++) maxlen = std::max<uint64_t>(maxlen, lmr_num_elems_pe(&L, p));
    const int ts = tile_shift(dtype);
    const uint64_t tiles = (maxlen + (uint64_t(1) << ts) - 1) >> ts;
    if (tiles == 0 || tiles > uint64_t(kMaxTiles)) return false;
    const int tl = bucket_tpb_log2();
    C = uint32_t((tiles + (uint64_t(1) << tl) - 1) >> tl);
    cshift = ts + tl;
    return uint64_t(C) * L.num_pes <= kBucketMaxKeys && uint64_t(C) * 4 <= kBucketHdr;
}

bool bucket_op_ok(int dtype, int op) {
    return dtype_bytes(dtype) > 0 && dtype <= LMR_I64 &&
           (op == LMR_OP_ADD || op == LMR_OP_SUB || op == LMR_OP_MUL || op == LMR_OP_AND || op == LMR_OP_OR ||
            op == LMR_OP_XOR);
}

uint32_t bucket_slice_cap(uint64_t R, uint32_t C, uint32_t eb) {
    if (C == 0 || R * 8 <= kBucketHdr) return 0;
    const uint64_t a = (R * 8 - kBucketHdr) / (uint64_t(C) * 4);
    const uint64_t b = eb ? R * 8 / (uint64_t(C) * eb) : a;
    return uint32_t(std::min<uint64_t>(std::min(a, b), 0xFFFF0000ull));
}

hipError_t launch_pack_bucket(const PackArgs& a, uint32_t C, int cshift, uint32_t cap_b, uint32_t* fill,
                              uint32_t* tot, hipStream_t s) {
    const uint32_t npes = a.layout.num_pes;
    if ((!a.out_idx_tab && !a.out_idx) || npes == 0 || npes > kBucketMaxSrc || uint64_t(C) * npes > kBucketMaxKeys)
        return hipErrorInvalidValue;
    uint64_t G = (a.n + 65535) / 65536;
    G = std::max<uint64_t>(1, std::min<uint64_t>(G, kMaxBinBlocks));
    BPackK p{};
    p.F = make_fast_layout(a.layout);
    p.gidx = a.gidx;
    p.vals = a.vals;
    p.val_bits = 0;
    p.n = a.n;
    p.chunk = std::max<uint64_t>(1, (a.n + G - 1) / G);
    p.npes = npes;
    p.C = C;
    p.cap_b = cap_b;
    p.cshift = cshift;
    p.idx_tab = a.out_idx_tab;
    p.val_tab = a.vals ? a.out_vals_tab : nullptr;
    p.idx_base = a.out_idx;
    p.val_base = a.vals ? a.out_vals : nullptr;
    p.idx_stride = kBucketHdr + uint64_t(C) * cap_b * 4;           // (send-buffer layout, bucket_region_bytes)
    p.val_stride = uint64_t(C) * cap_b * (a.vals ? a.val_bytes : 0);
    p.fill = fill;
    p.ovf_gidx = a.ovf_gidx;
    p.ovf_vals = a.ovf_vals;
    p.ovf_count = a.ovf_count;
    p.ovf_cap = a.ovf_cap;
    p.err = a.err;
    ProfScope ps(a.prof, LMR_STAGE_PACK, s, a.n);
    static const int rpt = [] { const char* e = getenv("LMR_BUCKET_RPT"); return (e && e[0] == '4') ? 4 : 8; }();
    static const bool pairs_on = [] { const char* e = getenv("LMR_PACK_PAIRS"); return !(e && e[0] == '0'); }();
    // (an even record count too: a block's last pair is loaded whole, so no load passes the arrays)
    const bool pairs = pairs_on && a.vals && a.val_bytes == 8 && (a.n & 1) == 0 &&
                       ((reinterpret_cast<uintptr_t>(a.gidx) | reinterpret_cast<uintptr_t>(a.vals)) & 15) == 0;
    if (pairs && (p.chunk & 1)) p.chunk += 1;
    if (a.n > 0) {
        const int mode = layout_map_mode(a.layout);
        const hipError_t e = bdispatch_vb(a.vals ? int(a.val_bytes) : 8, [&](auto vbt) {
            constexpr int VB = decltype(vbt)::value;
            auto go = [&](auto rt) {
                constexpr int R = decltype(rt)::value;
                constexpr bool kP = VB == 8;
                if (kP && pairs && mode == LMR_MAP_BLOCK)
                    hipLaunchKernelGGL((k_pack_bucket<VB, LMR_MAP_BLOCK, R, kP>), dim3(unsigned(G)), dim3(kBT), 0, s, p);
                else if (kP && pairs && mode == LMR_MAP_CYCLIC)
                    hipLaunchKernelGGL((k_pack_bucket<VB, LMR_MAP_CYCLIC, R, kP>), dim3(unsigned(G)), dim3(kBT), 0, s, p);
                else if (mode == LMR_MAP_BLOCK)
                    hipLaunchKernelGGL((k_pack_bucket<VB, LMR_MAP_BLOCK, R, false>), dim3(unsigned(G)), dim3(kBT), 0, s, p);
                else if (mode == LMR_MAP_CYCLIC)
                    hipLaunchKernelGGL((k_pack_bucket<VB, LMR_MAP_CYCLIC, R, false>), dim3(unsigned(G)), dim3(kBT), 0, s, p);
                else
                    hipLaunchKernelGGL((k_pack_bucket<VB, LMR_MAP_GENERIC, R, false>), dim3(unsigned(G)), dim3(kBT), 0, s,
                                       p);
            };
            if (rpt == 4) go(std::integral_constant<int, 4>{});
            else go(std::integral_constant<int, 8>{});
            return hipGetLastError();
        });
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_bucket_hdr, dim3(npes), dim3(256), 0, s, fill, C, cap_b, a.out_idx_tab, a.out_idx, p.idx_stride,
                       tot);
    return hipGetLastError();
}

uint64_t bucket_session_limit(const BucketSession& bs) {
    return uint64_t(bs.T) * bs.cap_t / 8 * 7;
}

hipError_t launch_fine_bucket(const BucketChunk& c, const BucketSession& bs, const TiledWs& w, hipStream_t st) {
    if (c.S == 0 || c.S > kBucketMaxSrc || uint64_t(bs.C) * c.S > 2 * kBucketMaxKeys || bs.T == 0 ||
        uint64_t(bs.T) * bs.cap_t > w.tmp_cap)
        return hipErrorInvalidValue;
    BFineK p{};
    for (uint32_t s = 0; s < c.S; s++) {
        p.idx[s] = c.idx[s];
        p.val[s] = c.val[s];
        p.sbits[s] = c.sbits[s];
        p.cap_b[s] = c.cap_b[s];
    }
    p.S = c.S;
    p.C = bs.C;
    p.T = bs.T;
    p.tpb = 1u << bs.tpb_log2;
    p.tile_shift = tile_shift(int(bs.desc.dtype));
    p.cap_t = bs.cap_t;
    p.bin_lidx = reinterpret_cast<uint16_t*>(w.tmp_idx);
    p.bin_val = w.tmp_val;
    p.tfill = bs.tfill;
    p.shard = bs.desc.shard;
    p.op = int(bs.desc.op);
    p.err = bs.err;
    ProfScope ps(bs.prof, LMR_STAGE_FINE_SCATTER, st, c.expect);
    static const int rpt = [] { const char* e = getenv("LMR_BUCKET_FRPT"); return (e && e[0] == '4') ? 4 : 8; }();
    return bdispatch_vb(dtype_bytes(int(bs.desc.dtype)), [&](auto vbt) {
        constexpr int VB = decltype(vbt)::value;
        if (rpt == 4) hipLaunchKernelGGL((k_fine_bucket<VB, 4>), dim3(1024), dim3(kBT), 0, st, p);
        else hipLaunchKernelGGL((k_fine_bucket<VB, 8>), dim3(1024), dim3(kBT), 0, st, p);
        return hipGetLastError();
    });
}

hipError_t launch_bucket_direct(const BucketChunk& c, const lmr_apply_desc_t& d, uint32_t C, int cshift, uint32_t* err,
                                hipStream_t st) {
    if (c.S == 0 || c.S > kBucketMaxSrc) return hipErrorInvalidValue;
    BFineK p{};
    for (uint32_t s = 0; s < c.S; s++) {
        p.idx[s] = c.idx[s];
        p.val[s] = c.val[s];
        p.sbits[s] = c.sbits[s];
        p.cap_b[s] = c.cap_b[s];
    }
    p.S = c.S;
    p.C = C;
    p.cshift = cshift;
    p.shard = d.shard;
    p.shard_len = d.shard_len;
    p.op = int(d.op);
    p.err = err;
    return bdispatch_vb(dtype_bytes(int(d.dtype)), [&](auto vbt) {
        constexpr int VB = decltype(vbt)::value;
        hipLaunchKernelGGL((k_bucket_direct<VB>), dim3(2048), dim3(256), 0, st, p);
        return hipGetLastError();
    });
}

uint64_t bucket_region_idx_bytes(uint32_t C, uint32_t cap_b) { return kBucketHdr + uint64_t(C) * cap_b * 4; }

hipError_t launch_bucket_sweep(BucketSession& bs, const TiledWs& w, hipStream_t st) {
    hipError_t e = hipSuccess;
    if (bs.open && bs.T > 0) {
        ProfScope ps(bs.prof, LMR_STAGE_TILE_APPLY, st, bs.staged);
        TileItem* items = reinterpret_cast<TileItem*>(w.items);
        hipLaunchKernelGGL(k_bucket_plan, dim3((bs.T + 255) / 256), dim3(256), 0, st, bs.tfill, bs.T, bs.cap_t, items);
        e = hipGetLastError();
        if (e == hipSuccess) {
            TileArgs t{};
            t.shard = bs.desc.shard;
            t.shard_len = bs.desc.shard_len;
            t.tile_shift = tile_shift(int(bs.desc.dtype));
            t.kind = int(bs.desc.kind);
            t.op = int(bs.desc.op);
            t.ret = LMR_RET_NONE;
            t.scalar = false;
            t.items = items;
            t.delta = items + kMaxTiles;
            t.delta_count = w.item_count;
            t.num_tiles = bs.T;
            t.bin_lidx = reinterpret_cast<const uint16_t*>(w.tmp_idx);
            t.bin_val = w.tmp_val;
            t.err = bs.err;
            t.nreg = 0;
            e = launch_tile_kernels(int(bs.desc.dtype), int(bs.desc.op), t, false, 0,
                                    st, w.side);
        }
    }
    bs.open = false;
    bs.staged = 0;
    return e;
}

}  // namespace lmr
