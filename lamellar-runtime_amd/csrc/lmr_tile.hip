// lmr_tile.hip — the tile sweep: k_tile_owner (one workgroup per 64 KiB shard tile, LDS
// atomics) and k_tile_delta (hot tiles of combinable ops split into pieces). Split from
// lmr_apply.hip so the two translation units compile in parallel.
#include "lmr_tile.hpp"
#include "lmr_device.hpp"
#include <cstdlib>

// records in flight per thread in k_tile_owner's 8-byte loop (A/B builds: -DLMR_OWN_UNROLL=...)
#ifndef LMR_OWN_UNROLL
#define LMR_OWN_UNROLL 4
#endif
// k_tile_owner reads 4 binned records per thread with wide loads (0: one record at a time)
#ifndef LMR_OWN_VEC
#define LMR_OWN_VEC 1
#endif

namespace lmr {

// delta mode: how records accumulate in LDS, how the block's delta reaches
// global memory, and how a record's old value is rebuilt from the base.
__device__ __forceinline__ int delta_acc_op(int op) {
    switch (op) {
    case LMR_OP_ADD: case LMR_OP_FETCH_ADD: case LMR_OP_SUB: case LMR_OP_FETCH_SUB: return LMR_OP_FETCH_ADD;
    case LMR_OP_AND: case LMR_OP_FETCH_AND: return LMR_OP_FETCH_AND;
    case LMR_OP_OR: case LMR_OP_FETCH_OR: return LMR_OP_FETCH_OR;
    default: return LMR_OP_FETCH_XOR;
    }
}
__device__ __forceinline__ int delta_global_op(int op) {
    switch (op) {
    case LMR_OP_ADD: case LMR_OP_FETCH_ADD: return LMR_OP_FETCH_ADD;
    case LMR_OP_SUB: case LMR_OP_FETCH_SUB: return LMR_OP_FETCH_SUB;
    case LMR_OP_AND: case LMR_OP_FETCH_AND: return LMR_OP_FETCH_AND;
    case LMR_OP_OR: case LMR_OP_FETCH_OR: return LMR_OP_FETCH_OR;
    default: return LMR_OP_FETCH_XOR;
    }
}
template <typename T>
__device__ __forceinline__ T delta_finish(int op, T base, T prefix) {
    using U = typename bits_of<T>::U;
    switch (op) {
    case LMR_OP_ADD: case LMR_OP_FETCH_ADD:
        if constexpr (is_flt<T>::v) return base + prefix; else return T(U(U(base) + U(prefix)));
    case LMR_OP_SUB: case LMR_OP_FETCH_SUB:
        if constexpr (is_flt<T>::v) return base - prefix; else return T(U(U(base) - U(prefix)));
    default: break;
    }
    if constexpr (!is_flt<T>::v) {
        if (op == LMR_OP_AND || op == LMR_OP_FETCH_AND) return T(base & prefix);
        if (op == LMR_OP_OR || op == LMR_OP_FETCH_OR) return T(base | prefix);
        return T(base ^ prefix);
    }
    return base;
}

// a (+) b for the delta accumulation ops (FETCH_ADD / AND / OR / XOR), wrapping for integers
template <typename T>
__device__ __forceinline__ T acc_comb(int acc, T a, T b) {
    using U = typename bits_of<T>::U;
    if (acc == LMR_OP_FETCH_ADD) {
        if constexpr (is_flt<T>::v) return a + b; else return T(U(U(a) + U(b)));
    }
    if constexpr (!is_flt<T>::v) {
        if (acc == LMR_OP_FETCH_AND) return T(a & b);
        if (acc == LMR_OP_FETCH_OR) return T(a | b);
        return T(a ^ b);
    }
    return a;
}
template <typename T>
__device__ __forceinline__ T shfl_t(T x, int src) {
    using U = typename bits_of<T>::U;
    if constexpr (sizeof(T) == 8) return from_bits<T>(U(__shfl((unsigned long long)U(to_bits(x)), src, 64)));
    else return from_bits<T>(U(__shfl(uint32_t(U(to_bits(x))), src, 64)));
}
template <typename T>
__device__ __forceinline__ T shfl_up_t(T x, int d) {
    using U = typename bits_of<T>::U;
    if constexpr (sizeof(T) == 8) return from_bits<T>(U(__shfl_up((unsigned long long)U(to_bits(x)), d, 64)));
    else return from_bits<T>(U(__shfl_up(uint32_t(U(to_bits(x))), d, 64)));
}

// One record per active lane accumulated into an LDS delta tile with `acc`, returning the
// element's previous delta. When many lanes of the wave name the first active lane's element
// (a hot element: Zipf streams put most of a hot tile's records on it), those lanes combine
// their values with a wave scan and one lane applies the sum: one LDS atomic instead of up to
// 64 serialised ones; lane j of the group gets base (+) the values of the group's lanes before j
// (the group applied in lane order, as one step). Called by every lane of the wave.
template <typename T>
__device__ __forceinline__ T lds_acc_wave(typename word_of<T>::W* tile, uint32_t l, T v, bool active, int acc,
                                          T ident, int kind, uint32_t* err) {
    const int lane = threadIdx.x & 63;
    const uint64_t act = __ballot(active);
    T res = ident;
    bool done = false;
    uint8_t ok = 0;
    if (act) {
        const int f = __ffsll((unsigned long long)act) - 1;
        const uint32_t l0 = __shfl(l, f, 64);
        const bool in = active && l == l0;
        const uint64_t m = __ballot(in);
        if (__popcll(m) >= 8) {
            T x = in ? v : ident;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const T y = shfl_up_t(x, d);
                if (lane >= d) x = acc_comb(acc, y, x);
            }
            T excl = shfl_up_t(x, 1);
            if (lane == 0) excl = ident;
            const T total = shfl_t(x, 63);
            T base = ident;
            if (lane == f) base = rmw_lds<T>(tile + l0, acc, kind, total, ident, ident, ok, err);
            base = shfl_t(base, f);
            if (in) {
                res = acc_comb(acc, base, excl);
                done = true;
            }
        }
    }
    if (active && !done) res = rmw_lds<T>(tile + l, acc, kind, v, ident, ident, ok, err);
    return res;
}

// the identity of addition: -0.0 for floats (-0.0 + x == x for every x, signed zeros included)
template <typename T>
__device__ __forceinline__ T add_ident() {
    using U = typename bits_of<T>::U;
    if constexpr (is_flt<T>::v) return from_bits<T>(U(U(1) << (8 * sizeof(U) - 1)));
    else return T(0);
}

// Off: measured no better (same box, alternating, profiles/r4/ab/r4l_*: C3 tile sweep 0.428-0.429 ->
// 0.433-0.435 ms, C2 unchanged): the owner tiles' warm elements are not where their time goes
#ifndef LMR_OWN_COMBINE
#define LMR_OWN_COMBINE 0
#endif
constexpr bool kOwnCombine = LMR_OWN_COMBINE != 0;   // wave-combined add in the owner kernel (A/B: -D...=1)

// OPT >= 0 fixes the op at compile time (hot paths); -1 reads it from the args.
// Owner mode: one block per tile — load the tile into LDS, apply the tile's
// records with LDS atomics, write it back. Kept free of the delta path's
// register arrays so two 1024-thread blocks (2 x 64 KiB LDS) fit per CU.
// PK: the wide path's packed records (a template parameter: a run-time test in the non-packed
// kernels cost C3's tile sweep 6-10 %, round 6)
template <typename T, int OPT, bool PK = false>
__global__ __launch_bounds__(1024, 8) void k_tile_owner(TileArgs a) {
    using U = typename bits_of<T>::U;
    using W = typename word_of<T>::W;
    extern __shared__ __align__(16) uint8_t lds_raw[];
    W* tile = reinterpret_cast<W*>(lds_raw);
    const TileItem w = a.items[blockIdx.x];
    if (w.mode != 0) return;
    const uint16_t* bin_lidx = a.bin_lidx;
    const T* bin_val = reinterpret_cast<const T*>(a.bin_val);
    int op = OPT >= 0 ? OPT : a.op;
    T cmp = from_bits<T>(U(a.cmp_bits)), eps = from_bits<T>(U(a.eps_bits));
    const T sv = from_bits<T>(U(a.val_bits));
    int ret = a.ret;
    const uint64_t base = uint64_t(w.tile) << a.tile_shift;
    const uint32_t len = uint32_t(min(uint64_t(1) << a.tile_shift, a.shard_len - base));
    T* shard = reinterpret_cast<T*>(a.shard) + base;
    // 16 B per lane when the shard is 16-B aligned (sub-array views may not be)
    const bool vec = sizeof(T) >= 4 && (reinterpret_cast<uintptr_t>(shard) & 15) == 0;
    if constexpr (sizeof(T) >= 4) {
        if (vec) {
            constexpr uint32_t per = 16 / sizeof(T);
            const uint32_t nv = len / per;
            // a full 64 KiB tile is 4 uint4 per thread: all four loads in flight, then the stores
            // (a load / wait / LDS-store loop kept one in flight); a 128 KiB wide tile is two such
            // groups (eight in flight spilled the 4-byte kernel's registers)
            if (nv == 4 * 1024u || nv == 8 * 1024u) {
                // (named registers, not a uint4[4]: the array stayed a stack object in the 4-byte
                // kernels, 48 B of dead scratch stores per thread and group)
                const uint4* src4 = reinterpret_cast<const uint4*>(shard) + threadIdx.x;
                uint4* dst4 = reinterpret_cast<uint4*>(tile) + threadIdx.x;
                for (uint32_t h = 0; h < nv; h += 4 * 1024u) {
                    const uint4 x0 = src4[h], x1 = src4[h + 1024u], x2 = src4[h + 2048u], x3 = src4[h + 3072u];
                    dst4[h] = x0;
                    dst4[h + 1024u] = x1;
                    dst4[h + 2048u] = x2;
                    dst4[h + 3072u] = x3;
                }
            } else {
                for (uint32_t v = threadIdx.x; v < nv; v += blockDim.x)
                    reinterpret_cast<uint4*>(tile)[v] = reinterpret_cast<const uint4*>(shard)[v];
            }
            for (uint32_t e = nv * per + threadIdx.x; e < len; e += blockDim.x) tile[e] = shard[e];
        } else {
            for (uint32_t e = threadIdx.x; e < len; e += blockDim.x) tile[e] = shard[e];   // W == T
        }
    } else {
        for (uint32_t e = threadIdx.x; e < len; e += blockDim.x) tile[e] = W(U(shard[e]));   // widen the bits
    }
    __syncthreads();
    // kOwnUnroll records per thread per round: all loads issued before the LDS atomics
    constexpr int kOwnUnroll = LMR_OWN_UNROLL;
    constexpr bool kOwnVec = LMR_OWN_VEC != 0;
    const uint32_t nrg = a.nreg ? a.nreg : 1u;
    for (uint32_t rg = 0; rg < nrg; rg++) {
    uint32_t lo = w.lo, hi = w.hi;
    if (a.nreg) {
        lo = a.rts[uint64_t(rg) * a.rstride + w.tile];
        hi = a.rts[uint64_t(rg) * a.rstride + w.tile + 1];
    }
    if (OPT < 0 && a.mixed) {          // the region's op; its records after every earlier region's
        op = a.rop[rg].op;
        ret = a.rop[rg].ret;
        cmp = from_bits<T>(U(a.rop[rg].cmp_bits));
        eps = from_bits<T>(U(a.rop[rg].eps_bits));
        if (rg) __syncthreads();
    }
    auto apply_one = [&](uint32_t r, uint32_t li, T vi) {
        uint8_t ok = 0;
        T old = rmw_lds<T>(tile + li, op, a.kind, vi, cmp, eps, ok, a.err);
        if (ret != LMR_RET_NONE) {
            reinterpret_cast<T*>(a.results)[r] = old;
            if (ret == LMR_RET_RESULT) a.ok[r] = ok;
        }
    };
    if constexpr (sizeof(T) <= 4) {
        // packed records (the wide path): one 8-B load per record, kPk in flight per thread
        if constexpr (PK) {
            const uint2* rec = reinterpret_cast<const uint2*>(a.bin_val);
            constexpr uint32_t kPk = 8;
            for (uint32_t b0 = lo; b0 < hi; b0 += kPk * 1024u) {
                uint2 x[kPk];
#pragma unroll
                for (uint32_t k = 0; k < kPk; k++) x[k] = rec[min(b0 + threadIdx.x + k * 1024u, hi - 1)];
#pragma unroll
                for (uint32_t k = 0; k < kPk; k++) {
                    const uint32_t r = b0 + threadIdx.x + k * 1024u;
                    if (r < hi) apply_one(r, x[k].x, from_bits<T>(U(x[k].y)));
                }
            }
            continue;
        }
    } else {
        // packed 16-B records of 8-byte values {index, 0, value}: one 16-B load per record
        if constexpr (PK) {
            const uint4* rec = reinterpret_cast<const uint4*>(a.bin_val);
            constexpr uint32_t kPk = 4;
            for (uint32_t b0 = lo; b0 < hi; b0 += kPk * 1024u) {
                uint4 x[kPk];
#pragma unroll
                for (uint32_t k = 0; k < kPk; k++) x[k] = rec[min(b0 + threadIdx.x + k * 1024u, hi - 1)];
#pragma unroll
                for (uint32_t k = 0; k < kPk; k++) {
                    const uint32_t r = b0 + threadIdx.x + k * 1024u;
                    if (r < hi) apply_one(r, x[k].x, from_bits<T>(U(uint64_t(x[k].z) | (uint64_t(x[k].w) << 32))));
                }
            }
            continue;
        }
    }
    if constexpr (sizeof(T) == 4) {
        // 4-byte values: 4 consecutive records per thread and iteration, one 8-B load of their
        // offsets and one 16-B load of their values (fewer, wider memory instructions than a 2-B
        // and a 4-B load per record); the unaligned head and the tail one record per thread.
        // Measured: C5 tile sweep 0.378 -> 0.354 ms; for 8-byte values the same grouping lost
        // (C2 tile 0.785 -> 0.80, C3 0.51 -> 0.54 ms), so they keep one record per load.
        if (kOwnVec && !a.scalar && ((reinterpret_cast<uintptr_t>(bin_lidx) & 7) | (reinterpret_cast<uintptr_t>(bin_val) & 15)) == 0) {
            const uint32_t a0 = min(hi, (lo + 3u) & ~3u);
            const uint32_t a1 = a0 + ((hi - a0) & ~3u);
            if (lo + threadIdx.x < a0) apply_one(lo + threadIdx.x, bin_lidx[lo + threadIdx.x], bin_val[lo + threadIdx.x]);
            if (a1 + threadIdx.x < hi) apply_one(a1 + threadIdx.x, bin_lidx[a1 + threadIdx.x], bin_val[a1 + threadIdx.x]);
            constexpr uint32_t kV = 2;           // groups of 4 records in flight per thread
            const uint32_t g0 = a0 >> 2, g1 = a1 >> 2;
            for (uint32_t q0 = g0 + threadIdx.x; q0 < g1; q0 += kV * 1024u) {
                uint2 lw[kV];
                T v[kV][4];
#pragma unroll
                for (uint32_t k = 0; k < kV; k++) {      // clamped, branch-free: every load in flight
                    const uint32_t q = min(q0 + k * 1024u, g1 - 1);
                    lw[k] = reinterpret_cast<const uint2*>(bin_lidx)[q];
                    const uint4 x = reinterpret_cast<const uint4*>(bin_val)[q];
                    v[k][0] = from_bits<T>(U(x.x)); v[k][1] = from_bits<T>(U(x.y));
                    v[k][2] = from_bits<T>(U(x.z)); v[k][3] = from_bits<T>(U(x.w));
                }
#pragma unroll
                for (uint32_t k = 0; k < kV; k++) {
                    const uint32_t q = q0 + k * 1024u;
                    if (q < g1) {
                        apply_one(4 * q + 0, lw[k].x & 0xffffu, v[k][0]);
                        apply_one(4 * q + 1, lw[k].x >> 16, v[k][1]);
                        apply_one(4 * q + 2, lw[k].y & 0xffffu, v[k][2]);
                        apply_one(4 * q + 3, lw[k].y >> 16, v[k][3]);
                    }
                }
            }
            continue;
        }
    }
    // add / fetch_add (compile-time op): a wave's records on one element (Zipf-warm elements of
    // an owner tile) are combined with a wave scan and applied with one LDS atomic (lds_acc_wave:
    // each record returns base (+) the values before it in the group, applied as one step); the
    // loop is block-uniform so every lane of a wave takes part in the scan
    constexpr bool kComb = kOwnCombine && (OPT == LMR_OP_ADD || OPT == LMR_OP_FETCH_ADD);
    for (uint32_t b0 = lo; b0 < hi; b0 += kOwnUnroll * 1024u) {
        const uint32_t r0 = b0 + threadIdx.x;
        uint32_t l[kOwnUnroll];
        T v[kOwnUnroll];
#pragma unroll
        for (int k = 0; k < kOwnUnroll; k++) {          // clamped, branch-free: every load in flight
            const uint32_t r = min(r0 + uint32_t(k) * 1024u, hi - 1);
            l[k] = bin_lidx[r];
            v[k] = a.scalar ? sv : bin_val[r];
        }
#pragma unroll
        for (int k = 0; k < kOwnUnroll; k++) {
            const uint32_t r = r0 + uint32_t(k) * 1024u;
            if constexpr (kComb) {
                const bool in = r < hi;
                const T old = lds_acc_wave<T>(tile, l[k], v[k], in, LMR_OP_FETCH_ADD, add_ident<T>(), a.kind, a.err);
                if (in && ret != LMR_RET_NONE) reinterpret_cast<T*>(a.results)[r] = old;
            } else if (r < hi) {
                uint8_t ok = 0;
                T old = rmw_lds<T>(tile + l[k], op, a.kind, v[k], cmp, eps, ok, a.err);
                if (ret != LMR_RET_NONE) {
                    reinterpret_cast<T*>(a.results)[r] = old;          // coalesced (binned order)
                    if (ret == LMR_RET_RESULT) a.ok[r] = ok;
                }
            }
        }
    }
    }
    __syncthreads();
    if (!op_is_read(op) || (OPT < 0 && a.mixed)) {
        if constexpr (sizeof(T) >= 4) {
            if (vec) {
                constexpr uint32_t per = 16 / sizeof(T);
                const uint32_t nv = len / per;
                for (uint32_t v = threadIdx.x; v < nv; v += blockDim.x)
                    reinterpret_cast<uint4*>(shard)[v] = reinterpret_cast<const uint4*>(tile)[v];
                for (uint32_t e = nv * per + threadIdx.x; e < len; e += blockDim.x) shard[e] = tile[e];
            } else {
                for (uint32_t e = threadIdx.x; e < len; e += blockDim.x) shard[e] = tile[e];
            }
        } else {
            for (uint32_t e = threadIdx.x; e < len; e += blockDim.x) shard[e] = T(U(tile[e]));
        }
    }
}

// Delta mode (combinable ops only; planned by k_tile_plan / k_stage_plan), persistent
// over the delta list: combine kSplit records in an identity-initialised LDS
// tile, push one device-scope atomic per touched element, rebuild fetch
// results as base (+) the record's LDS prefix.
template <typename T, int OPT, int TB = kTileBytes, bool PK = false>
__global__ __launch_bounds__(1024) void k_tile_delta(TileArgs a) {
    using U = typename bits_of<T>::U;
    using W = typename word_of<T>::W;
    extern __shared__ __align__(16) uint8_t lds_raw[];
    W* tile = reinterpret_cast<W*>(lds_raw);
    const int op = OPT >= 0 ? OPT : a.op;
    const T cmp = from_bits<T>(U(a.cmp_bits)), eps = from_bits<T>(U(a.eps_bits));
    const T sv = from_bits<T>(U(a.val_bits));
    const int ret = a.ret;
    const uint32_t nitems = *a.delta_count;
    const uint16_t* bin_lidx = a.bin_lidx;
    const T* bin_val = reinterpret_cast<const T*>(a.bin_val);
    // floats: -0.0 is the identity of IEEE addition (-0.0 + x == x for every x, +0.0 and
    // NaN included; +0.0 + -0.0 would be +0.0), and a - v is a + (-v) bit for bit, so a
    // float sub piece accumulates -v and is applied as an add: base + (sum of its values)
    // then keeps the sign of zero a serial chain of single RMWs gives
    constexpr bool kFlt = is_flt<T>::v;
    const bool fsub = kFlt && (op == LMR_OP_SUB || op == LMR_OP_FETCH_SUB);
    const U ident_bits = (op == LMR_OP_AND || op == LMR_OP_FETCH_AND) ? ~U(0)
                         : kFlt ? U(U(1) << (8 * sizeof(U) - 1)) : U(0);
    W ident;
    if constexpr (kFlt) ident = from_bits<T>(ident_bits);
    else ident = W(ident_bits);
    const int acc = delta_acc_op(op);
    const int gop = fsub ? int(LMR_OP_FETCH_ADD) : delta_global_op(op);
    const int fop = fsub ? int(LMR_OP_FETCH_ADD) : op;
    // elements some record of the piece touched (fetch forms: only those need their base)
    constexpr int kTileWords = TB / int(sizeof(W));
    __shared__ uint32_t touched[kTileWords / 32];
    for (uint32_t it = blockIdx.x; it < nitems; it += gridDim.x) {
        const TileItem w = a.delta[it];
        const uint64_t base = uint64_t(w.tile) << a.tile_shift;
        const uint32_t len = uint32_t(min(uint64_t(1) << a.tile_shift, a.shard_len - base));
        T* shard = reinterpret_cast<T*>(a.shard) + base;
        for (uint32_t e = threadIdx.x; e < len; e += blockDim.x) tile[e] = ident;
        if (ret != LMR_RET_NONE)
            for (uint32_t e = threadIdx.x; e < (len + 31) / 32; e += blockDim.x) touched[e] = 0;
        __syncthreads();
        T pre[kSplit / 1024];
        // the piece's records loaded first (clamped, branch-free: all in flight), then combined
        uint16_t lk[kSplit / 1024];
        T vk[kSplit / 1024];
        if constexpr (PK) {                                     // the wide path's packed records
#pragma unroll
            for (int k = 0; k < int(kSplit / 1024); k++) {
                const uint32_t r = min(w.lo + threadIdx.x + uint32_t(k) * 1024u, w.hi - 1);
                if constexpr (sizeof(T) <= 4) {
                    const uint2 x = reinterpret_cast<const uint2*>(a.bin_val)[r];
                    lk[k] = uint16_t(x.x);
                    vk[k] = from_bits<T>(U(x.y));
                } else {
                    const uint4 x = reinterpret_cast<const uint4*>(a.bin_val)[r];
                    lk[k] = uint16_t(x.x);
                    vk[k] = from_bits<T>(U(uint64_t(x.z) | (uint64_t(x.w) << 32)));
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < int(kSplit / 1024); k++) {
                const uint32_t r = min(w.lo + threadIdx.x + uint32_t(k) * 1024u, w.hi - 1);
                lk[k] = bin_lidx[r];
                vk[k] = a.scalar ? sv : bin_val[r];
            }
        }
#pragma unroll
        for (int k = 0; k < int(kSplit / 1024); k++) {
            const uint32_t r = w.lo + threadIdx.x + uint32_t(k) * 1024u;
            const bool in = r < w.hi;
            const uint32_t l = in ? lk[k] : 0u;
            T v = in ? vk[k] : T(0);
            if (fsub) v = -v;
            if (kWaveCombine) {
                pre[k] = lds_acc_wave<T>(tile, l, v, in, acc, from_bits<T>(ident_bits), a.kind, a.err);
            } else if (in) {
                uint8_t ok = 0;
                pre[k] = rmw_lds<T>(tile + l, acc, a.kind, v, cmp, eps, ok, a.err);
            }
            // the first record on an element sees the identity (later ones may too: harmless)
            if (in && ret != LMR_RET_NONE && U(to_bits(pre[k])) == U(ident_bits)) atomicOr(&touched[l >> 5], 1u << (l & 31));
        }
        __syncthreads();
        // one device-scope atomic per changed element, a load per touched unchanged one; every
        // element's operation of a group of up to 16 per thread is issued before any result is
        // waited for (a 128 KiB tile of 32-bit words is two groups)
        constexpr int kPer = kTileWords / 1024;           // elements per thread (a tile's words / 1024)
        constexpr int kGrp = kPer < 16 ? kPer : (kPer > 16 ? 8 : 16);   // (16 of 32 spilled)
        static_assert(kPer % kGrp == 0, "whole groups");
        for (int k0 = 0; k0 < kPer; k0 += kGrp) {
            T b[kGrp];
            bool need[kGrp];
#pragma unroll
            for (int k = 0; k < kGrp; k++) {
                const uint32_t e = threadIdx.x + uint32_t(k0 + k) * 1024u;
                need[k] = false;
                if (e < len) {
                    T d;
                    if constexpr (sizeof(T) >= 4) d = tile[e];
                    else d = T(U(tile[e]));
                    uint8_t ok = 0;
                    if (U(to_bits(d)) != U(ident_bits)) {
                        b[k] = rmw_global<T>(shard + e, gop, a.kind, d, cmp, eps, ok, a.err);
                        need[k] = true;
                    } else if (ret != LMR_RET_NONE && ((touched[e >> 5] >> (e & 31)) & 1u)) {
                        b[k] = rmw_global<T>(shard + e, LMR_OP_LOAD, a.kind, d, cmp, eps, ok, a.err);
                        need[k] = true;
                    }
                }
            }
            if (ret != LMR_RET_NONE) {
#pragma unroll
                for (int k = 0; k < kGrp; k++) {
                    const uint32_t e = threadIdx.x + uint32_t(k0 + k) * 1024u;
                    if (need[k]) {
                        if constexpr (sizeof(T) >= 4) tile[e] = b[k];
                        else tile[e] = W(U(b[k]));
                    }
                }
            }
        }
        if (ret != LMR_RET_NONE) {
            __syncthreads();
#pragma unroll
            for (int k = 0; k < int(kSplit / 1024); k++) {
                const uint32_t r = w.lo + threadIdx.x + uint32_t(k) * 1024u;
                if (r < w.hi) {
                    const uint32_t l = lk[k];
                    T bb;
                    if constexpr (sizeof(T) >= 4) bb = tile[l];
                    else bb = T(U(tile[l]));
                    reinterpret_cast<T*>(a.results)[r] = delta_finish<T>(fop, bb, pre[k]);
                }
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ dispatch
template <typename F>
static hipError_t dispatch_dtype_t(int dtype, F&& f) {
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
[[maybe_unused]] static hipError_t dispatch_iw(int iw, F&& f) {
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


// The delta pieces (hot tiles, device atomics and LDS combining: latency-bound) run on the side
// lane beside the owner tiles (HBM-bound); the owner kernel skips the split tiles, so the two
// touch disjoint tiles, records and results. LMR_DELTA_SIDE=0 keeps both on the launch stream.
static bool delta_side_enabled() {
    static const bool on = [] {
        const char* v = getenv("LMR_DELTA_SIDE");
        return !(v && v[0] == '0');
    }();
    return on;
}

// dynamic LDS above the default limit is declared once per kernel instantiation
template <typename K>
static hipError_t allow_lds(K kernel, uint32_t bytes) {
    if (bytes <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               int(bytes));
}

hipError_t launch_tile_kernels(int dtype, int opt, const TileArgs& t, bool delta, unsigned dgrid, hipStream_t s,
                               const SideLane& side, uint32_t tile_bytes) {
    const bool lane = delta && side.s && delta_side_enabled();
    if (tile_bytes != kTileBytes && tile_bytes != kWideBytes) return hipErrorInvalidValue;
    if (lane && (hipEventRecord(side.fork, s) != hipSuccess || hipStreamWaitEvent(side.s, side.fork, 0) != hipSuccess))
        return hipErrorUnknown;
    const hipError_t e = dispatch_dtype_t(dtype, [&](auto tag) {
        using Ty = decltype(tag);
        auto go = [&](auto optc, auto tbc, auto pkc) {
            constexpr int OPT = decltype(optc)::value, TB = decltype(tbc)::value;
            constexpr bool PK = decltype(pkc)::value;
            auto* kd = k_tile_delta<Ty, OPT, TB, PK>;
            auto* ko = k_tile_owner<Ty, OPT, PK>;
            hipError_t ea = allow_lds(kd, TB);
            if (ea == hipSuccess) ea = allow_lds(ko, TB);
            if (ea != hipSuccess) return ea;
            if (lane)          // first, so its blocks start while the owner grid fills the chip
                hipLaunchKernelGGL(kd, dim3(dgrid), dim3(1024), size_t(TB), side.s, t);
            hipLaunchKernelGGL(ko, dim3(t.num_tiles), dim3(1024), size_t(TB), s, t);
            if (delta && !lane)
                hipLaunchKernelGGL(kd, dim3(dgrid), dim3(1024), size_t(TB), s, t);
            return hipSuccess;
        };
        auto by_op = [&](auto tbc, auto pkc) {
            if (opt == LMR_OP_ADD) return go(std::integral_constant<int, LMR_OP_ADD>{}, tbc, pkc);
            if (opt == LMR_OP_FETCH_ADD) return go(std::integral_constant<int, LMR_OP_FETCH_ADD>{}, tbc, pkc);
            return go(std::integral_constant<int, -1>{}, tbc, pkc);
        };
        using W = std::integral_constant<int, int(kWideBytes)>;
        // (packed records only on the wide path)
        const hipError_t el = tile_bytes != kWideBytes ? by_op(std::integral_constant<int, kTileBytes>{}, std::false_type{})
                              : t.packed ? by_op(W{}, std::true_type{})
                                         : by_op(W{}, std::false_type{});
        return el != hipSuccess ? el : hipGetLastError();
    });
    // the launch stream continues after both (joined even when a launch failed)
    if (lane && (hipEventRecord(side.join, side.s) != hipSuccess || hipStreamWaitEvent(s, side.join, 0) != hipSuccess))
        return e != hipSuccess ? e : hipErrorUnknown;
    return e;
}

}  // namespace lmr
