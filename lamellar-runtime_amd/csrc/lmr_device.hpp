// lmr_device.hpp — device-side building blocks for the gfx950 batched
// element-op path: element-type traits, (sub)array index math, and the
// per-element read-modify-write that every apply kernel uses.
//
// The RMW restates the per-kind op semantics of the reference's generated
// apply bodies (impl/src/array_ops.rs:327-545, src/array/native_atomic.rs:29-113)
// as single device atomics where CDNA4 has one and as compare-and-swap loops
// where it does not. Every record is applied atomically per element, which is
// a valid linearisation of all reference array kinds (NativeAtomic: SeqCst
// RMW; Generic: per-element mutex; LocalLock/GlobalLock: whole-shard lock;
// Unsafe: racy, so any atomic order is allowed).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/lamellar_types.h"

namespace lmr {

// ---------------------------------------------------------------- traits
template <typename T> struct bits_of;
template <> struct bits_of<uint8_t>  { using U = uint8_t;  };
template <> struct bits_of<int8_t>   { using U = uint8_t;  };
template <> struct bits_of<uint16_t> { using U = uint16_t; };
template <> struct bits_of<int16_t>  { using U = uint16_t; };
template <> struct bits_of<uint32_t> { using U = uint32_t; };
template <> struct bits_of<int32_t>  { using U = uint32_t; };
template <> struct bits_of<uint64_t> { using U = uint64_t; };
template <> struct bits_of<int64_t>  { using U = uint64_t; };
template <> struct bits_of<float>    { using U = uint32_t; };
template <> struct bits_of<double>   { using U = uint64_t; };

template <typename T> struct is_flt { static constexpr bool v = false; };
template <> struct is_flt<float>  { static constexpr bool v = true; };
template <> struct is_flt<double> { static constexpr bool v = true; };

template <typename T> struct is_sgn { static constexpr bool v = T(-1) < T(0); };

template <typename T> __host__ __device__ inline constexpr T min_of() {
    return is_sgn<T>::v ? T(T(1) << (sizeof(T) * 8 - 1)) : T(0);
}

// LDS word type: 8/16-bit elements are widened to 32 bits in LDS tiles so the
// ds_* atomics apply (low bits hold the element; high bits are ignored).
template <typename T> struct word_of { using W = T; };
template <> struct word_of<uint8_t>  { using W = uint32_t; };
template <> struct word_of<int8_t>   { using W = uint32_t; };
template <> struct word_of<uint16_t> { using W = uint32_t; };
template <> struct word_of<int16_t>  { using W = uint32_t; };

template <typename T>
__device__ __forceinline__ T from_bits(typename bits_of<T>::U u) { return __builtin_bit_cast(T, u); }
template <typename T>
__device__ __forceinline__ typename bits_of<T>::U to_bits(T v) {
    return __builtin_bit_cast(typename bits_of<T>::U, v);
}

// ---------------------------------------------------------------- layout
// Restates UnsafeArray::pe_and_offset_for_global_index (src/array/unsafe.rs:1207-1223)
// and the helpers it calls (:1610-1647 full arrays, :1651-1673 and :1708-1736 sub-arrays).
__host__ __device__ inline bool pe_for_dist_index(const lmr_layout_t& L, uint64_t index,
                                                  uint64_t& pe) {
    if (!(L.size > index)) return false;
    uint64_t g = index + L.offset;
    if (L.distribution == LMR_DIST_BLOCK) {
        uint64_t rem_index = L.orig_remaining_elems * (L.orig_elem_per_pe + 1);
        pe = (g < rem_index) ? g / (L.orig_elem_per_pe + 1)
                             : L.orig_remaining_elems + (g - rem_index) / L.orig_elem_per_pe;
    } else {
        pe = g % L.num_pes;
    }
    return true;
}

__host__ __device__ inline bool pe_and_offset(const lmr_layout_t& L, uint64_t index,
                                              uint64_t& pe, uint64_t& off) {
    if (!(L.size > index)) return false;
    if (!L.sub) {
        if (L.distribution == LMR_DIST_BLOCK) {
            uint64_t rem_index = L.orig_remaining_elems * (L.orig_elem_per_pe + 1);
            if (index < rem_index) {
                pe = index / (L.orig_elem_per_pe + 1);
                off = index - pe * (L.orig_elem_per_pe + 1);
            } else {
                uint64_t t = index - rem_index;
                uint64_t tp = t / L.orig_elem_per_pe;
                pe = L.orig_remaining_elems + tp;
                off = t - tp * L.orig_elem_per_pe;
            }
        } else {
            pe = index % L.num_pes;
            off = index / L.num_pes;
        }
        return true;
    }
    pe_for_dist_index(L, index, pe);
    uint64_t start_pe;
    pe_for_dist_index(L, 0, start_pe);
    if (L.distribution == LMR_DIST_BLOCK) {
        if (start_pe == pe) { off = index; return true; }
        uint64_t g = L.offset + index;
        uint64_t rem_index = L.orig_remaining_elems * (L.orig_elem_per_pe + 1);
        if (g < rem_index) {
            off = g - pe * (L.orig_elem_per_pe + 1);
        } else {
            uint64_t t = g - rem_index;
            uint64_t tp = t / L.orig_elem_per_pe;
            off = t - tp * L.orig_elem_per_pe;
        }
        return true;
    }
    off = index / L.num_pes;  // (index + offset) % npes == pe holds by construction
    return true;
}

// Same mapping with the runtime 64-bit divisions replaced by a double-precision
// reciprocal and a one-step correction (exact for dividends below 2^52; larger
// ones take the generic path). A u64 `/` is a ~100-instruction sequence on
// CDNA, and the pack divides every record twice.
struct FastLayout {
    lmr_layout_t L;
    uint64_t a, b, rem_index;          // orig_elem_per_pe + 1, orig_elem_per_pe, rem * a
    double inv_a, inv_b, inv_np;
};

__host__ inline FastLayout make_fast_layout(const lmr_layout_t& L) {
    FastLayout f;
    f.L = L;
    f.a = L.orig_elem_per_pe + 1;
    f.b = L.orig_elem_per_pe;
    f.rem_index = L.orig_remaining_elems * f.a;
    f.inv_a = 1.0 / double(f.a);
    f.inv_b = f.b ? 1.0 / double(f.b) : 0.0;
    f.inv_np = L.num_pes ? 1.0 / double(L.num_pes) : 0.0;
    return f;
}

__host__ __device__ __forceinline__ void fast_divmod(uint64_t n, uint64_t d, double inv, uint64_t& q,
                                                     uint64_t& r) {
    if (n < (uint64_t(1) << 52)) {
        q = uint64_t(double(n) * inv);
        r = n - q * d;
        if (int64_t(r) < 0) { q--; r += d; }
        else if (r >= d) { q++; r -= d; }
    } else {
        q = n / d;
        r = n - q * d;
    }
}

__host__ __device__ __forceinline__ bool pe_and_offset_fast(const FastLayout& f, uint64_t index,
                                                            uint64_t& pe, uint64_t& off) {
    if (f.L.sub) return pe_and_offset(f.L, index, pe, off);
    if (!(f.L.size > index)) return false;
    if (f.L.distribution == LMR_DIST_BLOCK) {
        if (index < f.rem_index) {
            fast_divmod(index, f.a, f.inv_a, pe, off);
        } else {
            uint64_t tp;
            fast_divmod(index - f.rem_index, f.b, f.inv_b, tp, off);
            pe = f.L.orig_remaining_elems + tp;
        }
    } else {
        fast_divmod(index, f.L.num_pes, f.inv_np, off, pe);
    }
    return true;
}

// Layout mode resolved once on the host so the per-record mapping is branch-free:
// 0 = full Block array, 1 = full Cyclic array, 2 = anything else (sub-arrays).
enum { LMR_MAP_BLOCK = 0, LMR_MAP_CYCLIC = 1, LMR_MAP_GENERIC = 2 };

__host__ inline int layout_map_mode(const lmr_layout_t& L) {
    if (L.sub) return LMR_MAP_GENERIC;
    return L.distribution == LMR_DIST_BLOCK ? LMR_MAP_BLOCK : LMR_MAP_CYCLIC;
}

template <int MODE>
__host__ __device__ __forceinline__ bool pe_and_offset_mode(const FastLayout& f, uint64_t index, uint64_t& pe,
                                                            uint64_t& off) {
    if constexpr (MODE == LMR_MAP_GENERIC) {
        return pe_and_offset(f.L, index, pe, off);
    } else {
        if (!(f.L.size > index)) return false;
        if constexpr (MODE == LMR_MAP_BLOCK) {
            if (index < f.rem_index) {
                fast_divmod(index, f.a, f.inv_a, pe, off);
            } else {
                uint64_t tp;
                fast_divmod(index - f.rem_index, f.b, f.inv_b, tp, off);
                pe = f.L.orig_remaining_elems + tp;
            }
        } else {
            fast_divmod(index, f.L.num_pes, f.inv_np, off, pe);
        }
        return true;
    }
}

// ---------------------------------------------------------------- errors
__device__ __forceinline__ void raise_err(uint32_t* err, uint32_t bit) {
    if (err) __hip_atomic_fetch_or(err, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- op math
// new value for `old op v` (pure function, no memory). Returns false when the
// op must not be applied (Rust would panic): errbit is set accordingly.
// `ok` is written for the two Result ops; `ret` is the value the record returns.
template <typename T>
__device__ __forceinline__ bool op_math(int op, int kind, T old, T v, T cmp, T eps,
                                        T& nw, T& ret, uint8_t& ok, uint32_t& errbit) {
    using U = typename bits_of<T>::U;
    ret = old;
    nw = old;
    switch (op) {
    case LMR_OP_ADD: case LMR_OP_FETCH_ADD:
        if constexpr (is_flt<T>::v) nw = old + v; else nw = T(U(U(old) + U(v)));
        return true;
    case LMR_OP_SUB: case LMR_OP_FETCH_SUB:
        if constexpr (is_flt<T>::v) nw = old - v; else nw = T(U(U(old) - U(v)));
        return true;
    case LMR_OP_MUL: case LMR_OP_FETCH_MUL:
        if constexpr (is_flt<T>::v) nw = old * v;
        else if constexpr (sizeof(T) < 4) nw = T(U(uint32_t(U(old)) * uint32_t(U(v))));
        else nw = T(U(U(old) * U(v)));
        return true;
    case LMR_OP_DIV: case LMR_OP_FETCH_DIV:
        if constexpr (is_flt<T>::v) { nw = old / v; return true; }
        else {
            if (v == T(0)) { errbit = LMR_ERRBIT_DIVZERO; return false; }
            if constexpr (is_sgn<T>::v)
                if (old == min_of<T>() && v == T(-1)) { errbit = LMR_ERRBIT_OVERFLOW; return false; }
            nw = T(old / v);
            return true;
        }
    case LMR_OP_REM: case LMR_OP_FETCH_REM:
        if constexpr (is_flt<T>::v) { nw = fmod(old, v); return true; }
        else {
            if (v == T(0)) { errbit = LMR_ERRBIT_DIVZERO; return false; }
            if constexpr (is_sgn<T>::v)
                if (old == min_of<T>() && v == T(-1)) { errbit = LMR_ERRBIT_OVERFLOW; return false; }
            nw = T(old % v);
            return true;
        }
    case LMR_OP_STORE: case LMR_OP_PUT: case LMR_OP_SWAP:
        nw = v;
        return true;
    case LMR_OP_LOAD: case LMR_OP_GET:
        return true;
    case LMR_OP_COMPARE_EXCHANGE_EPS: {
        if constexpr (is_flt<T>::v) {
            bool same = (cmp > old) ? ((cmp - old) < eps) : ((old - cmp) < eps);
            if (same) { nw = v; ok = 1; ret = cmp; } else { ok = 0; }
            return true;
        } else {
            if (kind == LMR_KIND_NATIVE_ATOMIC) {
                // impl/src/array_ops.rs:391-419
                if (old == cmp) { nw = v; ok = 1; ret = v; return true; }
                U d = (old > cmp) ? U(U(old) - U(cmp)) : U(U(cmp) - U(old));
                if (T(d) < eps) { nw = v; ok = 1; ret = old; } else { ok = 0; }
                return true;
            }
            // impl/src/array_ops.rs:521-535
            bool same = (cmp > old) ? (T(U(U(cmp) - U(old))) < eps) : (T(U(U(old) - U(cmp))) < eps);
            if (same) { nw = v; ok = 1; ret = cmp; } else { ok = 0; }
            return true;
        }
    }
    default: break;
    }
    if constexpr (!is_flt<T>::v) {
        constexpr unsigned BITS = sizeof(T) * 8;
        switch (op) {
        case LMR_OP_AND: case LMR_OP_FETCH_AND: nw = T(old & v); return true;
        case LMR_OP_OR:  case LMR_OP_FETCH_OR:  nw = T(old | v); return true;
        case LMR_OP_XOR: case LMR_OP_FETCH_XOR: nw = T(old ^ v); return true;
        case LMR_OP_COMPARE_EXCHANGE:
            if (old == cmp) { nw = v; ok = 1; ret = cmp; } else { ok = 0; }
            return true;
        case LMR_OP_SHL: case LMR_OP_FETCH_SHL: {
            unsigned s = unsigned(U(v)) & (BITS - 1);
            if constexpr (sizeof(T) < 4) nw = T(U(uint32_t(U(old)) << s));
            else nw = T(U(U(old) << s));
            return true;
        }
        case LMR_OP_SHR: case LMR_OP_FETCH_SHR: {
            unsigned s = unsigned(U(v)) & (BITS - 1);
            nw = T(old >> s);
            return true;
        }
        default: break;
        }
    }
    errbit = LMR_ERRBIT_UNSUPPORTED;
    return false;
}

// true when `op` never changes the element (no write needed)
__device__ __forceinline__ bool op_is_read(int op) { return op == LMR_OP_LOAD || op == LMR_OP_GET; }

// ---------------------------------------------------------------- RMW on a
// naturally aligned 32/64-bit word (global or LDS; the address space is
// inferred after inlining). T has sizeof 4 or 8.
template <typename T>
__device__ __forceinline__ T rmw_word(T* p, int op, int kind, T v, T cmp, T eps,
                                      uint8_t& ok, uint32_t* err) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "word RMW");
    using U = typename bits_of<T>::U;
    U* up = reinterpret_cast<U*>(p);
    // single-instruction forms
    if constexpr (!is_flt<T>::v) {
        switch (op) {
        case LMR_OP_ADD: case LMR_OP_FETCH_ADD:
            return T(__hip_atomic_fetch_add(up, U(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        case LMR_OP_SUB: case LMR_OP_FETCH_SUB:
            return T(__hip_atomic_fetch_add(up, U(U(0) - U(v)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        case LMR_OP_AND: case LMR_OP_FETCH_AND:
            return T(__hip_atomic_fetch_and(up, U(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        case LMR_OP_OR: case LMR_OP_FETCH_OR:
            return T(__hip_atomic_fetch_or(up, U(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        case LMR_OP_XOR: case LMR_OP_FETCH_XOR:
            return T(__hip_atomic_fetch_xor(up, U(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        case LMR_OP_COMPARE_EXCHANGE: {
            U expected = U(cmp);
            __hip_atomic_compare_exchange_strong(up, &expected, U(v), __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // expected now holds the value that was there
            ok = (expected == U(cmp)) ? 1 : 0;
            return ok ? cmp : T(expected);
        }
        default: break;
        }
    } else {
        if (op == LMR_OP_ADD || op == LMR_OP_FETCH_ADD)
            return unsafeAtomicAdd(p, v);
        if (op == LMR_OP_SUB || op == LMR_OP_FETCH_SUB)
            return unsafeAtomicAdd(p, -v);   // x - y == x + (-y) in IEEE-754
    }
    if (op == LMR_OP_STORE || op == LMR_OP_PUT || op == LMR_OP_SWAP)
        return from_bits<T>(__hip_atomic_exchange(up, to_bits(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (op_is_read(op))
        return from_bits<T>(__hip_atomic_load(up, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    // compare-and-swap loop for mul/div/rem/shl/shr/compare_exchange_epsilon
    U cur = __hip_atomic_load(up, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (true) {
        T old = from_bits<T>(cur), nw, ret;
        uint32_t eb = 0;
        if (!op_math<T>(op, kind, old, v, cmp, eps, nw, ret, ok, eb)) {
            raise_err(err, eb);
            return old;
        }
        U nb = to_bits(nw);
        if (nb == cur) return ret;   // nothing to write (e.g. failed compare)
        U expected = cur;
        if (__hip_atomic_compare_exchange_strong(up, &expected, nb, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return ret;
        cur = expected;
    }
}

// RMW of an 8/16-bit element held in the low bits of a 32-bit LDS word.
template <typename T>
__device__ __forceinline__ T rmw_widened(uint32_t* p, int op, int kind, T v, T cmp, T eps,
                                         uint8_t& ok, uint32_t* err) {
    using U = typename bits_of<T>::U;
    // wrapping add/sub/and/or/xor on the low bits are exact in 32 bits
    switch (op) {
    case LMR_OP_ADD: case LMR_OP_FETCH_ADD:
        return T(U(__hip_atomic_fetch_add(p, uint32_t(U(v)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)));
    case LMR_OP_SUB: case LMR_OP_FETCH_SUB:
        return T(U(__hip_atomic_fetch_add(p, uint32_t(0) - uint32_t(U(v)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)));
    case LMR_OP_AND: case LMR_OP_FETCH_AND:
        return T(U(__hip_atomic_fetch_and(p, uint32_t(U(v)) | 0xFFFFFFFFu << (8 * sizeof(T)),
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)));
    case LMR_OP_OR: case LMR_OP_FETCH_OR:
        return T(U(__hip_atomic_fetch_or(p, uint32_t(U(v)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)));
    case LMR_OP_XOR: case LMR_OP_FETCH_XOR:
        return T(U(__hip_atomic_fetch_xor(p, uint32_t(U(v)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)));
    case LMR_OP_STORE: case LMR_OP_PUT: case LMR_OP_SWAP:
        return T(U(__hip_atomic_exchange(p, uint32_t(U(v)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)));
    case LMR_OP_LOAD: case LMR_OP_GET:
        return T(U(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)));
    default: break;
    }
    uint32_t cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (true) {
        T old = T(U(cur)), nw, ret;
        uint32_t eb = 0;
        if (!op_math<T>(op, kind, old, v, cmp, eps, nw, ret, ok, eb)) {
            raise_err(err, eb);
            return old;
        }
        uint32_t nb = uint32_t(U(nw));
        if (nb == (cur & ((1u << (8 * sizeof(T))) - 1u))) return ret;
        uint32_t expected = cur;
        if (__hip_atomic_compare_exchange_strong(p, &expected, nb, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
            return ret;
        cur = expected;
    }
}

// RMW of an 8/16-bit element in global memory: CAS on the naturally aligned
// 32-bit word that contains it. Requires the shard allocation to be readable
// up to the next 4-byte boundary (hipMalloc/torch allocations are 256-B granular).
template <typename T>
__device__ __forceinline__ T rmw_subword_global(T* p, int op, int kind, T v, T cmp, T eps,
                                                uint8_t& ok, uint32_t* err) {
    using U = typename bits_of<T>::U;
    uintptr_t a = reinterpret_cast<uintptr_t>(p);
    uint32_t* wp = reinterpret_cast<uint32_t*>(a & ~uintptr_t(3));
    const unsigned sh = unsigned(a & 3) * 8;
    const uint32_t mask = uint32_t((1u << (8 * sizeof(T))) - 1u) << sh;
    uint32_t cur = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (true) {
        T old = T(U((cur & mask) >> sh)), nw, ret;
        uint32_t eb = 0;
        if (!op_math<T>(op, kind, old, v, cmp, eps, nw, ret, ok, eb)) {
            raise_err(err, eb);
            return old;
        }
        if (op_is_read(op)) return ret;
        uint32_t nb = (cur & ~mask) | (uint32_t(U(nw)) << sh);
        if (nb == cur) return ret;
        uint32_t expected = cur;
        if (__hip_atomic_compare_exchange_strong(wp, &expected, nb, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return ret;
        cur = expected;
    }
}

// Global-memory RMW of one element of any supported type.
template <typename T>
__device__ __forceinline__ T rmw_global(T* p, int op, int kind, T v, T cmp, T eps,
                                        uint8_t& ok, uint32_t* err) {
    if constexpr (sizeof(T) >= 4) return rmw_word<T>(p, op, kind, v, cmp, eps, ok, err);
    else return rmw_subword_global<T>(p, op, kind, v, cmp, eps, ok, err);
}

// LDS-tile RMW (tile words of type word_of<T>::W).
template <typename T>
__device__ __forceinline__ T rmw_lds(typename word_of<T>::W* p, int op, int kind, T v, T cmp,
                                     T eps, uint8_t& ok, uint32_t* err) {
    if constexpr (sizeof(T) >= 4) return rmw_word<T>(p, op, kind, v, cmp, eps, ok, err);
    else return rmw_widened<T>(p, op, kind, v, cmp, eps, ok, err);
}

// ---------------------------------------------------------------- wave key matching
// Match by key bits: `bits` ballots give every lane the mask of active lanes
// holding its key (keys < 2^bits); the lowest lane of each group adds the group's
// size to hist[key] (one LDS atomic instruction for all groups, distinct
// addresses) and broadcasts the returned base. Constant cost in the number of
// distinct keys, where wave_agg_rank loops once per key.
__device__ __forceinline__ uint64_t wave_key_mask(uint32_t key, bool active, int bits) {
    uint64_t m = __ballot(active);
    for (int b = 0; b < bits; b++) {
        const bool on = (key >> b) & 1u;
        const uint64_t bb = __ballot(on);
        m &= on ? bb : ~bb;
    }
    return m;
}
__device__ __forceinline__ uint32_t wave_match_rank(uint32_t* hist, uint32_t key, bool active, int bits) {
    const int lane = threadIdx.x & 63;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint64_t m = wave_key_mask(key, active, bits);
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (active && lane == leader) base = atomicAdd(&hist[key], uint32_t(__popcll(m)));
    base = __shfl(base, active ? leader : lane, 64);
    return base + uint32_t(__popcll(m & lt));
}
__device__ __forceinline__ void wave_match_count(uint32_t* hist, uint32_t key, bool active, int bits) {
    const int lane = threadIdx.x & 63;
    const uint64_t m = wave_key_mask(key, active, bits);
    if (active && lane == __ffsll((unsigned long long)m) - 1) atomicAdd(&hist[key], uint32_t(__popcll(m)));
}
__host__ __device__ inline int key_bits(uint32_t nkeys) {
    int b = 0;
    while ((1u << b) < nkeys) b++;
    return b;
}

// ---------------------------------------------------------------- XCD-grouped block ids
// Blocks b and b + 8 share an XCD (observed round-robin placement; speed only, never
// correctness). The swizzled id gives each XCD a contiguous range of ids, so work items
// with consecutive ids (runs appended to the same bins) are written through one L2 and
// the partial lines where one run meets the next merge there instead of being written
// back from two XCDs (count-free fine pass, C2: 1.55 -> 1.29 ms on one box).
__device__ __forceinline__ uint32_t xcd_block(bool on) {
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    return (on && (nb & 7) == 0) ? (b & 7) * (nb >> 3) + (b >> 3) : b;
}

// ---------------------------------------------------------------- LDS-staged write-out
// Write-out of one bucket-sorted LDS round: bucket c's hist[c] records, staged at
// LDS [base[c], base[c] + hist[c]), go to global [cursor[c], ...). Waves take
// whole buckets (several waves share a bucket when there are fewer buckets than
// waves) and their lanes stream contiguous records, so the bucket / offsets are
// wave-uniform LDS broadcasts and every store instruction covers one contiguous
// run: put(lds_pos, global_pos) per record.
template <typename F>
__device__ __forceinline__ void bucket_writeout(const uint32_t* hist, const uint32_t* base,
                                                const uint32_t* cursor, uint32_t nb, F&& put) {
    const uint32_t nw = blockDim.x >> 6, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t wpb = nb >= nw ? 1u : nw / nb;       // waves per bucket
    const uint32_t bstep = nw / wpb;
    for (uint32_t c = wave / wpb; c < nb; c += bstep) {
        const uint32_t len = hist[c], b = base[c], d = cursor[c];
        for (uint32_t i = (wave % wpb) * 64 + lane; i < len; i += wpb * 64) put(b + i, d + i);
    }
}

// ---------------------------------------------------------------- buffer loads
// A block-uniform stream [base, base + bytes) read through a buffer descriptor:
// 32-bit per-lane offsets instead of 64-bit pointers (the fine passes otherwise
// keep one hoisted 64-bit pointer per record of a round alive and spill them),
// and loads past `bytes` return 0. base / bytes must be the same on every lane:
// they go through readfirstlane so the compiler knows (no waterfall loops).
struct BufStream {
    __amdgpu_buffer_rsrc_t r;
    __device__ __forceinline__ BufStream(const void* base, uint32_t bytes) {
        const uint64_t b = reinterpret_cast<uint64_t>(base);
        const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(b));
        const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(b >> 32));
        const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
        r = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t(hi) << 32) | lo), 0, n, 0x00020000);
    }
    template <typename V>
    __device__ __forceinline__ V load(uint32_t byte_off) const {
        if constexpr (sizeof(V) == 1) return V(__builtin_amdgcn_raw_buffer_load_b8(r, byte_off, 0, 0));
        else if constexpr (sizeof(V) == 2) return V(__builtin_amdgcn_raw_buffer_load_b16(r, byte_off, 0, 0));
        else if constexpr (sizeof(V) == 4) return V(__builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
        else {
            auto x = __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, 0);
            return __builtin_bit_cast(V, x);
        }
    }
};

// ---------------------------------------------------------------- global address space
// A pointer read from memory (a device table, LDS) is a generic pointer: its loads and stores
// become flat_* instructions, which count on the LDS counter too, so the next LDS access waits
// for them (a write-out loop's stores, a prefetch's loads). For memory known to be global (device
// allocations, IPC-mapped peer memory) the cast makes them global_* instructions.
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* as_global(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}

// ---------------------------------------------------------------- index load
template <int IW> struct idx_t;
template <> struct idx_t<1> { using I = uint8_t; };
template <> struct idx_t<2> { using I = uint16_t; };
template <> struct idx_t<4> { using I = uint32_t; };
template <> struct idx_t<8> { using I = uint64_t; };

// wave64 inclusive scan; block-wide (1024 threads) exclusive scan of one value per thread
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

// block-wide exclusive scan of one value per thread (blockDim.x == 1024); returns the
// exclusive prefix, writes the block total to *total.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* total) {
    __shared__ uint32_t wsum[16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = wave_incl_scan(x);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    if (w == 0) {
        uint32_t v = lane < 16 ? wsum[lane] : 0;
        uint32_t vi = wave_incl_scan(v);
        if (lane < 16) wsum[lane] = vi - v;
        if (lane == 15) *total = vi;
    }
    __syncthreads();
    uint32_t r = inc - x + wsum[w];
    __syncthreads();
    return r;
}

}  // namespace lmr
