// lmr_ordered.hip — LMR_STRATEGY_ORDERED: the records of one call applied per element in
// record (buffer) order, each element's records as one atomic block.
//
// The reference's generated apply AM walks its op buffer sequentially
// (impl/src/array_ops.rs:203-250: `for elem in idx_vals { slice[elem.index] op= elem.val }`,
// the same loop shape in the fetch / result bodies :1041-1079, :1226-1264), so a buffer that
// is one AM -- every 1-PE batch of fewer than 1000 records (one OpInput chunk,
// src/array/operations.rs:462-469, far below one AM's records, unsafe/operations.rs:679-681),
// or an lmr_apply_mvmi call handed exactly one AM's idx_vals -- ends in one deterministic
// state with deterministic fetch / Result values. AUTO takes this path below 1000 records.
//
// Per element the records are applied on a register copy of the element and published with
// one compare-and-swap (retried from the new value if another kernel changed the element
// meanwhile): one atomic block per element, like the MVSI path and the LocalLock kind's
// shard lock (array_ops.rs:557-560); any interleaving with concurrent calls is one the
// reference allows (its AMs apply concurrently, SeqCst per record).
//   n <= 1024 : k_order_small -- one workgroup; the first record of each element (no earlier
//               record names it: an LDS scan) walks the element's later records in order.
//   n > 1024  : keys (local index, out-of-bounds last) sorted stably with their record
//               positions (rocPRIM's onesweep radix sort), then k_order_chains: the first
//               record of every run of equal keys walks its run, i.e. the element's records in
//               input order.
// Larger calls go in pieces of the reserved capacity, one after another on the stream: every
// record of a piece is applied before any of the next, so each element still sees its records
// in input order. The sort buffers are reserved with the context (lmr_ctx_create: 2^16
// records; lmr_ctx_reserve: up to 2^22), so the ordered path never allocates.
#include "lmr_internal.hpp"
#include "lmr_device.hpp"
#include <rocprim/device/device_radix_sort.hpp>
#include <algorithm>

namespace lmr {

struct OrdBufs {
    void* p = nullptr;
    size_t bytes = 0;
    uint64_t recs = 0;        // records of one sorted piece
    size_t tmp = 0;           // rocPRIM temporary storage for a piece of `recs`
};

void ord_bufs_free(OrdBufs* b) {
    if (!b) return;
    if (b->p) (void)hipFree(b->p);
    delete b;
}

namespace {

template <typename T>
__device__ __forceinline__ T ord_val(const ApplyArgs& a, uint64_t k) {
    if (a.val) return *reinterpret_cast<const T*>(a.val + k * a.val_stride);
    return from_bits<T>(typename bits_of<T>::U(a.val_bits));
}

template <int IW>
__device__ __forceinline__ uint64_t ord_idx(const ApplyArgs& a, uint64_t k) {
    using I = typename idx_t<IW>::I;
    return uint64_t(*reinterpret_cast<const I*>(a.idx + k * a.idx_stride));
}

// Walk cursors c0, next(c0), next(next(c0)), ... (next returns ~0 at the end), applying record
// rec(c) of each to element p in that order on a register copy; publish with one CAS (the
// containing 32-bit word for 8/16-bit T), re-walking from the current value when the CAS loses.
// Results / Ok flags go to the records' own slots.
template <typename T, typename Next, typename Rec>
__device__ void apply_chain(T* p, const ApplyArgs& a, uint64_t c0, Next next, Rec rec) {
    using U = typename bits_of<T>::U;
    const T cmp = from_bits<T>(U(a.cmp_bits)), eps = from_bits<T>(U(a.eps_bits));
    const bool ret = a.ret != LMR_RET_NONE;
    auto walk = [&](T s, uint32_t& errs) -> T {
        for (uint64_t c = c0; c != ~uint64_t(0); c = next(c)) {
            const uint64_t k = rec(c);
            T v = ord_val<T>(a, k), nw, r;
            uint8_t ok = 0;
            uint32_t eb = 0;
            if (op_math<T>(a.op, a.kind, s, v, cmp, eps, nw, r, ok, eb)) s = nw;
            else errs |= eb;
            if (ret) reinterpret_cast<T*>(a.results)[k] = r;
            if (a.ret == LMR_RET_RESULT) a.ok[k] = ok;
        }
        return s;
    };
    if constexpr (sizeof(T) >= 4) {
        U cur = __hip_atomic_load(reinterpret_cast<U*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (true) {
            uint32_t errs = 0;
            const T s = walk(from_bits<T>(cur), errs);
            U expected = cur;
            if (to_bits(s) == cur ||
                __hip_atomic_compare_exchange_strong(reinterpret_cast<U*>(p), &expected, to_bits(s), __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                if (errs) raise_err(a.err, errs);
                return;
            }
            cur = expected;
        }
    } else {
        const uintptr_t ad = reinterpret_cast<uintptr_t>(p);
        uint32_t* wp = reinterpret_cast<uint32_t*>(ad & ~uintptr_t(3));
        const unsigned sh = unsigned(ad & 3) * 8;
        const uint32_t mask = uint32_t((1u << (8 * sizeof(T))) - 1u) << sh;
        uint32_t cur = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (true) {
            uint32_t errs = 0;
            const T s = walk(T(U((cur & mask) >> sh)), errs);
            const uint32_t nb = (cur & ~mask) | (uint32_t(U(s)) << sh);
            uint32_t expected = cur;
            if (nb == cur || __hip_atomic_compare_exchange_strong(wp, &expected, nb, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT)) {
                if (errs) raise_err(a.err, errs);
                return;
            }
            cur = expected;
        }
    }
}

constexpr uint32_t kSmall = 1024;

template <typename T, int IW>
__global__ __launch_bounds__(1024) void k_order_small(ApplyArgs a) {
    __shared__ uint64_t sidx[kSmall];
    const uint32_t n = uint32_t(a.n);
    const uint32_t k = threadIdx.x;
    if (k < n) sidx[k] = ord_idx<IW>(a, k);
    __syncthreads();
    if (k >= n) return;
    const uint64_t e = sidx[k];
    if (e >= a.shard_len) {                       // skipped, as on every other path
        raise_err(a.err, LMR_ERRBIT_OOB);
        return;
    }
    for (uint32_t j = 0; j < k; j++)
        if (sidx[j] == e) return;                 // an earlier record leads this element
    apply_chain<T>(
        reinterpret_cast<T*>(a.shard) + e, a, k,
        [&](uint64_t c) -> uint64_t {
            for (uint32_t j = uint32_t(c) + 1; j < n; j++)
                if (sidx[j] == e) return j;
            return ~uint64_t(0);
        },
        [](uint64_t c) { return c; });
}

template <int IW>
__global__ void k_order_keys(ApplyArgs a, uint64_t* keys, uint32_t* pos) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < a.n; k += stride) {
        uint64_t e = ord_idx<IW>(a, k);
        if (e >= a.shard_len) {
            raise_err(a.err, LMR_ERRBIT_OOB);
            e = a.shard_len;                      // sorts after every valid key; skipped
        }
        keys[k] = e;
        pos[k] = uint32_t(k);
    }
}

template <typename T>
__global__ void k_order_chains(ApplyArgs a, const uint64_t* keys, const uint32_t* pos) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < a.n; t += stride) {
        const uint64_t e = keys[t];
        if (e >= a.shard_len || (t > 0 && keys[t - 1] == e)) continue;
        // the run of e in sorted order holds its records in input order (stable sort): walk it by
        // sorted slot, applying each slot's record
        const uint64_t n = a.n;
        apply_chain<T>(
            reinterpret_cast<T*>(a.shard) + e, a, t,
            [&](uint64_t c) -> uint64_t { return (c + 1 < n && keys[c + 1] == e) ? c + 1 : ~uint64_t(0); },
            [&](uint64_t c) -> uint64_t { return pos[c]; });
    }
}

template <typename F>
hipError_t ord_dtype(int dtype, F&& f) {
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
hipError_t ord_iw(int iw, F&& f) {
    switch (iw) {
    case 1: return f(std::integral_constant<int, 1>{});
    case 2: return f(std::integral_constant<int, 2>{});
    case 4: return f(std::integral_constant<int, 4>{});
    case 8: return f(std::integral_constant<int, 8>{});
    default: return hipErrorInvalidValue;
    }
}

size_t al256(size_t b) { return (b + 255) & ~size_t(255); }

hipError_t sort_storage(uint64_t n, int bits, size_t& tmp) {
    tmp = 0;
    return rocprim::radix_sort_pairs(nullptr, tmp, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (const uint32_t*)nullptr, (uint32_t*)nullptr, size_t(n), 0u, unsigned(bits),
                                     hipStream_t(0));
}

size_t piece_bytes(uint64_t recs, size_t tmp) { return 2 * al256(recs * 8) + 2 * al256(recs * 4) + al256(tmp); }

}  // namespace

hipError_t ord_reserve(lmr_ctx* ctx, uint64_t recs) {
    recs = std::min<uint64_t>(std::max<uint64_t>(recs, kOrderedMinPiece), kOrderedMaxPiece);
    if (!ctx->ord) ctx->ord = new OrdBufs();
    OrdBufs* B = ctx->ord;
    if (B->recs >= recs) return hipSuccess;
    size_t tmp = 0;
    hipError_t e = sort_storage(recs, 64, tmp);          // the widest key range: covers every shard
    if (e != hipSuccess) return e;
    void* p = nullptr;
    if ((e = hipMalloc(&p, piece_bytes(recs, tmp))) != hipSuccess) return e;
    if (B->p)                                            // (outside the hot path: lmr_ctx_reserve, whose
        (void)hipFree(B->p);                             //  caller has completed the context's work)
    B->p = p;
    B->bytes = piece_bytes(recs, tmp);
    B->recs = recs;
    B->tmp = tmp;
    return hipSuccess;
}

namespace {

hipError_t apply_ordered_piece(const OrdBufs* B, int dtype, int iw, const ApplyArgs& a, hipStream_t s) {
    if (a.n <= kSmall) {
        return ord_dtype(dtype, [&](auto tag) {
            using T = decltype(tag);
            return ord_iw(iw, [&](auto w) {
                constexpr int IW = decltype(w)::value;
                hipLaunchKernelGGL((k_order_small<T, IW>), dim3(1), dim3(kSmall), 0, s, a);
                return hipGetLastError();
            });
        });
    }
    // sort keys = local index (bits up to the shard length), values = record positions
    const uint64_t n = a.n;
    int bits = 1;
    while (bits < 64 && (a.shard_len >> bits) != 0) bits++;
    size_t tmp = 0;
    hipError_t e = sort_storage(n, bits, tmp);
    if (e != hipSuccess) return e;
    if (tmp > B->tmp) return hipErrorInvalidValue;       // (never: storage grows with n and bits)
    uint8_t* q = static_cast<uint8_t*>(B->p);
    uint64_t* k_in = reinterpret_cast<uint64_t*>(q);   q += al256(B->recs * 8);
    uint64_t* k_out = reinterpret_cast<uint64_t*>(q);  q += al256(B->recs * 8);
    uint32_t* p_in = reinterpret_cast<uint32_t*>(q);   q += al256(B->recs * 4);
    uint32_t* p_out = reinterpret_cast<uint32_t*>(q);  q += al256(B->recs * 4);
    void* t = q;
    const unsigned grid = unsigned(std::min<uint64_t>((n + 255) / 256, 4096));
    e = ord_iw(iw, [&](auto w) {
        constexpr int IW = decltype(w)::value;
        hipLaunchKernelGGL((k_order_keys<IW>), dim3(grid), dim3(256), 0, s, a, k_in, p_in);
        return hipGetLastError();
    });
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_pairs(t, tmp, k_in, k_out, p_in, p_out, size_t(n), 0u, unsigned(bits), s);
    if (e != hipSuccess) return e;
    return ord_dtype(dtype, [&](auto tag) {
        using T = decltype(tag);
        hipLaunchKernelGGL((k_order_chains<T>), dim3(grid), dim3(256), 0, s, a, k_out, p_out);
        return hipGetLastError();
    });
}

}  // namespace

hipError_t launch_apply_ordered(lmr_ctx* ctx, int dtype, int iw, const ApplyArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const OrdBufs* B = ctx->ord;
    if (!B || B->recs == 0) return hipErrorNotInitialized;
    ProfScope ps(a.prof, LMR_STAGE_ORDERED, s, a.n);
    const int eb = dtype_bytes(dtype);
    for (uint64_t p0 = 0; p0 < a.n; p0 += B->recs) {
        ApplyArgs b = a;
        b.n = std::min<uint64_t>(a.n - p0, B->recs);
        b.idx = a.idx + p0 * a.idx_stride;
        if (a.val) b.val = a.val + p0 * a.val_stride;
        if (a.results) b.results = static_cast<uint8_t*>(a.results) + p0 * uint64_t(eb);
        if (a.ok) b.ok = a.ok + p0;
        const hipError_t e = apply_ordered_piece(B, dtype, iw, b, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace lmr
