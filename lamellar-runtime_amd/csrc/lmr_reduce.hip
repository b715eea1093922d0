// lmr_reduce.hip — local part of the array reductions (sum / prod / max / min).
//
// Restates the per-PE step of the reference's reduction AMs
// (impl/src/array_reduce.rs:82-88: `local_data().iter().reduce(op)`, with the
// ops of :283-319: `acc + val`, `acc * val`, `if a > b {a} else {b}`,
// `if a < b {a} else {b}`; dispatched from UnsafeArray::reduce / sum / prod /
// max / min, src/array/unsafe.rs:1414-1557). The cross-PE tree (:90-107) is
// combined on the host from every PE's (has, value) pair.
//
// Integer sum / prod wrap (release-mode Rust arithmetic). The device folds in a
// tree order (per-thread strided fold -> wave shuffles -> block -> final block):
// bit-exact for integers and for max / min of non-NaN values; a float sum or
// product differs from the sequential fold by rounding only.
#include "lmr_internal.hpp"
#include "lmr_device.hpp"

namespace lmr {

template <typename T, int OP>
__device__ __forceinline__ T red_op(T a, T b) {
    using U = typename bits_of<T>::U;
    if constexpr (OP == LMR_REDUCE_SUM) {
        if constexpr (is_flt<T>::v) return a + b; else return T(U(U(a) + U(b)));
    } else if constexpr (OP == LMR_REDUCE_PROD) {
        if constexpr (is_flt<T>::v) return a * b; else return T(U(U(a) * U(b)));
    } else if constexpr (OP == LMR_REDUCE_MAX) {
        return a > b ? a : b;
    } else {
        return a < b ? a : b;
    }
}

// (value, has) pair combine: an empty side is the identity, as None is in the
// reference's tree (:97-103).
template <typename T, int OP>
__device__ __forceinline__ void red_pair(T& v, bool& h, T v2, bool h2) {
    if (h2) {
        v = h ? red_op<T, OP>(v, v2) : v2;
        h = true;
    }
}

template <typename T>
__device__ __forceinline__ T shfl_down_t(T v, int d) {
    using U = typename bits_of<T>::U;
    if constexpr (sizeof(T) == 8) {
        uint64_t u = __builtin_bit_cast(uint64_t, v);
        uint32_t lo = __shfl_down(uint32_t(u), d, 64), hi = __shfl_down(uint32_t(u >> 32), d, 64);
        return __builtin_bit_cast(T, (uint64_t(hi) << 32) | lo);
    } else if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, __shfl_down(__builtin_bit_cast(uint32_t, v), d, 64));
    } else {
        return T(U(__shfl_down(uint32_t(U(v)), d, 64)));
    }
}

// block-wide (v, h) reduction in left-to-right lane / wave order; result in thread 0
template <typename T, int OP>
__device__ __forceinline__ void block_reduce(T& v, bool& h) {
    __shared__ T sv[16];
    __shared__ uint8_t sh[16];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T v2 = shfl_down_t(v, d);
        bool h2 = __shfl_down(int(h), d, 64) != 0;
        if ((threadIdx.x & 63) + d < 64) red_pair<T, OP>(v, h, v2, h2);
    }
    const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    if ((threadIdx.x & 63) == 0) { sv[w] = v; sh[w] = h; }
    __syncthreads();
    if (threadIdx.x == 0) {
        v = sv[0]; h = sh[0] != 0;
        for (int i = 1; i < nw; i++) red_pair<T, OP>(v, h, sv[i], sh[i] != 0);
    }
}

template <typename T, int OP>
__global__ __launch_bounds__(1024) void k_reduce_partial(const T* __restrict__ x, uint64_t n, uint64_t chunk,
                                                         T* part, uint8_t* part_has) {
    const uint64_t lo = uint64_t(blockIdx.x) * chunk;
    const uint64_t hi = min(lo + chunk, n);
    T v{};
    bool h = false;
    for (uint64_t k = lo + threadIdx.x; k < hi; k += blockDim.x) red_pair<T, OP>(v, h, x[k], true);
    block_reduce<T, OP>(v, h);
    if (threadIdx.x == 0) { part[blockIdx.x] = v; part_has[blockIdx.x] = h; }
}

template <typename T, int OP>
__global__ __launch_bounds__(1024) void k_reduce_final(const T* part, const uint8_t* part_has, uint32_t m,
                                                       uint64_t* out, uint8_t* has) {
    T v{};
    bool h = false;
    // each thread folds a contiguous run of partials so the order stays left to right
    const uint32_t per = (m + blockDim.x - 1) / blockDim.x;
    for (uint32_t i = threadIdx.x * per; i < min(m, (threadIdx.x + 1) * per); i++)
        red_pair<T, OP>(v, h, part[i], part_has[i] != 0);
    block_reduce<T, OP>(v, h);
    if (threadIdx.x == 0) {
        using U = typename bits_of<T>::U;
        *out = h ? uint64_t(U(to_bits(v))) : 0ull;
        if (has) *has = h;
    }
}

hipError_t launch_reduce(int dtype, int op, const void* x, uint64_t n, uint64_t* out, uint8_t* has,
                         void* part, uint8_t* part_has, hipStream_t s) {
    uint64_t G = (n + 65535) / 65536;
    if (G > uint64_t(kReduceBlocks)) G = kReduceBlocks;
    if (G < 1) G = 1;
    const uint64_t chunk = (n + G - 1) / G > 0 ? (n + G - 1) / G : 1;
    auto go = [&](auto tag, auto opc) -> hipError_t {
        using T = decltype(tag);
        constexpr int OP = decltype(opc)::value;
        hipLaunchKernelGGL((k_reduce_partial<T, OP>), dim3(unsigned(G)), dim3(1024), 0, s,
                           reinterpret_cast<const T*>(x), n, chunk, reinterpret_cast<T*>(part), part_has);
        hipLaunchKernelGGL((k_reduce_final<T, OP>), dim3(1), dim3(1024), 0, s,
                           reinterpret_cast<const T*>(part), part_has, uint32_t(G), out, has);
        return hipGetLastError();
    };
    auto by_op = [&](auto tag) -> hipError_t {
        using std::integral_constant;
        switch (op) {
        case LMR_REDUCE_SUM: return go(tag, integral_constant<int, LMR_REDUCE_SUM>{});
        case LMR_REDUCE_PROD: return go(tag, integral_constant<int, LMR_REDUCE_PROD>{});
        case LMR_REDUCE_MAX: return go(tag, integral_constant<int, LMR_REDUCE_MAX>{});
        case LMR_REDUCE_MIN: return go(tag, integral_constant<int, LMR_REDUCE_MIN>{});
        default: return hipErrorInvalidValue;
        }
    };
    switch (dtype) {
    case LMR_U8: return by_op(uint8_t{});
    case LMR_U16: return by_op(uint16_t{});
    case LMR_U32: return by_op(uint32_t{});
    case LMR_U64: return by_op(uint64_t{});
    case LMR_I8: return by_op(int8_t{});
    case LMR_I16: return by_op(int16_t{});
    case LMR_I32: return by_op(int32_t{});
    case LMR_I64: return by_op(int64_t{});
    case LMR_F32: return by_op(float{});
    case LMR_F64: return by_op(double{});
    default: return hipErrorInvalidValue;
    }
}

}  // namespace lmr
