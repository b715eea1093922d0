// lmr_scan.hip — exclusive prefix sum over u32 counters (bin / pack offsets).
// Reduce-then-scan in three launches; each block covers kScanItems = 4096
// elements with 1024 threads x 4 items, wave64 shuffles for the intra-wave scan.
#include "lmr_internal.hpp"

namespace lmr {

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

__global__ __launch_bounds__(1024) void k_scan_reduce(const uint32_t* __restrict__ d, uint64_t m,
                                                      uint32_t* __restrict__ partials, const uint32_t* only_if) {
    if (only_if && *only_if == 0) return;
    const uint64_t base = uint64_t(blockIdx.x) * kScanItems + uint64_t(threadIdx.x) * 4;
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 4; i++)
        if (base + i < m) s += d[base + i];
    __shared__ uint32_t tot;
    block_excl_scan(s, &tot);
    if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

// single block: exclusive scan of the partials in place, grand total to *d_total
__global__ __launch_bounds__(1024) void k_scan_partials(uint32_t* __restrict__ partials,
                                                        uint64_t nb, uint32_t* __restrict__ d_total,
                                                        const uint32_t* only_if) {
    if (only_if && *only_if == 0) return;
    __shared__ uint32_t tot;
    uint32_t carry = 0;
    for (uint64_t b0 = 0; b0 < nb; b0 += 1024) {
        uint64_t i = b0 + threadIdx.x;
        uint32_t x = i < nb ? partials[i] : 0;
        uint32_t e = block_excl_scan(x, &tot);
        if (i < nb) partials[i] = carry + e;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0 && d_total) *d_total = carry;
}

__global__ __launch_bounds__(1024) void k_scan_apply(uint32_t* __restrict__ d, uint64_t m,
                                                     const uint32_t* __restrict__ partials, const uint32_t* only_if) {
    if (only_if && *only_if == 0) return;
    const uint64_t base = uint64_t(blockIdx.x) * kScanItems + uint64_t(threadIdx.x) * 4;
    uint32_t v[4];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        v[i] = (base + i < m) ? d[base + i] : 0;
        s += v[i];
    }
    __shared__ uint32_t tot;
    uint32_t e = block_excl_scan(s, &tot) + partials[blockIdx.x];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (base + i < m) d[base + i] = e;
        e += v[i];
    }
}

// one block for short arrays (tile starts, plans, coarse offsets): kScanItems elements per
// pass with the carry in registers, one launch instead of three
__global__ __launch_bounds__(1024) void k_scan_single(uint32_t* __restrict__ d, uint64_t m,
                                                      uint32_t* __restrict__ d_total, const uint32_t* only_if) {
    if (only_if && *only_if == 0) return;
    __shared__ uint32_t tot;
    uint32_t carry = 0;
    for (uint64_t b0 = 0; b0 < m; b0 += kScanItems) {
        const uint64_t base = b0 + uint64_t(threadIdx.x) * 4;
        uint32_t v[4];
        uint32_t sum = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            v[i] = (base + i < m) ? d[base + i] : 0;
            sum += v[i];
        }
        uint32_t e = carry + block_excl_scan(sum, &tot);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if (base + i < m) d[base + i] = e;
            e += v[i];
        }
        carry += tot;
    }
    if (threadIdx.x == 0 && d_total) *d_total = carry;
}

constexpr uint64_t kScanSingleMax = 16 * kScanItems;

hipError_t scan_exclusive_u32(uint32_t* d, uint64_t m, uint32_t* partials, uint32_t* d_total,
                              hipStream_t s, const uint32_t* only_if) {
    if (m == 0) {
        if (d_total) return hipMemsetAsync(d_total, 0, sizeof(uint32_t), s);
        return hipSuccess;
    }
    if (m <= kScanSingleMax) {
        hipLaunchKernelGGL(k_scan_single, dim3(1), dim3(1024), 0, s, d, m, d_total, only_if);
        return hipGetLastError();
    }
    uint64_t nb = (m + kScanItems - 1) / kScanItems;
    hipLaunchKernelGGL(k_scan_reduce, dim3(unsigned(nb)), dim3(1024), 0, s, d, m, partials, only_if);
    hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(1024), 0, s, partials, nb, d_total, only_if);
    hipLaunchKernelGGL(k_scan_apply, dim3(unsigned(nb)), dim3(1024), 0, s, d, m, partials, only_if);
    return hipGetLastError();
}

}  // namespace lmr
