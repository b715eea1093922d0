// lmr_scan.hip — exclusive prefix sum over u32 counters (bin / pack offsets).
// Up to 64K counters: one block walks the array with the carry in registers. Above:
// a single-pass scan with decoupled look-back, one launch: blocks take 4096-counter
// tiles in ticket order, publish their aggregate, and wave 0 of each block folds up
// to 64 predecessors' status words per step until it meets an inclusive prefix.
// The status words and counters live in the caller's scratch and are zero between
// calls: the last block to finish clears them, so no memset precedes a launch.
#include "lmr_internal.hpp"
#include "lmr_device.hpp"

namespace lmr {

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
constexpr uint64_t kStAgg = uint64_t(1) << 32, kStPrefix = uint64_t(2) << 32;

// scratch: [0] ticket, [1] blocks done, then nb u64 status words (flag << 32 | value)
__global__ __launch_bounds__(1024) void k_scan_lookback(uint32_t* __restrict__ d, uint64_t m,
                                                        uint32_t* __restrict__ scratch, uint32_t nb,
                                                        uint32_t* __restrict__ d_total, const uint32_t* only_if) {
    if (only_if && *only_if == 0) return;
    uint32_t* ctl = scratch;
    uint64_t* st = reinterpret_cast<uint64_t*>(scratch + 2);
    __shared__ uint32_t s_tile, s_excl, s_last, tot;
    if (threadIdx.x == 0) s_tile = atomicAdd(&ctl[0], 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    // a ticket past the last tile means the scratch was not zero at launch (two scans sharing
    // one context's scratch from different streams, which the C ABI rules out): write nothing
    // outside the scratch sized for this m
    if (tile >= nb) return;
    const uint64_t base = uint64_t(tile) * kScanItems + uint64_t(threadIdx.x) * 4;
    uint32_t v[4];
    uint32_t sum = 0;
    if (base + 4 <= m && (reinterpret_cast<uintptr_t>(d) & 15) == 0) {
        const uint4 q = *reinterpret_cast<const uint4*>(d + base);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = (base + i < m) ? d[base + i] : 0;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) sum += v[i];
    uint32_t e = block_excl_scan(sum, &tot);
    if (threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x;
        const uint32_t agg = tot;
        uint32_t excl = 0;
        if (tile == 0) {
            if (lane == 0) __hip_atomic_store(&st[0], kStPrefix | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(&st[tile], kStAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t top = int64_t(tile) - 1;              // the nearest predecessor not folded yet
            while (true) {
                const int64_t j = top - int64_t(lane);
                const uint64_t w = j >= 0 ? __hip_atomic_load(&st[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                          : kStPrefix;   // before tile 0: an empty prefix
                const uint32_t flag = uint32_t(w >> 32);
                const uint64_t pre = __ballot(flag == 2u);
                const uint64_t inv = __ballot(flag == 0u);
                const int p = pre ? __ffsll(static_cast<unsigned long long>(pre)) - 1 : 64;   // nearest prefix
                const uint64_t need = p >= 63 ? ~uint64_t(0) : ((uint64_t(2) << p) - 1);
                if (inv & need) {                          // a predecessor up to it has not published
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                uint32_t x = int(lane) <= p ? uint32_t(w) : 0u;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
                excl += x;
                if (pre) break;
                top -= 64;
            }
            if (lane == 0) __hip_atomic_store(&st[tile], kStPrefix | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_excl = excl;
    }
    __syncthreads();
    e += s_excl;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (base + i < m) d[base + i] = e;
        e += v[i];
    }
    if (tile == nb - 1 && threadIdx.x == 0 && d_total) *d_total = s_excl + tot;
    // the last block to finish (every look-back read done) leaves the scratch zeroed
    if (threadIdx.x == 0) s_last = atomicAdd(&ctl[1], 1u) == nb - 1;
    __syncthreads();
    if (s_last) {
        for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x)
            __hip_atomic_store(&st[j], uint64_t(0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (threadIdx.x == 0) {
            __hip_atomic_store(&ctl[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

uint64_t scan_scratch_words(uint64_t m) { return 4 + 2 * ((m + kScanItems - 1) / kScanItems); }

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
    const uint64_t nb = (m + kScanItems - 1) / kScanItems;
    hipLaunchKernelGGL(k_scan_lookback, dim3(unsigned(nb)), dim3(1024), 0, s, d, m, partials, uint32_t(nb),
                       d_total, only_if);
    return hipGetLastError();
}

}  // namespace lmr
