// l2atomic.hip — can device-scope atomics on an L2-resident shard slice replace the fine
// partition pass + the LDS tile sweep of C2?
//
//   A: pure atomics (indices hashed in registers), every XCD on its own region of R bytes
//      (R = 256 KiB ... 64 MiB) vs one region over the whole 512 MiB shard.
//   B: the apply after a 256-way coarse partition: bucket b (2^18 u64 elements, 2 MiB) holds
//      2^20 records (u32 bucket-local index, u64 value, structure of arrays); XCD x walks buckets
//      x, x+8, ... in order through a per-XCD work queue of 4096-record chunks, so each XCD's
//      L2 holds the slice of the bucket it is on. Atomics with and without a return value.
// build: hipcc -O3 --offload-arch=gfx950 tools/l2atomic.hip -o tools/l2atomic
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7; }

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

// A: `per` atomics per thread into region xcc (per_xcd != 0) or the whole array
__global__ __launch_bounds__(256) void k_hash_atomics(uint64_t* a, uint64_t region_elems, int per_xcd, int per) {
    const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t base = per_xcd ? uint64_t(xcc_id()) * region_elems : 0;
    for (int i = 0; i < per; i++) {
        const uint64_t e = mix(tid * 1315423911ull + i) & (region_elems - 1);
        __hip_atomic_fetch_add(a + base + e, uint64_t(1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

constexpr uint32_t kChunk = 4096;

// B: per-XCD queue over its buckets' chunks, in bucket order
template <bool RET>
__global__ __launch_bounds__(256) void k_bucket_apply(uint64_t* shard, const uint32_t* idx, const uint64_t* val,
                                                       uint32_t nbuckets, uint32_t recs_per_bucket,
                                                       uint32_t elems_per_bucket, uint32_t* queue, uint64_t* sink) {
    const uint32_t x = xcc_id();
    const uint32_t my_buckets = (nbuckets - x + 7) / 8;
    const uint32_t chunks_per_bucket = recs_per_bucket / kChunk;
    const uint32_t total = my_buckets * chunks_per_bucket;
    __shared__ uint32_t s_item;
    uint64_t acc = 0;
    while (true) {
        if (threadIdx.x == 0) s_item = atomicAdd(&queue[x * 32], 1u);
        __syncthreads();
        const uint32_t it = s_item;
        __syncthreads();
        if (it >= total) break;
        const uint32_t b = x + 8 * (it / chunks_per_bucket);
        const uint64_t r0 = uint64_t(b) * recs_per_bucket + uint64_t(it % chunks_per_bucket) * kChunk;
        uint64_t* sb = shard + uint64_t(b) * elems_per_bucket;
#pragma unroll 4
        for (uint32_t k = threadIdx.x; k < kChunk; k += 256) {
            const uint32_t l = idx[r0 + k];
            const uint64_t v = val[r0 + k];
            if (RET) acc += __hip_atomic_fetch_add(sb + l, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else __hip_atomic_fetch_add(sb + l, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (RET && acc == 0x1234567ull) sink[0] = acc;
}

// B': the same records with the bucket loop in plain grid order (no XCD affinity)
__global__ __launch_bounds__(256) void k_flat_apply(uint64_t* shard, const uint32_t* idx, const uint64_t* val,
                                                     uint64_t n, uint32_t recs_per_bucket, uint32_t elems_per_bucket) {
    const uint64_t s = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < n; r += s) {
        const uint64_t b = r / recs_per_bucket;
        __hip_atomic_fetch_add(shard + b * elems_per_bucket + idx[r], val[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void k_fill(uint32_t* idx, uint64_t* val, uint64_t n, uint32_t elems_per_bucket) {
    const uint64_t s = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < n; r += s) {
        const uint64_t h = mix(r + 77);
        idx[r] = uint32_t(h % elems_per_bucket);
        val[r] = h >> 20;
    }
}

int main() {
    const uint64_t shard_elems = uint64_t(1) << 26;      // 512 MiB of u64
    uint64_t* a;
    CHECK(hipMalloc(&a, shard_elems * 8));
    CHECK(hipMemset(a, 0, shard_elems * 8));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    printf("CUs %d\n", cus);
    auto timeit = [&](auto launch, int reps) -> float {
        launch();
        hipEventRecord(e0);
        for (int r = 0; r < reps; r++) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        return ms / reps;
    };
    // ---- A
    const unsigned grid = unsigned(cus) * 8;
    const int per = 64;
    const double nat = double(grid) * 256 * per;
    for (uint64_t rb : {uint64_t(256) << 10, uint64_t(1) << 20, uint64_t(2) << 20, uint64_t(4) << 20, uint64_t(8) << 20,
                        uint64_t(64) << 20}) {
        const uint64_t re = rb / 8;
        float ms = timeit([&] { hipLaunchKernelGGL(k_hash_atomics, dim3(grid), dim3(256), 0, 0, a, re, 1, per); }, 5);
        printf("A per-XCD region %6llu KiB : %8.3f ms  %7.1f G atomics/s\n", (unsigned long long)(rb >> 10), ms,
               nat / ms / 1e6);
    }
    {
        float ms = timeit([&] { hipLaunchKernelGGL(k_hash_atomics, dim3(grid), dim3(256), 0, 0, a, shard_elems, 0, per); }, 5);
        printf("A whole 512 MiB shard       : %8.3f ms  %7.1f G atomics/s\n", ms, nat / ms / 1e6);
    }
    // ---- B
    const uint64_t n = uint64_t(1) << 28;
    uint32_t* idx;
    uint64_t* val;
    uint32_t* queue;
    uint64_t* sink;
    CHECK(hipMalloc(&idx, n * 4));
    CHECK(hipMalloc(&val, n * 8));
    CHECK(hipMalloc(&queue, 8 * 32 * 4));
    CHECK(hipMalloc(&sink, 64));
    for (uint32_t nb : {64u, 128u, 256u, 512u, 1024u}) {
        const uint32_t epb = uint32_t(shard_elems / nb), rpb = uint32_t(n / nb);
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, idx, val, n, epb);
        CHECK(hipDeviceSynchronize());
        for (int ret = 0; ret < 2; ret++) {
            for (unsigned g : {unsigned(cus) * 4, unsigned(cus) * 8}) {
                float ms = timeit([&] {
                    hipMemsetAsync(queue, 0, 8 * 32 * 4, 0);
                    if (ret) hipLaunchKernelGGL((k_bucket_apply<true>), dim3(g), dim3(256), 0, 0, a, idx, val, nb, rpb, epb, queue, sink);
                    else hipLaunchKernelGGL((k_bucket_apply<false>), dim3(g), dim3(256), 0, 0, a, idx, val, nb, rpb, epb, queue, sink);
                }, 5);
                printf("B %4u buckets (%5u KiB) ret=%d grid=%5u : %8.3f ms  %7.1f G rec/s  %6.0f GB/s records\n", nb,
                       epb * 8 / 1024, ret, g, ms, double(n) / ms / 1e6, double(n) * 12 / ms / 1e6);
            }
        }
        float ms = timeit([&] { hipLaunchKernelGGL(k_flat_apply, dim3(unsigned(cus) * 8), dim3(256), 0, 0, a, idx, val, n, rpb, epb); }, 3);
        printf("B' %4u buckets flat order         : %8.3f ms  %7.1f G rec/s\n", nb, ms, double(n) / ms / 1e6);
    }
    return 0;
}
