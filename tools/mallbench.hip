// mallbench.hip — does a write-then-read ring that fits the 256 MiB Infinity
// Cache (MALL) stay on-die?  Question behind it: if the fine partition's output
// for a group of coarse buckets is re-read by the tile apply right after it is
// written, are those 2 x 10 B/op served by the MALL instead of HBM?
//   ring  S : repeat { write S bytes; read S bytes }           (2 S moved)
//   feed  S : repeat { copy S bytes from a 4 GiB HBM stream into the ring;
//                      read the ring }                           (3 S moved)
// build: hipcc -O3 --offload-arch=gfx950 tools/mallbench.hip -o tools/mallbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <algorithm>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_write(uint4* __restrict__ b, size_t n, uint32_t salt) {
    size_t s = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += s)
        b[i] = make_uint4(uint32_t(i) ^ salt, salt, uint32_t(i >> 32), 1u);
}
__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ a, size_t n, uint32_t* out) {
    size_t s = size_t(gridDim.x) * blockDim.x;
    uint32_t acc = 0;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += s) {
        uint4 x = a[i];
        acc ^= x.x ^ x.y ^ x.z ^ x.w;
    }
    if (acc == 0x12345u) out[0] = acc;
}
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
    size_t s = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += s) b[i] = a[i];
}

int main() {
    const size_t big = size_t(4) << 30;
    void *src, *ring;
    uint32_t* sink;
    CHECK(hipMalloc(&src, big));
    CHECK(hipMalloc(&ring, big));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(src, 1, big));
    CHECK(hipMemset(ring, 0, big));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int grid = 8192;
    const size_t MB = size_t(1) << 20;
    for (size_t S : {32 * MB, 64 * MB, 128 * MB, 160 * MB, 192 * MB, 256 * MB, 512 * MB, 2048 * MB}) {
        const size_t n = S / 16;
        const int reps = int(std::max<size_t>(4, (8192 * MB) / S / 4));
        for (int w = 0; w < 2; w++) {
            hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, (uint4*)ring, n, uint32_t(w));
            hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (const uint4*)ring, n, sink);
        }
        CHECK(hipEventRecord(e0));
        for (int r = 0; r < reps; r++) {
            hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, (uint4*)ring, n, uint32_t(r));
            hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (const uint4*)ring, n, sink);
        }
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double t_ring = ms / reps;
        size_t off = 0;
        auto feed = [&]() {
            if (off + S > big) off = 0;
            hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (const uint4*)((uint8_t*)src + off), (uint4*)ring, n);
            hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (const uint4*)ring, n, sink);
            off += S;
        };
        for (int w = 0; w < 2; w++) feed();
        CHECK(hipEventRecord(e0));
        for (int r = 0; r < reps; r++) feed();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double t_feed = ms / reps;
        printf("S %5zu MB  ring(write+read) %7.3f ms %6.2f TB/s   feed(copy-in+read) %7.3f ms %6.2f TB/s\n",
               S / MB, t_ring, 2.0 * S / (t_ring * 1e-3) / 1e12, t_feed, 3.0 * S / (t_feed * 1e-3) / 1e12);
    }
    return 0;
}
