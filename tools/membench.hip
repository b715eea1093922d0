// membench.hip — HBM calibration on the GPU box: copy / read / write streams at
// 4-, 8- and 16-byte lanes, the measured ceiling beside the 8 TB/s spec.
// build: hipcc -O3 --offload-arch=gfx950 tools/membench.hip -o build/membench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <typename V>
__global__ __launch_bounds__(256) void k_copy(const V* __restrict__ a, V* __restrict__ b, size_t n) {
    size_t s = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += s) b[i] = a[i];
}

template <typename V>
__global__ __launch_bounds__(256) void k_read(const V* __restrict__ a, size_t n, V* out) {
    size_t s = size_t(gridDim.x) * blockDim.x;
    V acc{};
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += s) acc ^= a[i];
    if (acc == V(0x12345)) out[0] = acc;
}

template <typename V>
__global__ __launch_bounds__(256) void k_write(V* __restrict__ b, size_t n) {
    size_t s = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += s) b[i] = V(i);
}

struct u4 { uint4 v; };

__global__ __launch_bounds__(256) void k_copy16(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
    size_t s = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += s) b[i] = a[i];
}
__global__ __launch_bounds__(256) void k_read16(const uint4* __restrict__ a, size_t n, uint4* out) {
    size_t s = size_t(gridDim.x) * blockDim.x;
    uint32_t acc = 0;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += s) { uint4 x = a[i]; acc ^= x.x ^ x.y ^ x.z ^ x.w; }
    if (acc == 0x12345u) out[0].x = acc;
}

int main() {
    const size_t bytes = size_t(2) << 30;   // 2 GiB per buffer (beyond the 256 MiB MALL)
    void *a, *b;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMemset(a, 1, bytes));
    CHECK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto time = [&](auto launch, double moved, const char* name) {
        for (int w = 0; w < 2; w++) launch();
        hipEventRecord(e0);
        const int reps = 10;
        for (int r = 0; r < reps; r++) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s %8.3f ms  %7.2f TB/s\n", name, ms / reps, moved / (ms / reps * 1e-3) / 1e12);
    };
    for (int grid : {2048, 8192, 32768}) {
        printf("grid %d x 256\n", grid);
        time([&] { hipLaunchKernelGGL(k_copy16, dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16); }, 2.0 * bytes, "copy 16B/lane");
        time([&] { hipLaunchKernelGGL(k_copy<uint64_t>, dim3(grid), dim3(256), 0, 0, (const uint64_t*)a, (uint64_t*)b, bytes / 8); }, 2.0 * bytes, "copy 8B/lane");
        time([&] { hipLaunchKernelGGL(k_copy<uint32_t>, dim3(grid), dim3(256), 0, 0, (const uint32_t*)a, (uint32_t*)b, bytes / 4); }, 2.0 * bytes, "copy 4B/lane");
        time([&] { hipLaunchKernelGGL(k_read16, dim3(grid), dim3(256), 0, 0, (const uint4*)a, bytes / 16, (uint4*)b); }, 1.0 * bytes, "read 16B/lane");
        time([&] { hipLaunchKernelGGL(k_read<uint64_t>, dim3(grid), dim3(256), 0, 0, (const uint64_t*)a, bytes / 8, (uint64_t*)b); }, 1.0 * bytes, "read 8B/lane");
        time([&] { hipLaunchKernelGGL(k_write<uint64_t>, dim3(grid), dim3(256), 0, 0, (uint64_t*)b, bytes / 8); }, 1.0 * bytes, "write 8B/lane");
    }
    return 0;
}
