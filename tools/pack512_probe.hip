// pack512_probe.hip — standalone probe (not product code) for the multi-GPU design question of
// can the sender's pack group records by (owner PE, owner coarse bucket) -- 8 PEs x 64
// buckets = 512 keys -- at a rate that lets the owner skip its coarse pass?
//
// One chunk of n records (u64 global index uniform over 8 PEs x 2^26 elements, Block layout; u64
// value) is packed in LDS rounds of R records ranked by key (LDS atomics, a block scan over the
// keys) and written as runs, output records = (u32 bucket-local index, u64 value) = 12 B:
//   private : every (key, producer block) owns a fixed segment of the key's region (capacity from
//             the uniform share + headroom, overflow counted): no global atomics at all
//   atomic  : each round reserves its run of every key with one atomicAdd on the key's fill counter
//             (the count-free pack's method, lmr_pack.hip k_pack_stage)
// with 512 keys and, for comparison, 8 keys (owner PE only: today's pack). Algorithmic bytes per
// record: 16 read + 12 written. Timed with HIP events over reps launches; prints GB/s.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/pack512_probe tools/pack512_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kT = 1024;
constexpr int kRpt = 8;
constexpr int kR = kRpt * kT;                 // 8K records per round: 14 B staged each = 112 KB
constexpr int kMaxKeys = 512;

struct P {
    const uint64_t* gidx;
    const uint64_t* val;
    uint64_t n, chunk;
    int pe_shift, bucket_shift, nb_log2;      // owner = g >> pe_shift; bucket = local >> bucket_shift
    int nkeys;
    uint32_t* out_idx;
    uint64_t* out_val;
    uint32_t cap;                             // private: records per (key, block) segment
    uint32_t G;
    uint32_t* fill;                           // atomic: per-key fill; private: overflow counter at [0]
    uint64_t region;                          // atomic: records per key region
};

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* tot) {
    __shared__ uint32_t ws[16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
    }
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    if (w == 0) {
        uint32_t v = lane < 16 ? ws[lane] : 0, vi = v;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const uint32_t y = __shfl_up(vi, d, 64);
            if (lane >= d) vi += y;
        }
        if (lane < 16) ws[lane] = vi - v;
        if (lane == 15) *tot = vi;
    }
    __syncthreads();
    const uint32_t r = inc - x + ws[w];
    __syncthreads();
    return r;
}

template <bool PRIVATE>
__global__ __launch_bounds__(1024) void k_pack(P p) {
    __shared__ uint32_t hist[kMaxKeys], base[kMaxKeys], cur[kMaxKeys], s_tot;
    __shared__ uint16_t s_k[kR];
    __shared__ uint32_t s_i[kR];
    __shared__ uint64_t s_v[kR];
    const uint32_t b = blockIdx.x;
    const uint64_t lo = uint64_t(b) * p.chunk, hi = min(lo + p.chunk, p.n);
    for (int x = threadIdx.x; x < p.nkeys; x += kT) cur[x] = 0;
    const uint32_t lmask = (1u << p.bucket_shift) - 1u;
    const uint64_t pmask = (uint64_t(1) << p.pe_shift) - 1;
    uint32_t ovf = 0;
    for (uint64_t r0 = lo; r0 < hi; r0 += kR) {
        for (int x = threadIdx.x; x < p.nkeys; x += kT) hist[x] = 0;
        __syncthreads();
        uint64_t g[kRpt], v[kRpt];
        uint32_t key[kRpt];
#pragma unroll
        for (int j = 0; j < kRpt; j++) {
            const uint64_t k = r0 + uint64_t(j) * kT + threadIdx.x;
            g[j] = k < hi ? p.gidx[k] : ~uint64_t(0);
            v[j] = k < hi ? p.val[k] : 0;
        }
#pragma unroll
        for (int j = 0; j < kRpt; j++) {
            if (g[j] == ~uint64_t(0)) { key[j] = ~0u; continue; }
            const uint32_t owner = uint32_t(g[j] >> p.pe_shift);
            const uint32_t local = uint32_t(g[j] & pmask);
            const uint32_t kk = p.nkeys == 8 ? owner : (owner << p.nb_log2) | (local >> p.bucket_shift);
            key[j] = (kk << 16) | atomicAdd(&hist[kk], 1u);
        }
        __syncthreads();
        const uint32_t h = threadIdx.x < p.nkeys ? hist[threadIdx.x] : 0u;
        const uint32_t e = block_excl_scan(h, &s_tot);
        if (threadIdx.x < p.nkeys) base[threadIdx.x] = e;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kRpt; j++) {
            if (key[j] == ~0u) continue;
            const uint32_t kk = key[j] >> 16;
            const uint32_t q = base[kk] + (key[j] & 0xFFFFu);
            const uint32_t local = uint32_t(g[j] & pmask);
            s_k[q] = uint16_t(kk);
            s_i[q] = p.nkeys == 8 ? local : (local & lmask);
            s_v[q] = v[j];
        }
        if (!PRIVATE) {                                   // one reservation per key and round
            if (threadIdx.x < p.nkeys && h) cur[threadIdx.x] = atomicAdd(&p.fill[threadIdx.x], h);
        }
        __syncthreads();
        const uint32_t tot = s_tot;
        for (uint32_t q = threadIdx.x; q < tot; q += kT) {
            const uint32_t kk = s_k[q];
            const uint32_t pos = cur[kk] + (q - base[kk]);
            uint64_t dst;
            if (PRIVATE) {
                if (pos >= p.cap) { ovf++; continue; }
                dst = (uint64_t(kk) * p.G + b) * p.cap + pos;
            } else {
                if (pos >= p.region) { ovf++; continue; }
                dst = uint64_t(kk) * p.region + pos;
            }
            p.out_idx[dst] = s_i[q];
            p.out_val[dst] = s_v[q];
        }
        __syncthreads();
        if (PRIVATE)
            for (int x = threadIdx.x; x < p.nkeys; x += kT) cur[x] += hist[x];
    }
    if (ovf) atomicAdd(&p.fill[kMaxKeys], ovf);
}

__global__ void k_init(uint64_t* g, uint64_t* v, uint64_t n, uint64_t range, uint64_t seed) {
    for (uint64_t k = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; k < n; k += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t z = (k + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        g[k] = z % range;
        v[k] = z;
    }
}

int main(int argc, char** argv) {
    const uint64_t n = uint64_t(1) << (argc > 1 ? atoi(argv[1]) : 26);
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const int pe_shift = 26, npes = 8, nb_log2 = 6, bucket_shift = pe_shift - nb_log2;
    uint64_t *g, *v;
    CK(hipMalloc(&g, n * 8));
    CK(hipMalloc(&v, n * 8));
    hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, g, v, n, uint64_t(npes) << pe_shift, 12345ull);
    const uint32_t G = 256;
    const uint64_t chunk = (n + G - 1) / G;
    uint32_t* fill;
    CK(hipMalloc(&fill, (kMaxKeys + 1) * 4));
    // output space: the larger of the two layouts
    const uint64_t slots = n * 2 + uint64_t(kMaxKeys) * G * 64;
    uint32_t* oi;
    uint64_t* ov;
    CK(hipMalloc(&oi, slots * 4));
    CK(hipMalloc(&ov, slots * 8));
    hipEvent_t a, z;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&z));
    for (int nkeys : {8, 512}) {
        for (int priv = 0; priv < 2; priv++) {
            P p{};
            p.gidx = g; p.val = v; p.n = n; p.chunk = chunk; p.pe_shift = pe_shift; p.bucket_shift = bucket_shift;
            p.nb_log2 = nb_log2; p.nkeys = nkeys; p.out_idx = oi; p.out_val = ov; p.G = G; p.fill = fill;
            const double mean = double(n) / nkeys / G;
            p.cap = uint32_t(mean * 1.125 + 64);
            p.region = uint64_t(double(n) / nkeys * 1.125 + 4096);
            float best = 1e30f, tot = 0;
            for (int r = 0; r < reps + 2; r++) {
                CK(hipMemset(fill, 0, (kMaxKeys + 1) * 4));
                CK(hipEventRecord(a));
                if (priv) hipLaunchKernelGGL(k_pack<true>, dim3(G), dim3(kT), 0, 0, p);
                else hipLaunchKernelGGL(k_pack<false>, dim3(G), dim3(kT), 0, 0, p);
                CK(hipEventRecord(z));
                CK(hipEventSynchronize(z));
                float ms;
                CK(hipEventElapsedTime(&ms, a, z));
                if (r >= 2) { best = ms < best ? ms : best; tot += ms; }
            }
            uint32_t ov_cnt = 0;
            CK(hipMemcpy(&ov_cnt, fill + kMaxKeys, 4, hipMemcpyDeviceToHost));
            const double avg = tot / reps;
            printf("keys %3d %-8s n 2^%d: avg %.3f ms best %.3f ms = %.2f TB/s (28 B/record), overflow %u\n", nkeys,
                   priv ? "private" : "atomic", __builtin_ctzll(n), avg, best, 28.0 * n / (avg * 1e-3) / 1e12, ov_cnt);
        }
    }
    return 0;
}
