// One-level partition probe (C3 design question, round 5): is an LDS-staged NB-way partition of
// 2^26 (u64 index, f64 value) records into shard buckets, NB = 256..2048, fast enough to replace
// the coarse + fine passes, and its one-level inverse (olds back to input order) fast enough to
// replace the two gathers? Count-based slices: block g's records of bucket b are one contiguous
// run of bucket b's region across all of g's rounds; every round records its per-bucket counts
// (u16) so the inverse replays the same cursors.
//   scatter : read idx 8 + val 8, write lidx 2 + val 8 + qpos 2     = 28 B/record
//   inverse : read olds 8 + qpos 2, write 8                          = 18 B/record
// build: hipcc --offload-arch=gfx950 -O3 -o tools/onelevel_probe tools/onelevel_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <random>
#include <algorithm>
#include <cmath>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kT = 1024;

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}

__global__ void k_gen(uint64_t* idx, double* val, uint64_t n, uint64_t shard_len, int zipfish) {
    for (uint64_t k = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; k < n; k += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t h = mix(k * 0x9E3779B97F4A7C15ULL + 1);
        uint64_t r = h % shard_len;
        if (zipfish) {   // a skewed draw: 1/u-ish ranks, then scrambled over the shard
            const double u = double((h >> 11) & ((1ull << 40) - 1)) / double(1ull << 40) + 1e-12;
            uint64_t rank = uint64_t(1.0 / u) - 1;
            if (rank >= shard_len) rank = h % shard_len;
            r = mix(rank + 7) % shard_len;
        }
        idx[k] = r;
        val[k] = double(k & 1023);
    }
}

// per-(bucket, block) counts, bucket-major: cnt[b * G + g]
template <int NB>
__global__ __launch_bounds__(kT) void k_count(const uint64_t* idx, uint64_t n, uint64_t chunk, int shift, uint32_t* cnt) {
    __shared__ uint32_t h[NB];
    for (int b = threadIdx.x; b < NB; b += kT) h[b] = 0;
    __syncthreads();
    const uint64_t lo = blockIdx.x * chunk, hi = min(lo + chunk, n);
    for (uint64_t k = lo + threadIdx.x; k < hi; k += kT) atomicAdd(&h[idx[k] >> shift], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < NB; b += kT) cnt[uint64_t(b) * gridDim.x + blockIdx.x] = h[b];
}

// exclusive scan of m u32 in one block (probe only)
__global__ __launch_bounds__(kT) void k_scan1(uint32_t* a, uint32_t m) {
    __shared__ uint32_t s[kT];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < m; base += kT) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < m ? a[i] : 0u;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < kT; o <<= 1) {
            const uint32_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0u;
            __syncthreads();
            s[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < m) a[i] = carry + s[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == kT - 1) carry += s[kT - 1];
        __syncthreads();
    }
}

// block-wide exclusive scan of NB counters (NB <= 2048, 1024 threads)
template <int NB>
__device__ __forceinline__ void scan_nb(const uint32_t* in, uint32_t* out, uint32_t* tmp) {
    constexpr int PER = (NB + kT - 1) / kT;
    uint32_t v[PER], s = 0;
#pragma unroll
    for (int j = 0; j < PER; j++) {
        const int b = threadIdx.x * PER + j;
        v[j] = b < NB ? in[b] : 0u;
        s += v[j];
    }
    // wave scan then across the 16 waves
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) tmp[w] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t c = 0;
        for (int i = 0; i < kT / 64; i++) { const uint32_t t = tmp[i]; tmp[i] = c; c += t; }
    }
    __syncthreads();
    uint32_t e = tmp[w] + x - s;
#pragma unroll
    for (int j = 0; j < PER; j++) {
        const int b = threadIdx.x * PER + j;
        if (b < NB) out[b] = e;
        e += v[j];
    }
}

template <int NB, int RPT>
__global__ __launch_bounds__(kT) void k_scatter(const uint64_t* __restrict__ idx, const double* __restrict__ val,
                                                uint64_t n, uint64_t chunk, int shift, const uint32_t* __restrict__ off,
                                                uint16_t* __restrict__ out_l, double* __restrict__ out_v,
                                                uint16_t* __restrict__ qpos, uint16_t* __restrict__ rhist) {
    constexpr uint32_t R = RPT * kT;
    __shared__ uint32_t hist[NB], base[NB], cursor[NB], tmp[kT / 64];
    __shared__ uint16_t s_l[R], s_b[R];
    __shared__ double s_v[R];
    const uint32_t g = blockIdx.x, G = gridDim.x;
    for (int b = threadIdx.x; b < NB; b += kT) cursor[b] = off[uint64_t(b) * G + g];
    const uint64_t lo = g * chunk, hi = min(lo + chunk, n);
    const uint32_t lmask = (1u << shift) - 1u;
    uint64_t rid = (lo / R);
    for (uint64_t r0 = lo; r0 < hi; r0 += R, rid++) {
        for (int b = threadIdx.x; b < NB; b += kT) hist[b] = 0;
        __syncthreads();
        uint64_t ix[RPT];
        double vv[RPT];
        uint32_t rk[RPT];
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint64_t k = r0 + j * kT + threadIdx.x;
            ix[j] = k < hi ? idx[k] : 0;
            vv[j] = k < hi ? val[k] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint64_t k = r0 + j * kT + threadIdx.x;
            if (k < hi) rk[j] = atomicAdd(&hist[ix[j] >> shift], 1u);
        }
        __syncthreads();
        scan_nb<NB>(hist, base, tmp);
        __syncthreads();
        for (int b = threadIdx.x; b < NB; b += kT) rhist[rid * NB + b] = uint16_t(hist[b]);
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint64_t k = r0 + j * kT + threadIdx.x;
            if (k >= hi) continue;
            const uint32_t b = uint32_t(ix[j] >> shift);
            const uint32_t q = base[b] + rk[j];
            s_l[q] = uint16_t(ix[j] & lmask);
            s_b[q] = uint16_t(b);
            s_v[q] = vv[j];
            qpos[k] = uint16_t(q);
        }
        __syncthreads();
        const uint32_t tot = uint32_t(min(uint64_t(R), hi - r0));
        for (uint32_t q = threadIdx.x; q < tot; q += kT) {
            const uint32_t b = s_b[q];
            const uint32_t dst = cursor[b] + (q - base[b]);
            out_l[dst] = s_l[q];
            out_v[dst] = s_v[q];
        }
        __syncthreads();
        for (int b = threadIdx.x; b < NB; b += kT) cursor[b] += hist[b];
        __syncthreads();
    }
}

// variant: no values staged in LDS -- the round's staging order keeps each record's source
// position (u16), and the writeout gathers the value from global memory (the round's 8*R bytes of
// values, just read once in order to warm L2). 6 B of LDS per record instead of 12: rounds of 16K.
template <int NB, int RPT>
__global__ __launch_bounds__(kT) void k_scatter_src(const uint64_t* __restrict__ idx, const double* __restrict__ val,
                                                    uint64_t n, uint64_t chunk, int shift, const uint32_t* __restrict__ off,
                                                    uint16_t* __restrict__ out_l, double* __restrict__ out_v,
                                                    uint16_t* __restrict__ qpos, uint16_t* __restrict__ rhist, int warm) {
    constexpr uint32_t R = RPT * kT;
    __shared__ uint32_t hist[NB], base[NB], cursor[NB], tmp[kT / 64];
    __shared__ uint16_t s_l[R], s_b[R], s_src[R];
    const uint32_t g = blockIdx.x, G = gridDim.x;
    for (int b = threadIdx.x; b < NB; b += kT) cursor[b] = off[uint64_t(b) * G + g];
    const uint64_t lo = g * chunk, hi = min(lo + chunk, n);
    const uint32_t lmask = (1u << shift) - 1u;
    uint64_t rid = (lo / R);
    for (uint64_t r0 = lo; r0 < hi; r0 += R, rid++) {
        for (int b = threadIdx.x; b < NB; b += kT) hist[b] = 0;
        __syncthreads();
        uint64_t ix[RPT];
        uint32_t rk[RPT];
        double sink = 0.0;
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint64_t k = r0 + j * kT + threadIdx.x;
            ix[j] = k < hi ? idx[k] : 0;
            if (warm && k < hi) sink += val[k];          // coalesced: the round's values into L2
        }
        if (sink == 1.2345e300) out_v[0] = sink;        // keep the warm loads
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint64_t k = r0 + j * kT + threadIdx.x;
            if (k < hi) rk[j] = atomicAdd(&hist[ix[j] >> shift], 1u);
        }
        __syncthreads();
        scan_nb<NB>(hist, base, tmp);
        __syncthreads();
        for (int b = threadIdx.x; b < NB; b += kT) rhist[rid * NB + b] = uint16_t(hist[b]);
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const uint64_t k = r0 + j * kT + threadIdx.x;
            if (k >= hi) continue;
            const uint32_t b = uint32_t(ix[j] >> shift);
            const uint32_t q = base[b] + rk[j];
            s_l[q] = uint16_t(ix[j] & lmask);
            s_b[q] = uint16_t(b);
            s_src[q] = uint16_t(j * kT + threadIdx.x);
            qpos[k] = uint16_t(q);
        }
        __syncthreads();
        const uint32_t tot = uint32_t(min(uint64_t(R), hi - r0));
        for (uint32_t q = threadIdx.x; q < tot; q += kT) {
            const uint32_t b = s_b[q];
            const uint32_t dst = cursor[b] + (q - base[b]);
            out_l[dst] = s_l[q];
            out_v[dst] = val[r0 + s_src[q]];
        }
        __syncthreads();
        for (int b = threadIdx.x; b < NB; b += kT) cursor[b] += hist[b];
        __syncthreads();
    }
}

// inverse: the same blocks and rounds; each round's runs (per-bucket counts from rhist, cursors
// replayed) read into LDS in staging order, then dst[k] = s_v[qpos[k]]
template <int NB, int RPT>
__global__ __launch_bounds__(kT) void k_inverse(const double* __restrict__ olds, uint64_t n, uint64_t chunk,
                                                const uint32_t* __restrict__ off, const uint16_t* __restrict__ qpos,
                                                const uint16_t* __restrict__ rhist, double* __restrict__ dst) {
    constexpr uint32_t R = RPT * kT;
    __shared__ uint32_t hist[NB], base[NB], cursor[NB], tmp[kT / 64];
    __shared__ double s_v[R];
    const uint32_t g = blockIdx.x, G = gridDim.x;
    for (int b = threadIdx.x; b < NB; b += kT) cursor[b] = off[uint64_t(b) * G + g];
    const uint64_t lo = g * chunk, hi = min(lo + chunk, n);
    uint64_t rid = lo / R;
    for (uint64_t r0 = lo; r0 < hi; r0 += R, rid++) {
        for (int b = threadIdx.x; b < NB; b += kT) hist[b] = rhist[rid * NB + b];
        __syncthreads();
        scan_nb<NB>(hist, base, tmp);
        __syncthreads();
        const uint32_t tot = uint32_t(min(uint64_t(R), hi - r0));
        constexpr int U = 4;
        for (uint32_t x0 = threadIdx.x; x0 < tot; x0 += U * kT) {
            uint32_t sp[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t x = min(x0 + uint32_t(u) * kT, tot - 1);
                uint32_t lo_b = 0, hi_b = NB;
#pragma unroll
                for (int it = 0; (1 << it) < NB; it++) {
                    const uint32_t m = (lo_b + hi_b) >> 1;
                    if (base[m] <= x) lo_b = m; else hi_b = m;
                }
                sp[u] = cursor[lo_b] + (x - base[lo_b]);
            }
            double v[U];
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = olds[sp[u]];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t x = x0 + uint32_t(u) * kT;
                if (x < tot) s_v[x] = v[u];
            }
        }
        __syncthreads();
        for (uint64_t k = r0 + threadIdx.x; k < r0 + tot; k += kT) dst[k] = s_v[qpos[k]];
        __syncthreads();
        for (int b = threadIdx.x; b < NB; b += kT) cursor[b] += hist[b];
        __syncthreads();
    }
}

// C3's indices as bench.py draws them: Zipf(0.99) ranks over the shard, mapped through a fixed
// random permutation
static std::vector<uint64_t> zipf_host(uint64_t n, uint64_t shard) {
    std::vector<double> cdf(shard);
    double c = 0;
    for (uint64_t r = 0; r < shard; r++) { c += std::pow(double(r + 1), -0.99); cdf[r] = c; }
    for (auto& x : cdf) x /= c;
    std::vector<uint64_t> perm(shard);
    for (uint64_t i = 0; i < shard; i++) perm[i] = i;
    std::mt19937_64 g(0xC3);
    std::shuffle(perm.begin(), perm.end(), g);
    std::vector<uint64_t> out(n);
    std::uniform_real_distribution<double> u(0.0, 1.0);
    for (uint64_t k = 0; k < n; k++) {
        uint64_t r = std::lower_bound(cdf.begin(), cdf.end(), u(g)) - cdf.begin();
        out[k] = perm[std::min(r, shard - 1)];
    }
    return out;
}
static std::vector<uint64_t> g_zipf;

template <int NB, int RPT, int SRC = 0>
void run(int zipfish, int G) {
    constexpr int src = SRC;
    const uint64_t n = 1ull << 26, shard = 1ull << 24;
    int shift = 0;
    while ((shard >> shift) > NB) shift++;
    constexpr uint32_t R = RPT * kT;
    const uint64_t chunk = ((n + G - 1) / G + R - 1) / R * R;
    const uint64_t rounds = (n + R - 1) / R + G;
    uint64_t* idx; double *val, *ov, *back; uint16_t *ol, *qp, *rh; uint32_t* off;
    CK(hipMalloc(&idx, n * 8)); CK(hipMalloc(&val, n * 8)); CK(hipMalloc(&ov, n * 8)); CK(hipMalloc(&back, n * 8));
    CK(hipMalloc(&ol, n * 2)); CK(hipMalloc(&qp, n * 2)); CK(hipMalloc(&rh, rounds * NB * 2));
    CK(hipMalloc(&off, uint64_t(NB) * G * 4));
    hipLaunchKernelGGL(k_gen, dim3(2048), dim3(256), 0, 0, idx, val, n, shard, zipfish == 1);
    if (zipfish == 2) {
        if (g_zipf.empty()) g_zipf = zipf_host(n, shard);
        CK(hipMemcpy(idx, g_zipf.data(), n * 8, hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1, e2, e3;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2)); CK(hipEventCreate(&e3));
    float tc = 0, ts = 0, ti = 0;
    const int reps = 8;
    for (int it = 0; it < reps + 2; it++) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_count<NB>), dim3(G), dim3(kT), 0, 0, idx, n, chunk, shift, off);
        hipLaunchKernelGGL(k_scan1, dim3(1), dim3(kT), 0, 0, off, uint32_t(NB * G));
        CK(hipEventRecord(e1));
        if constexpr (SRC != 0)
            hipLaunchKernelGGL((k_scatter_src<NB, RPT>), dim3(G), dim3(kT), 0, 0, idx, reinterpret_cast<const double*>(val), n,
                               chunk, shift, off, ol, ov, qp, rh, src == 2 ? 1 : 0);
        else
            hipLaunchKernelGGL((k_scatter<NB, RPT>), dim3(G), dim3(kT), 0, 0, idx, val, n, chunk, shift, off, ol, ov, qp, rh);
        CK(hipEventRecord(e2));
        hipLaunchKernelGGL((k_inverse<NB, RPT>), dim3(G), dim3(kT), 0, 0, ov, n, chunk, off, qp, rh, back);
        CK(hipEventRecord(e3));
        CK(hipEventSynchronize(e3));
        CK(hipGetLastError());
        float a, b, c;
        CK(hipEventElapsedTime(&a, e0, e1)); CK(hipEventElapsedTime(&b, e1, e2)); CK(hipEventElapsedTime(&c, e2, e3));
        if (it >= 2) { tc += a; ts += b; ti += c; }
    }
    tc /= reps; ts /= reps; ti /= reps;
    // check: back == val, and every bucket run holds its bucket's records
    std::vector<double> hv(n), hb(n);
    CK(hipMemcpy(hv.data(), val, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), back, n * 8, hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    for (uint64_t k = 0; k < n; k++) bad += hv[k] != hb[k];
    printf("%s NB=%5d R=%6u G=%4d %s  count+scan %.3f ms  scatter %.3f ms (%.2f TB/s at 28 B)  inverse %.3f ms (%.2f TB/s at 18 B)  %s\n",
           src == 2 ? "src+warm" : src ? "src     " : "staged  ", NB, R, G, zipfish == 2 ? "zipf.99" : zipfish ? "skewed " : "uniform", tc, ts, n * 28.0 / ts / 1e9, ti, n * 18.0 / ti / 1e9,
           bad ? "MISMATCH" : "ok");
    fflush(stdout);
    CK(hipFree(idx)); CK(hipFree(val)); CK(hipFree(ov)); CK(hipFree(back)); CK(hipFree(ol)); CK(hipFree(qp));
    CK(hipFree(rh)); CK(hipFree(off));
}

int main() {
    const int z = 2;
    run<1024, 8>(z, 256);
    run<1024, 8, 1>(z, 256);
    run<1024, 16, 1>(z, 256);
    run<1024, 16, 2>(z, 256);
    run<1024, 16, 1>(z, 512);
    run<1024, 8>(z, 256);
    run<1024, 16, 1>(z, 256);
    return 0;
}
