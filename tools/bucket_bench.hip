// bucket_bench.hip — measures the bucketed peer push's passes at the geometry of an 8-GPU run on
// one GPU (not product code): the library's own launchers (liblamellar_gpu_ops.so)
// on the per-GPU work of one N = 8 step.
//
//   pack  : one PE's 2^26-record chunk of u64 add records, uniform over a Block array of 8 x 2^26
//           elements, packed by (owner, owner bucket: 256 tiles by default, LMR_BUCKET_TPB) = 256 keys into eight owners'
//           receive regions (uncached device memory, as the peer transport allocates them; on one
//           GPU all eight are local, so no xGMI time is in these numbers)
//   fine  : one owner's chunk: the eight regions read back as its eight sources' bucket slices
//           (each holds bucket-local offsets, the shape an owner receives) and binned into the
//           session's fixed tile regions
//   both  : pack and fine at once on two streams (the exchange overlaps chunk j's fine pass with
//           chunk j + 1's pack), on separate region sets
//   sweep : the tile sweep of a session of four chunks (2^28 records) over the 2^26-element shard
// usage: tools/bucket_bench [reps]      (BB_CACHED=1: plain cached regions, a probe only)
// build: see tools/bucket_bench.sh
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../lamellar-runtime_amd/csrc/lmr_internal.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace lmr;

__global__ void k_init(uint64_t* g, uint64_t* v, uint64_t n, uint64_t range, uint64_t seed) {
    for (uint64_t k = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; k < n; k += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t z = (k + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        g[k] = z % range;
        v[k] = z & 0xFFFF;
    }
}

struct Regions {
    std::vector<uint8_t*> idx, val;
    uint8_t** d_idx = nullptr;
    uint8_t** d_val = nullptr;
};

static Regions make_regions(uint32_t npes, uint64_t R) {
    Regions r;
    r.idx.resize(npes);
    r.val.resize(npes);
    // BB_CACHED=1: plain (coarse-grained, cached) device memory instead of the peer transport's
    // uncached regions (a probe of what the uncached write path costs; not a valid peer region)
    static const bool cached = getenv("BB_CACHED") && getenv("BB_CACHED")[0] == '1';
    for (uint32_t q = 0; q < npes; q++) {
        if (cached) {
            CK(hipMalloc(reinterpret_cast<void**>(&r.idx[q]), R * 8));
            CK(hipMalloc(reinterpret_cast<void**>(&r.val[q]), R * 8));
        } else {
            CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&r.idx[q]), R * 8, hipDeviceMallocUncached));
            CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&r.val[q]), R * 8, hipDeviceMallocUncached));
        }
    }
    CK(hipMalloc(&r.d_idx, npes * sizeof(void*)));
    CK(hipMalloc(&r.d_val, npes * sizeof(void*)));
    CK(hipMemcpy(r.d_idx, r.idx.data(), npes * sizeof(void*), hipMemcpyHostToDevice));
    CK(hipMemcpy(r.d_val, r.val.data(), npes * sizeof(void*), hipMemcpyHostToDevice));
    return r;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    const uint32_t npes = 8;
    const uint64_t per_pe = uint64_t(1) << 26, n = uint64_t(1) << 26;
    const uint64_t q = n / npes, R = q + q / 8 + 4096;   // the peer transport's default region
    lmr_layout_t L{};
    L.num_pes = npes;
    L.my_pe = 0;
    L.distribution = LMR_DIST_BLOCK;
    L.size = per_pe * npes;
    L.orig_elem_per_pe = per_pe;
    L.orig_remaining_elems = 0;
    uint32_t C = 0;
    int cshift = 0;
    if (!bucket_geometry(L, LMR_U64, C, cshift)) { printf("geometry refused\n"); return 1; }
    const uint32_t cap_b = bucket_slice_cap(R, C, 8);
    printf("geometry: %u PEs x %u buckets = %u keys, slice %u records (chunk share %lu)\n", npes, C, npes * C, cap_b,
           (unsigned long)(n / (npes * C)));
    uint64_t *g, *v;
    CK(hipMalloc(&g, n * 8));
    CK(hipMalloc(&v, n * 8));
    hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, g, v, n, L.size, 777ull);
    Regions A = make_regions(npes, R), B = make_regions(npes, R);
    uint32_t *fill, *tot, *err, *ovf;
    uint64_t* ovf_g;
    CK(hipMalloc(&fill, npes * C * 4));
    CK(hipMemset(fill, 0, npes * C * 4));
    CK(hipMalloc(&tot, npes * 4));
    CK(hipMalloc(&err, 4));
    CK(hipMemset(err, 0, 4));
    CK(hipMalloc(&ovf, 8));
    CK(hipMalloc(&ovf_g, n * 8));
    uint8_t* ovf_v;
    CK(hipMalloc(&ovf_v, n * 8));
    // owner session: shard of 2^26 u64, workspace for 2^30 records (bench.py's default)
    uint64_t* shard;
    CK(hipMalloc(&shard, per_pe * 8));
    CK(hipMemset(shard, 0, per_pe * 8));
    const uint64_t cap = uint64_t(1) << 30;
    uint8_t* ws;
    CK(hipMalloc(&ws, tiled_ws_bytes(cap)));
    TiledWs w = carve_tiled_ws(ws, cap);
    uint32_t* tfill;
    CK(hipMalloc(&tfill, kMaxTiles * 4));
    CK(hipMemset(tfill, 0, kMaxTiles * 4));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t a1, z1, a2, z2;
    for (hipEvent_t* e : {&a1, &z1, &a2, &z2}) CK(hipEventCreate(e));

    auto pack = [&](Regions& r, hipStream_t s) {
        PackArgs pa{};
        pa.layout = L;
        pa.gidx = g;
        pa.vals = reinterpret_cast<const uint8_t*>(v);
        pa.val_bytes = 8;
        pa.n = n;
        pa.index_size = 4;
        pa.err = err;
        pa.ovf_gidx = ovf_g;
        pa.ovf_vals = ovf_v;
        pa.ovf_count = ovf;
        pa.ovf_cap = n;
        pa.out_idx_tab = r.d_idx;
        pa.out_vals_tab = r.d_val;
        CK(launch_pack_bucket(pa, C, cshift, cap_b, fill, tot, s));
    };
    BucketSession bs;
    bs.open = true;
    bs.desc.shard = shard;
    bs.desc.shard_len = per_pe;
    bs.desc.kind = LMR_KIND_NATIVE_ATOMIC;
    bs.desc.dtype = LMR_U64;
    bs.desc.op = LMR_OP_ADD;
    bs.C = C;
    bs.tpb_log2 = bucket_tpb_log2();
    bs.T = uint32_t(per_pe >> tile_shift(LMR_U64));
    bs.cap_t = std::min<uint64_t>(w.tmp_cap, 0xFFFFFFFFull) / bs.T;
    bs.tfill = tfill;
    bs.err = err;
    auto fine = [&](Regions& r, hipStream_t s) {
        BucketChunk c;
        c.S = npes;
        for (uint32_t p = 0; p < npes; p++) {
            c.idx[p] = r.idx[p];
            c.val[p] = r.val[p];
            c.cap_b[p] = cap_b;
        }
        c.expect = n;
        CK(launch_fine_bucket(c, bs, w, s));
        bs.staged += n;
    };
    auto ms_of = [&](hipEvent_t a, hipEvent_t z) { float m = 0; CK(hipEventElapsedTime(&m, a, z)); return m; };
    // fill both region sets once
    CK(hipMemset(ovf, 0, 8));
    pack(A, s1);
    pack(B, s1);
    CK(hipStreamSynchronize(s1));
    uint32_t h_ovf = 0;
    CK(hipMemcpy(&h_ovf, ovf, 4, hipMemcpyDeviceToHost));
    printf("overflow records per chunk: %u\n", h_ovf / 2);
    double t_pack = 0, t_fine = 0, t_both = 0, t_p2 = 0, t_f2 = 0, t_sweep = 0;
    int sweeps = 0;
    for (int r = 0; r < reps + 1; r++) {
        CK(hipMemset(ovf, 0, 8));
        CK(hipEventRecord(a1, s1));
        pack(A, s1);
        CK(hipEventRecord(z1, s1));
        CK(hipEventSynchronize(z1));
        const double tp = ms_of(a1, z1);
        CK(hipEventRecord(a1, s1));
        fine(B, s1);
        CK(hipEventRecord(z1, s1));
        CK(hipEventSynchronize(z1));
        const double tf = ms_of(a1, z1);
        // both at once: a pack into A while the fine pass reads B
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a1, s1));
        CK(hipStreamWaitEvent(s2, a1, 0));
        CK(hipEventRecord(a2, s2));
        pack(A, s1);
        fine(B, s2);
        CK(hipEventRecord(z1, s1));
        CK(hipEventRecord(z2, s2));
        CK(hipEventSynchronize(z1));
        CK(hipEventSynchronize(z2));
        const double tb = std::max(ms_of(a1, z1), ms_of(a1, z2));
        if (r > 0) { t_pack += tp; t_fine += tf; t_both += tb; t_p2 += ms_of(a1, z1); t_f2 += ms_of(a2, z2); }
        if (bs.staged >= (uint64_t(1) << 28) * 3 / 2 || bs.staged + 2 * n > bucket_session_limit(bs)) {
            // a session of records from every fine pass so far: one sweep (timed per 2^28 records)
            const uint64_t st = bs.staged;
            CK(hipEventRecord(a1, s1));
            CK(launch_bucket_sweep(bs, w, s1));
            CK(hipEventRecord(z1, s1));
            CK(hipEventSynchronize(z1));
            t_sweep += ms_of(a1, z1) * double(uint64_t(1) << 28) / double(st);
            sweeps++;
            bs.open = true;
        }
    }
    uint32_t e = 0;
    CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    const double tp = t_pack / reps, tf = t_fine / reps, tb = t_both / reps;
    const double recs = double(n);
    printf("pack  alone   %.3f ms per 2^26 records (28 B/rec: %.2f TB/s)\n", tp, 28.0 * recs / (tp * 1e-3) / 1e12);
    printf("fine  alone   %.3f ms per 2^26 records (22 B/rec: %.2f TB/s)\n", tf, 22.0 * recs / (tf * 1e-3) / 1e12);
    printf("both at once  %.3f ms (pack %.3f, fine %.3f on their streams; 50 B/rec: %.2f TB/s)\n", tb, t_p2 / reps,
           t_f2 / reps, 50.0 * recs / (tb * 1e-3) / 1e12);
    if (sweeps) printf("sweep         %.3f ms per 2^28 session records (%d sweeps)\n", t_sweep / sweeps, sweeps);
    printf("error bits 0x%x\n", e);
    return 0;
}
