// lmr_pack.hip — device pack of a batched op into per-destination op buffers.
//
// Restates the pack loops of the reference (src/array/unsafe/operations.rs:
// multi_val_multi_index :709-778, one_val_multi_indices :518-552): every global
// index is mapped to (destination PE, local offset) with the array's Block /
// Cyclic / sub-array math (src/array/unsafe.rs:1207-1223, 1610-1736), narrowed
// to the array's IndexSize, and appended to that PE's buffer together with its
// input position j (the reference's res_buffs, used to put fetch results back
// in input order, operations/handle.rs:315-317).
//
// The device version is a stable counting sort by PE: per-block PE counts ->
// exclusive scan over (PE, block) -> scatter with wave-ballot ranks, so each
// PE's buffer holds its records in input order — the concatenation, in order,
// of the reference's per-PE op buffers. Output is structure-of-arrays
// (indices, values, positions): coalesced for the apply kernels and for RCCL.
#include "lmr_internal.hpp"
#include "lmr_device.hpp"

namespace lmr {

struct PackK {
    lmr_layout_t L;
    const uint64_t* gidx;
    const uint8_t* vals;
    uint32_t vb;
    uint64_t n;
    uint32_t iw;
    uint64_t chunk;
    uint32_t G;
    uint32_t npes;
    uint32_t* counts;       // [npes * G], pe-major
    uint8_t* out_idx;
    uint8_t* out_vals;
    uint32_t* out_pos;
    uint32_t* err;
};

__global__ __launch_bounds__(1024) void k_pack_count(PackK p) {
    extern __shared__ uint32_t cnt[];
    for (uint32_t i = threadIdx.x; i < p.npes; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    const uint64_t lo = uint64_t(blockIdx.x) * p.chunk;
    const uint64_t hi = min(lo + p.chunk, p.n);
    bool oob = false;
    for (uint64_t k = lo + threadIdx.x; k < hi; k += blockDim.x) {
        uint64_t pe, off;
        if (!pe_and_offset(p.L, p.gidx[k], pe, off)) { oob = true; continue; }
        atomicAdd(&cnt[uint32_t(pe)], 1u);
    }
    if (oob) raise_err(p.err, LMR_ERRBIT_OOB);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < p.npes; i += blockDim.x)
        p.counts[uint64_t(i) * p.G + blockIdx.x] = cnt[i];
}

__device__ __forceinline__ void store_idx(uint8_t* base, uint32_t iw, uint64_t pos, uint64_t v) {
    switch (iw) {
    case 1: base[pos] = uint8_t(v); break;
    case 2: reinterpret_cast<uint16_t*>(base)[pos] = uint16_t(v); break;
    case 4: reinterpret_cast<uint32_t*>(base)[pos] = uint32_t(v); break;
    default: reinterpret_cast<uint64_t*>(base)[pos] = v; break;
    }
}

__device__ __forceinline__ void copy_val(uint8_t* dst, const uint8_t* src, uint32_t vb, uint64_t dpos,
                                         uint64_t spos) {
    switch (vb) {
    case 1: dst[dpos] = src[spos]; break;
    case 2: reinterpret_cast<uint16_t*>(dst)[dpos] = reinterpret_cast<const uint16_t*>(src)[spos]; break;
    case 4: reinterpret_cast<uint32_t*>(dst)[dpos] = reinterpret_cast<const uint32_t*>(src)[spos]; break;
    default: reinterpret_cast<uint64_t*>(dst)[dpos] = reinterpret_cast<const uint64_t*>(src)[spos]; break;
    }
}

// Stable scatter. The block walks its chunk in rounds of 1024 records (in
// order); inside a round, wave w holds records [64w, 64w+64). Rank of a record
// = records of the same PE in earlier rounds (cursor) + in earlier waves of
// this round (wave_base) + in earlier lanes of this wave (ballot popcount).
__global__ __launch_bounds__(1024) void k_pack_scatter(PackK p) {
    extern __shared__ uint32_t sm[];
    uint32_t* cursor = sm;                     // [npes]
    uint32_t* wcnt = sm + p.npes;              // [16][npes]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t i = threadIdx.x; i < p.npes; i += blockDim.x)
        cursor[i] = p.counts[uint64_t(i) * p.G + blockIdx.x];
    const uint64_t lo = uint64_t(blockIdx.x) * p.chunk;
    const uint64_t hi = min(lo + p.chunk, p.n);
    for (uint64_t r0 = lo; r0 < hi; r0 += 1024) {
        for (uint32_t i = threadIdx.x; i < 16 * p.npes; i += blockDim.x) wcnt[i] = 0;
        __syncthreads();
        const uint64_t k = r0 + threadIdx.x;
        uint64_t pe = 0, off = 0;
        bool valid = (k < hi) && pe_and_offset(p.L, p.gidx[k], pe, off);
        const uint32_t mype = valid ? uint32_t(pe) : 0xFFFFFFFFu;
        // group lanes by PE (match-any by repeated ballot over distinct values)
        uint64_t remaining = __ballot(true);
        uint64_t mine = 0;
        while (remaining) {
            int leader = __ffsll((unsigned long long)remaining) - 1;
            uint32_t x = __shfl(mype, leader, 64);
            uint64_t m = __ballot(mype == x);
            if (mype == x) mine = m;
            remaining &= ~m;
        }
        const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
        const uint32_t rank = __popcll(mine & lt);
        const bool first = (mine & lt) == 0;
        if (valid && first) wcnt[w * p.npes + mype] = __popcll(mine);
        __syncthreads();
        // per PE: exclusive scan over the 16 waves, advance the cursor
        for (uint32_t i = threadIdx.x; i < p.npes; i += blockDim.x) {
            uint32_t run = cursor[i];
            for (int ww = 0; ww < 16; ww++) {
                uint32_t c = wcnt[ww * p.npes + i];
                wcnt[ww * p.npes + i] = run;
                run += c;
            }
            cursor[i] = run;
        }
        __syncthreads();
        if (valid) {
            uint64_t pos = uint64_t(wcnt[w * p.npes + mype]) + rank;
            store_idx(p.out_idx, p.iw, pos, off);
            if (p.vals) copy_val(p.out_vals, p.vals, p.vb, pos, k);
            if (p.out_pos) p.out_pos[pos] = uint32_t(k);
        }
        __syncthreads();
    }
}

__global__ void k_dest_offsets(const uint32_t* counts, uint32_t npes, uint32_t G, const uint32_t* total,
                               uint64_t* dest_offsets, uint64_t* dest_counts) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= npes) {
        uint64_t o = (i < npes) ? counts[uint64_t(i) * G] : *total;
        dest_offsets[i] = o;
    }
    if (i < npes && dest_counts) {
        uint64_t nx = (i + 1 < npes) ? counts[uint64_t(i + 1) * G] : *total;
        dest_counts[i] = nx - counts[uint64_t(i) * G];
    }
}

hipError_t launch_pack(const PackArgs& a, uint32_t* counts, uint32_t* partials, uint32_t* total,
                       hipStream_t s) {
    const uint32_t npes = a.layout.num_pes;
    if (npes == 0 || npes > uint32_t(kMaxPackPes)) return hipErrorInvalidValue;
    uint64_t G = (a.n + 65535) / 65536;
    if (G > uint64_t(kMaxBinBlocks)) G = kMaxBinBlocks;
    if (G < 1) G = 1;
    PackK p;
    p.L = a.layout; p.gidx = a.gidx; p.vals = a.vals; p.vb = a.val_bytes; p.n = a.n;
    p.iw = a.index_size; p.chunk = (a.n + G - 1) / G; if (p.chunk == 0) p.chunk = 1;
    p.G = uint32_t(G); p.npes = npes; p.counts = counts;
    p.out_idx = a.out_idx; p.out_vals = a.out_vals; p.out_pos = a.out_pos; p.err = a.err;
    ProfScope ps(a.prof, LMR_STAGE_PACK, s);
    if (a.n > 0) {
        hipLaunchKernelGGL(k_pack_count, dim3(unsigned(G)), dim3(1024), size_t(npes) * 4, s, p);
    } else {
        hipError_t e0 = hipMemsetAsync(counts, 0, size_t(npes) * G * 4, s);
        if (e0 != hipSuccess) return e0;
    }
    hipError_t e = scan_exclusive_u32(counts, uint64_t(npes) * G, partials, total, s);
    if (e != hipSuccess) return e;
    if (a.n > 0)
        hipLaunchKernelGGL(k_pack_scatter, dim3(unsigned(G)), dim3(1024), size_t(npes) * 17 * 4, s, p);
    hipLaunchKernelGGL(k_dest_offsets, dim3((npes + 1 + 255) / 256), dim3(256),
                       0, s, counts, npes, uint32_t(G), total, a.dest_offsets, a.dest_counts);
    return hipGetLastError();
}

// ------------------------------------------------------------------ results
template <typename V>
__global__ void k_scatter_results(const V* __restrict__ in, const uint32_t* __restrict__ pos, uint64_t n,
                                  V* __restrict__ out, const uint8_t* ok_in, uint8_t* ok_out) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < n; k += stride) {
        uint32_t p = pos[k];
        out[p] = in[k];
        if (ok_in) ok_out[p] = ok_in[k];
    }
}

hipError_t launch_scatter_results(const uint8_t* in, const uint32_t* pos, uint64_t n,
                                  uint32_t elem_bytes, uint8_t* out, const uint8_t* ok_in,
                                  uint8_t* ok_out, Prof* prof, hipStream_t s) {
    if (n == 0) return hipSuccess;
    ProfScope ps(prof, LMR_STAGE_SCATTER_RESULTS, s);
    uint64_t g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    switch (elem_bytes) {
    case 1: hipLaunchKernelGGL((k_scatter_results<uint8_t>), dim3(unsigned(g)), dim3(256), 0, s,
                               in, pos, n, out, ok_in, ok_out); break;
    case 2: hipLaunchKernelGGL((k_scatter_results<uint16_t>), dim3(unsigned(g)), dim3(256), 0, s,
                               reinterpret_cast<const uint16_t*>(in), pos, n,
                               reinterpret_cast<uint16_t*>(out), ok_in, ok_out); break;
    case 4: hipLaunchKernelGGL((k_scatter_results<uint32_t>), dim3(unsigned(g)), dim3(256), 0, s,
                               reinterpret_cast<const uint32_t*>(in), pos, n,
                               reinterpret_cast<uint32_t*>(out), ok_in, ok_out); break;
    case 8: hipLaunchKernelGGL((k_scatter_results<uint64_t>), dim3(unsigned(g)), dim3(256), 0, s,
                               reinterpret_cast<const uint64_t*>(in), pos, n,
                               reinterpret_cast<uint64_t*>(out), ok_in, ok_out); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace lmr
