// lmr_host.hip — host-buffer ingestion of op buffers.
//
// In the reference the packed IdxVal<I,T> records of an op AM live in host
// memory: the shmem lamellae heap or a socket buffer
// (src/lamellae/shmem/shmem_comm.rs:302-352; the AM body deserialised in
// src/active_messaging/registered_active_message.rs:260-304, 443-497) and the
// fetch results go back as a host Vec<T>. lmr_apply_mvmi_host takes those host
// bytes as they are and pipelines them through the device:
//
//   h2d stream : copy piece i into slot i%2            (waits until slot's apply i-2 is done)
//   stream     : apply piece i (lmr_apply_mvmi)        (waits for copy i, and for slot's results D2H i-2)
//   d2h stream : copy piece i's results / Ok flags out (waits for apply i)
//
// so piece i+1's upload and piece i-1's result download overlap piece i's
// apply; PCIe (full duplex) is the bound. The DMA engines read in place what is page-locked for
// the library's purposes: a lamellae heap page-locked once for its lifetime
// (lmr_host_register_heap) and memory the HIP runtime allocated pinned (lmr_host_alloc).
//
// The library DMAs only between the device and host memory it knows is page-locked: the inner
// pages of a heap registered with lmr_host_register_heap, memory the HIP runtime itself allocated
// pinned (lmr_host_alloc / hipHostMalloc), and its own pinned bounce buffers (lmr_host_register
// only records a range: its buffers are staged like pageable ones). Records in pageable memory
// are copied by the host into a pinned slot before their upload; results / Ok flags bound for
// pageable memory land in a pinned slot and the host copies them out (the call then returns
// once they are written).
//
// Registration contract (round 5). Device faults (rounds 3 and 4, and twice more in round 5)
// surfaced as "illegal memory access" at a host<->device copy that followed tests which had
// registered (hipHostRegister) host ranges, unregistered them and freed the memory: first with two
// registrations sharing a page (round 4), then with a reference-counted page-aligned union
// (round 5, r5n, in a serialised run: every kernel had completed), then with only the whole pages
// inside each range pinned, one lock per range (r5t, at the next device-to-host copy). No library
// kernel was running at any of them, and the runs that never unpinned user memory (round 3's
// `_KEEP`) never faulted. The library therefore no longer page-locks caller memory at all:
// lmr_host_register records a caller range (refusing overlaps, as before) and copies through it
// are staged through the library's pinned bounce slots like any pageable buffer. Memory the HIP
// runtime allocated pinned -- lmr_host_alloc / hipHostMalloc, torch's pinned allocator -- is DMA'd
// in place: that is the reference's own contract, a lamellae heap mapped once at world init and
// dropped at shutdown (shmem_comm.rs:47-80), and the zero-copy path for callers.
#include "lmr_internal.hpp"
#include "../../include/lamellar_gpu_ops.h"
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <iterator>
#include <vector>
#include <map>
#include <mutex>
#include <set>
#include <shared_mutex>

namespace lmr {


// a recorded caller range [lo, hi)
struct HostRange {
    uintptr_t hi;
};
// a heap [lo, hi) whose whole inner pages [plo, phi) are pinned from registration to shutdown
struct HostHeap {
    uintptr_t hi, plo, phi;
};
struct HostRegistry {
    std::mutex mu;                                   // registry maps and the stage list
    std::shared_mutex pin;                           // shared: a call DMAs through pinned memory; unique: lmr_host_free
    std::map<uintptr_t, HostRange> ranges;
    std::map<uintptr_t, HostHeap> heaps;             // lmr_host_register_heap: pinned for their lifetime
    std::set<HostStage*> stages;                     // every context's host stage (drained before an unpin)
    std::map<uintptr_t, uint64_t> allocs;            // lmr_host_alloc blocks: base -> bytes
};
HostRegistry& reg() {
    static HostRegistry r;
    return r;
}
// memory the runtime allocated pinned (hipHostMalloc, torch's pinned allocator) covering the
// whole range: DMA'd in place as well
static bool runtime_pinned(const void* p, uint64_t bytes) {
    if (!p || bytes == 0) return false;
    const uintptr_t lo = reinterpret_cast<uintptr_t>(p), hi = lo + bytes;
    {
        std::lock_guard<std::mutex> g(reg().mu);
        auto& A = reg().allocs;
        auto it = A.upper_bound(lo);
        if (it != A.begin() && std::prev(it)->first + std::prev(it)->second >= hi) return true;
    }
    // other runtime allocations (torch's pinned allocator): both ends host memory of one
    // allocation (hipPointerGetAttributes reports the queried address itself, not the base)
    hipPointerAttribute_t a{}, b{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return false; }
    if (a.type != hipMemoryTypeHost) return false;
    const void* last = static_cast<const uint8_t*>(p) + bytes - 1;
    if (hipPointerGetAttributes(&b, last) != hipSuccess) { (void)hipGetLastError(); return false; }
    if (b.type != hipMemoryTypeHost) return false;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, const_cast<void*>(p)) != hipSuccess) { (void)hipGetLastError(); return false; }
    const uintptr_t bl = reinterpret_cast<uintptr_t>(base);
    return bl <= lo && hi <= bl + size;
}
// the part of [p, p + bytes) a DMA may touch in place, as offsets [*a, *b) (*a == *b: none): all
// of it when the runtime allocated it pinned, nothing otherwise (caller memory is never locked)
static void pinned_span(const void* p, uint64_t bytes, uint64_t* a, uint64_t* b) {
    *a = *b = 0;
    if (!p || bytes == 0) return;
    const uintptr_t lo = reinterpret_cast<uintptr_t>(p), hi = lo + bytes;
    {   // inside a registered heap: its pinned inner pages in place, the partial end pages staged
        std::lock_guard<std::mutex> g(reg().mu);
        auto& H = reg().heaps;
        auto it = H.upper_bound(lo);
        if (it != H.begin()) {
            --it;
            if (it->first <= lo && hi <= it->second.hi) {
                const uintptr_t x = std::max(lo, it->second.plo), y = std::min(hi, it->second.phi);
                if (x < y) { *a = x - lo; *b = y - lo; }
                return;
            }
        }
    }
    if (runtime_pinned(p, bytes)) *b = bytes;
}

// [lo, hi) overlaps a recorded range or heap (caller holds reg().mu)
static bool overlaps_locked(uintptr_t lo, uintptr_t hi) {
    auto& R = reg().ranges;
    auto it = R.lower_bound(lo);
    if (it != R.end() && it->first < hi) return true;
    if (it != R.begin() && std::prev(it)->second.hi > lo) return true;
    auto& H = reg().heaps;
    auto ht = H.lower_bound(lo);
    if (ht != H.end() && ht->first < hi) return true;
    return ht != H.begin() && std::prev(ht)->second.hi > lo;
}

struct HostStage {
    hipStream_t h2d = nullptr, d2h = nullptr;
    uint8_t* d_rec[2] = {nullptr, nullptr};
    uint8_t* d_res[2] = {nullptr, nullptr};
    uint8_t* d_ok[2] = {nullptr, nullptr};
    // pinned bounce slots for pageable host buffers (made on first use)
    uint8_t* h_rec[2] = {nullptr, nullptr};
    uint8_t* h_res[2] = {nullptr, nullptr};
    uint8_t* h_ok[2] = {nullptr, nullptr};
    hipEvent_t copied[2] = {}, applied[2] = {}, drained[2] = {};
    uint64_t piece_recs = 0;
    uint64_t rec_bytes_cap = 0;   // bytes per record slot capacity (largest record size supported: 16)
};

void host_stage_free(HostStage* h) {
    if (!h) return;
    {
        std::lock_guard<std::mutex> g(reg().mu);
        reg().stages.erase(h);
    }
    if (h->h2d) (void)hipStreamSynchronize(h->h2d);
    if (h->d2h) (void)hipStreamSynchronize(h->d2h);
    for (int b = 0; b < 2; b++) {
        if (h->d_rec[b]) (void)hipFree(h->d_rec[b]);
        if (h->d_res[b]) (void)hipFree(h->d_res[b]);
        if (h->d_ok[b]) (void)hipFree(h->d_ok[b]);
        if (h->h_rec[b]) (void)hipHostFree(h->h_rec[b]);
        if (h->h_res[b]) (void)hipHostFree(h->h_res[b]);
        if (h->h_ok[b]) (void)hipHostFree(h->h_ok[b]);
        if (h->copied[b]) (void)hipEventDestroy(h->copied[b]);
        if (h->applied[b]) (void)hipEventDestroy(h->applied[b]);
        if (h->drained[b]) (void)hipEventDestroy(h->drained[b]);
    }
    if (h->h2d) (void)hipStreamDestroy(h->h2d);
    if (h->d2h) (void)hipStreamDestroy(h->d2h);
    delete h;
}

static uint64_t host_piece_records() {
    const char* v = getenv("LMR_HOST_PIECE_RECORDS");
    uint64_t x = (v && *v) ? strtoull(v, nullptr, 10) : (uint64_t(1) << 22);
    if (x < 1024) x = 1024;
    if (x > (uint64_t(1) << 26)) x = uint64_t(1) << 26;
    return x;
}

static hipError_t host_stage_get(lmr_ctx* ctx, HostStage** out) {
    if (ctx->host) { *out = ctx->host; return hipSuccess; }
    HostStage* h = new HostStage();
    h->piece_recs = host_piece_records();
    h->rec_bytes_cap = 16;
    hipError_t e = hipStreamCreateWithFlags(&h->h2d, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->d2h, hipStreamNonBlocking);
    for (int b = 0; b < 2 && e == hipSuccess; b++) {
        e = hipMalloc(&h->d_rec[b], h->piece_recs * h->rec_bytes_cap);
        if (e == hipSuccess) e = hipMalloc(&h->d_res[b], h->piece_recs * 8);
        if (e == hipSuccess) e = hipMalloc(&h->d_ok[b], h->piece_recs);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->copied[b], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->applied[b], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->drained[b], hipEventDisableTiming);
    }
    if (e != hipSuccess) { host_stage_free(h); return e; }
    {
        std::lock_guard<std::mutex> g(reg().mu);
        reg().stages.insert(h);
    }
    ctx->host = h;
    *out = h;
    return hipSuccess;
}

static hipError_t host_bounce_get(HostStage* h) {
    hipError_t e = hipSuccess;
    for (int b = 0; b < 2 && e == hipSuccess; b++) {
        if (!h->h_rec[b]) e = hipHostMalloc(&h->h_rec[b], h->piece_recs * h->rec_bytes_cap, hipHostMallocDefault);
        if (e == hipSuccess && !h->h_res[b]) e = hipHostMalloc(&h->h_res[b], h->piece_recs * 8, hipHostMallocDefault);
        if (e == hipSuccess && !h->h_ok[b]) e = hipHostMalloc(&h->h_ok[b], h->piece_recs, hipHostMallocDefault);
    }
    return e;
}

// every context's host-stage copies done (caller holds reg().mu and the unique pin lock: no
// lmr_apply_mvmi_host is between its checks and its last enqueued copy)
static hipError_t drain_host_stages_locked() {
    hipError_t r = hipSuccess;
    for (HostStage* h : reg().stages) {
        hipError_t e = hipStreamSynchronize(h->h2d);
        if (e == hipSuccess) e = hipStreamSynchronize(h->d2h);
        if (e != hipSuccess) r = e;
    }
    return r;
}


}  // namespace lmr

using namespace lmr;

extern "C" {

lmr_status_t lmr_host_register(void* ptr, uint64_t bytes) {
    if (!ptr || bytes == 0) return LMR_E_INVALID;
    const uintptr_t lo = reinterpret_cast<uintptr_t>(ptr), hi = lo + bytes;
    if (hi < lo) return LMR_E_INVALID;
    HostRegistry& R = reg();
    std::lock_guard<std::mutex> g(R.mu);
    if (overlaps_locked(lo, hi)) return LMR_E_INVALID;   // overlapping an earlier range or heap: refused
    R.ranges[lo] = HostRange{hi};
    return LMR_OK;
}

lmr_status_t lmr_host_register_heap(void* ptr, uint64_t bytes) {
    if (!ptr || bytes == 0) return LMR_E_INVALID;
    const uintptr_t lo = reinterpret_cast<uintptr_t>(ptr), hi = lo + bytes;
    if (hi < lo) return LMR_E_INVALID;
    HostRegistry& R = reg();
    std::unique_lock<std::shared_mutex> pin(R.pin);
    std::lock_guard<std::mutex> g(R.mu);
    if (overlaps_locked(lo, hi)) return LMR_E_INVALID;
    const uintptr_t page = 4096;
    const uintptr_t plo = (lo + page - 1) & ~(page - 1), phi = std::max(plo, hi & ~(page - 1));
    if (phi > plo && hipHostRegister(reinterpret_cast<void*>(plo), phi - plo, hipHostRegisterDefault) != hipSuccess) {
        (void)hipGetLastError();
        return LMR_E_HIP;
    }
    R.heaps[lo] = HostHeap{hi, plo, phi};
    return LMR_OK;
}

lmr_status_t lmr_host_unregister_heap(void* ptr) {
    if (!ptr) return LMR_E_INVALID;
    HostRegistry& R = reg();
    std::unique_lock<std::shared_mutex> pin(R.pin);
    std::lock_guard<std::mutex> g(R.mu);
    auto it = R.heaps.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == R.heaps.end()) return LMR_E_INVALID;
    if (it->second.phi > it->second.plo) {
        if (drain_host_stages_locked() != hipSuccess) return LMR_E_HIP;
        if (hipHostUnregister(reinterpret_cast<void*>(it->second.plo)) != hipSuccess) {
            (void)hipGetLastError();
            return LMR_E_HIP;
        }
    }
    R.heaps.erase(it);
    return LMR_OK;
}

lmr_status_t lmr_host_unregister(void* ptr) {
    if (!ptr) return LMR_E_INVALID;
    HostRegistry& R = reg();
    std::lock_guard<std::mutex> g(R.mu);
    auto it = R.ranges.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == R.ranges.end()) return LMR_E_INVALID;      // not the start of a registration
    R.ranges.erase(it);
    return LMR_OK;
}

lmr_status_t lmr_host_registered(const void* ptr, uint64_t bytes, uint64_t* pin_base, uint64_t* pin_bytes,
                                 uint32_t* ranges) {
    if (!ptr || bytes == 0) return LMR_E_INVALID;
    const uintptr_t lo = reinterpret_cast<uintptr_t>(ptr), hi = lo + bytes;
    HostRegistry& R = reg();
    std::lock_guard<std::mutex> g(R.mu);
    auto ht = R.heaps.upper_bound(lo);
    if (ht != R.heaps.begin() && std::prev(ht)->first <= lo && hi <= std::prev(ht)->second.hi) {
        --ht;
        if (pin_base) *pin_base = ht->second.plo;
        if (pin_bytes) *pin_bytes = ht->second.phi - ht->second.plo;
        if (ranges) *ranges = 1;
        return LMR_OK;
    }
    auto it = R.ranges.upper_bound(lo);
    if (it == R.ranges.begin()) return LMR_E_INVALID;
    --it;
    if (!(it->first <= lo && hi <= it->second.hi)) return LMR_E_INVALID;
    if (pin_base) *pin_base = 0;                         // a recorded range: nothing is page-locked
    if (pin_bytes) *pin_bytes = 0;
    if (ranges) *ranges = 1;
    return LMR_OK;
}

lmr_status_t lmr_host_alloc(uint64_t bytes, void** out) {
    if (!out || bytes == 0) return LMR_E_INVALID;
    *out = nullptr;
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) { (void)hipGetLastError(); return LMR_E_HIP; }
    std::lock_guard<std::mutex> g(reg().mu);
    reg().allocs[reinterpret_cast<uintptr_t>(p)] = bytes;
    *out = p;
    return LMR_OK;
}

lmr_status_t lmr_host_free(void* ptr) {
    if (!ptr) return LMR_E_INVALID;
    HostRegistry& R = reg();
    std::unique_lock<std::shared_mutex> pin(R.pin);
    std::lock_guard<std::mutex> g(R.mu);
    if (!R.allocs.count(reinterpret_cast<uintptr_t>(ptr))) return LMR_E_INVALID;
    if (drain_host_stages_locked() != hipSuccess) return LMR_E_HIP;
    if (hipHostFree(ptr) != hipSuccess) { (void)hipGetLastError(); return LMR_E_HIP; }
    R.allocs.erase(reinterpret_cast<uintptr_t>(ptr));
    return LMR_OK;
}

lmr_status_t lmr_apply_mvmi_host(lmr_ctx_t* ctx, const lmr_apply_desc_t* desc, const void* h_idx_vals,
                                 uint64_t nbytes, uint32_t index_size, void* h_results, uint8_t* h_ok,
                                 lmr_stream_t stream) {
    if (!ctx || !desc) return LMR_E_INVALID;
    index_size = am_index_width(index_size);
    if (desc->dtype >= LMR_NUM_DTYPES) return LMR_E_INVALID;
    const uint32_t rb = lmr_record_bytes(index_size, desc->dtype);
    const uint32_t eb = rb ? uint32_t(dtype_bytes(int(desc->dtype))) : 0;
    if (rb == 0 || rb > 16) return LMR_E_INVALID;
    const uint64_t n = nbytes / rb;
    if (n == 0) return LMR_OK;
    if (!h_idx_vals) return LMR_E_INVALID;
    (void)hipSetDevice(ctx->device);
    HostStage* h = nullptr;
    if (host_stage_get(ctx, &h) != hipSuccess) return LMR_E_HIP;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uint64_t P = h->piece_recs;
    if (desc->strategy != LMR_STRATEGY_DIRECT && P >= 65536 && ctx->rec_cap < P) {
        // the workspace grows (once): the context's earlier work is ordered on `stream` (one
        // stream at a time per context) plus the library's own side and host-stage streams
        if (hipStreamSynchronize(s) != hipSuccess || (ctx->side && hipStreamSynchronize(ctx->side) != hipSuccess) ||
            hipStreamSynchronize(h->h2d) != hipSuccess || hipStreamSynchronize(h->d2h) != hipSuccess)
            return LMR_E_HIP;
        lmr_status_t st = lmr_ctx_reserve(ctx, P);
        if (st != LMR_OK) return st;
    }
    // lmr_host_alloc blocks stay allocated while this call enqueues copies through them
    // (lmr_host_free takes the lock exclusively and drains the host-stage streams first)
    std::shared_lock<std::shared_mutex> pin(reg().pin);
    const uint32_t ret = lmr_op_ret_kind(desc->op);
    const bool want_res = h_results && ret != LMR_RET_NONE;
    const bool want_ok = h_ok && ret == LMR_RET_RESULT;
    // pageable buffers go through the pinned bounce slots
    const uint8_t* src = reinterpret_cast<const uint8_t*>(h_idx_vals);
    // the pinned bounce slots, made on the first copy that stages anything
    auto stage_ready = [&]() -> bool { return h->h_rec[0] || host_bounce_get(h) == hipSuccess; };
    // host -> device: runtime-pinned memory DMA'd in place, anything else (pageable or registered
    // caller memory) copied by the host into slot b's bounce buffer first (once that slot's
    // previous upload is done)
    auto upload = [&](uint8_t* dev, const uint8_t* hp, uint64_t bytes, int b, uint64_t piece) -> lmr_status_t {
        uint64_t x, y;
        pinned_span(hp, bytes, &x, &y);
        if (y > x && hipMemcpyAsync(dev + x, hp + x, y - x, hipMemcpyHostToDevice, h->h2d) != hipSuccess)
            return LMR_E_HIP;
        if (x == 0 && y == bytes) return LMR_OK;
        if (!stage_ready()) return LMR_E_HIP;
        if (piece >= 2 && hipEventSynchronize(h->copied[b]) != hipSuccess) return LMR_E_HIP;
        if (x == y) x = y = bytes;                      // nothing pinned: one staged copy of the whole
        uint8_t* slot = h->h_rec[b];
        memcpy(slot, hp, x);
        memcpy(slot + x, hp + y, bytes - y);
        if (x > 0 && hipMemcpyAsync(dev, slot, x, hipMemcpyHostToDevice, h->h2d) != hipSuccess) return LMR_E_HIP;
        if (bytes > y && hipMemcpyAsync(dev + y, slot + x, bytes - y, hipMemcpyHostToDevice, h->h2d) != hipSuccess)
            return LMR_E_HIP;
        return LMR_OK;
    };
    // device -> host: the pinned part in place, the rest into a bounce buffer of slot b (copied
    // out by the host once the download is done: Part)
    struct Part { uint8_t* dst = nullptr; const uint8_t* slot = nullptr; uint64_t x = 0, y = 0, bytes = 0; };
    auto download = [&](uint8_t* hp, const uint8_t* dev, uint64_t bytes, uint8_t* const* slots, int b,
                        Part* part) -> lmr_status_t {
        uint64_t x, y;
        pinned_span(hp, bytes, &x, &y);
        *part = Part{};
        if (y > x && hipMemcpyAsync(hp + x, dev + x, y - x, hipMemcpyDeviceToHost, h->d2h) != hipSuccess)
            return LMR_E_HIP;
        if (x == 0 && y == bytes) return LMR_OK;
        if (!stage_ready()) return LMR_E_HIP;
        if (x == y) x = y = bytes;
        uint8_t* slot = slots[b];
        if (x > 0 && hipMemcpyAsync(slot, dev, x, hipMemcpyDeviceToHost, h->d2h) != hipSuccess) return LMR_E_HIP;
        if (bytes > y && hipMemcpyAsync(slot + x, dev + y, bytes - y, hipMemcpyDeviceToHost, h->d2h) != hipSuccess)
            return LMR_E_HIP;
        *part = Part{hp, slot, x, y, bytes};
        return LMR_OK;
    };
    // results of a piece staged through a slot are copied out by the host once its download is done
    struct Out { bool live = false; Part res, ok; };
    Out pend[2];
    auto copy_out = [](const Part& q) {
        if (!q.dst) return;
        memcpy(q.dst, q.slot, q.x);
        memcpy(q.dst + q.y, q.slot + q.x, q.bytes - q.y);
    };
    auto drain_out = [&](int b) -> lmr_status_t {
        if (!pend[b].live) return LMR_OK;
        if (hipEventSynchronize(h->drained[b]) != hipSuccess) return LMR_E_HIP;
        copy_out(pend[b].res);
        copy_out(pend[b].ok);
        pend[b].live = false;
        return LMR_OK;
    };
    uint64_t i = 0;
    for (uint64_t r0 = 0; r0 < n; r0 += P, i++) {
        const int b = int(i & 1);
        const uint64_t m = (n - r0 < P) ? n - r0 : P;
        // upload: the slot's previous apply must have consumed its records, and the bounce slot's
        // previous upload must be done before the host writes it again
        if (hipStreamWaitEvent(h->h2d, h->applied[b], 0) != hipSuccess) return LMR_E_HIP;
        lmr_status_t st = upload(h->d_rec[b], src + r0 * rb, m * rb, b, i);
        if (st != LMR_OK) return st;
        if (hipEventRecord(h->copied[b], h->h2d) != hipSuccess) return LMR_E_HIP;
        // apply on the caller's stream (after the upload and the slot's previous download)
        if (hipStreamWaitEvent(s, h->copied[b], 0) != hipSuccess) return LMR_E_HIP;
        if (hipStreamWaitEvent(s, h->drained[b], 0) != hipSuccess) return LMR_E_HIP;
        st = lmr_apply_mvmi(ctx, desc, h->d_rec[b], m * rb, index_size, want_res ? h->d_res[b] : nullptr,
                            want_ok ? h->d_ok[b] : nullptr, stream);
        if (st != LMR_OK) return st;
        if (hipEventRecord(h->applied[b], s) != hipSuccess) return LMR_E_HIP;
        // download of the returned values (into the caller's pinned pages or a bounce slot)
        if (want_res || want_ok) {
            if ((st = drain_out(b)) != LMR_OK) return st;   // the slot's previous results are out
            if (hipStreamWaitEvent(h->d2h, h->applied[b], 0) != hipSuccess) return LMR_E_HIP;
            Out o;
            if (want_res && (st = download(static_cast<uint8_t*>(h_results) + r0 * eb, h->d_res[b], m * eb,
                                           h->h_res, b, &o.res)) != LMR_OK)
                return st;
            if (want_ok && (st = download(h_ok + r0, h->d_ok[b], m, h->h_ok, b, &o.ok)) != LMR_OK) return st;
            if (hipEventRecord(h->drained[b], h->d2h) != hipSuccess) return LMR_E_HIP;
            o.live = o.res.dst || o.ok.dst;
            pend[b] = o;
        }
    }
    for (int b = 0; b < 2; b++) {
        const lmr_status_t st = drain_out(b);
        if (st != LMR_OK) return st;
    }
    // completion on the caller's stream covers the downloads too
    for (int b = 0; b < 2; b++)
        if (hipStreamWaitEvent(s, h->drained[b], 0) != hipSuccess) return LMR_E_HIP;
    return LMR_OK;
}

}  // extern "C"
