// lmr_peer.hip — the peer-memory transport: the exchange's records pushed straight into the
// owners' HBM over xGMI (IPC-mapped receive regions), with a shared-memory mailbox for the
// per-chunk counts and flags.
//
// The reference's shmem lamellae is a peer-segment protocol already: every PE maps a
// /dev/shm heap at world init (src/lamellae/shmem/shmem_comm.rs:47-80, 302-352), a sender
// announces a message with a {addr, size, hash} command in the receiver's command queue
// (src/lamellae/command_queues.rs:26-35, 725-807) and the receiver copies the bytes out of the
// sender's segment (:996-1021). Here the heap is HBM: every PE allocates fixed receive regions
// (one per source PE and chunk parity) and exports them with hipIpcGetMemHandle; every other PE
// maps them (hipIpcOpenMemHandle). A sender's count-free pack writes each destination's runs
// directly into that destination's region (no send buffer, no RCCL copy: 88 B/op per GPU at
// N = 8 instead of 109), then publishes the region's record count and a sequence
// number in the mailbox; the owner's apply stream waits for every source's sequence number,
// stages each region with its count read on the device, and marks the region free for the
// sender's next use. The mailbox is a /dev/shm segment shared by the PEs of the node (the
// reference's own fake network, lamellar_run.sh:31-40) registered with HIP, so flags cross
// processes and GPUs coherently (fine-grained host memory, system-scope loads and stores).
// Nothing is waited for on the host per chunk: one host handshake per batch agrees on the
// chunk count and whether every PE can take the push path.
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>
#include <vector>
#include "lmr_internal.hpp"
#include "lmr_device.hpp"

namespace lmr {

namespace {

constexpr uint64_t kPeerMagic = 0x4c4d52504545520aull;   // "LMRPEER\n"
constexpr uint32_t kPeerMaxPes = 64;
constexpr int kInfoWords = 8;

// one IPC allocation per (source, parity, index | values) region: every allocation stays far below
// 2 GiB (a 2.4 GB receive block stalled hipIpcOpenMemHandle in the importing process; 1 GB did not)
constexpr int kRegionAllocs = 4;          // per source: parity 0 / 1 x index / values
struct PeSlot {
    hipIpcMemHandle_t handle[kPeerMaxPes][kRegionAllocs];
    uint64_t region_recs;
    uint64_t ready;                       // 1: handle valid
    uint64_t opened;                      // 1: this PE has mapped every peer's regions and built its tables
    uint64_t bseq[2];                     // batch handshake, double-buffered by batch parity
    int64_t info[2][kInfoWords];
    uint64_t closing;
    uint64_t mapped;                      // 1: this PE's hipIpcOpenMemHandle calls are done
    uint64_t pad[4];
};

struct MbHeader {
    uint64_t magic;
    uint64_t npes;
    uint64_t created;
    uint64_t pad[5];
};

// mailbox flag arrays, index (owner q, source p, parity b) = (q * npes + p) * 2 + b
struct Mailbox {
    MbHeader* hdr;
    PeSlot* slots;
    uint64_t* pub;        // source p published its chunk for owner q (sequence number)
    int64_t* cnt;         // the records it put in q's region for that chunk
    uint64_t* freed;      // owner q has consumed source p's region (sequence number)
};

size_t mailbox_bytes(uint32_t npes) {
    const size_t flags = size_t(npes) * npes * 2 * 8;
    return (sizeof(MbHeader) + sizeof(PeSlot) * npes + 3 * flags + 4095) & ~size_t(4095);
}

Mailbox carve(void* base, uint32_t npes) {
    Mailbox m;
    uint8_t* p = static_cast<uint8_t*>(base);
    m.hdr = reinterpret_cast<MbHeader*>(p);
    p += sizeof(MbHeader);
    m.slots = reinterpret_cast<PeSlot*>(p);
    p += sizeof(PeSlot) * npes;
    const size_t flags = size_t(npes) * npes * 2;
    m.pub = reinterpret_cast<uint64_t*>(p);
    m.cnt = reinterpret_cast<int64_t*>(p + flags * 8);
    m.freed = reinterpret_cast<uint64_t*>(p + 2 * flags * 8);
    return m;
}

inline uint64_t ld_acq(const volatile uint64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void st_rel(volatile uint64_t* p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }

double now_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return double(t.tv_sec) + 1e-9 * double(t.tv_nsec);
}

// spin on the host until pred() holds (timeout: the peers never arrived)
template <typename F>
bool host_wait(F&& pred, double timeout_s) {
    const double t0 = now_s();
    uint32_t spins = 0;
    while (!pred()) {
        if (++spins > 1024) {
            if (now_s() - t0 > timeout_s) return false;
            usleep(20);
        }
    }
    return true;
}

double peer_timeout_s() {
    const char* e = getenv("LAMELLAR_PEER_TIMEOUT");
    const double v = (e && *e) ? atof(e) : 120.0;
    return v > 0 ? v : 120.0;
}

// ---- device side: waits on, and stores of, mailbox words (fine-grained host memory).
// A wait is one wave; every lane watches some of the words and gives up after `ticks` of the
// 100 MHz wall clock with LMR_ERRBIT_TRANSPORT set, so a PE that never arrives cannot hang the
// GPU (every wave reaches an exit).
__global__ void k_peer_wait(const uint64_t* words, uint32_t n, uint32_t stride, uint64_t want, uint32_t* err,
                            uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint64_t* w = words + uint64_t(i) * stride;
        while (__hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
            if (wall_clock64() - t0 > ticks) {
                raise_err(err, LMR_ERRBIT_TRANSPORT);
                return;
            }
            __builtin_amdgcn_s_sleep(16);
        }
    }
}

// source `me` publishes chunk `seq` to every owner q: the count its pack reserved in q's region
// (fill[q], past-capacity records included: the owner clamps), then the sequence number
__global__ void k_peer_publish(const uint32_t* fill, uint32_t npes, int64_t* cnt, uint64_t* pub, uint32_t stride,
                               uint64_t seq) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= npes) return;
    __hip_atomic_store(cnt + uint64_t(q) * stride, int64_t(fill ? fill[q] : 0u), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __hip_atomic_store(pub + uint64_t(q) * stride, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// owner `me` has consumed every source's region of sequence `seq`
__global__ void k_peer_free(uint64_t* freed, uint32_t npes, uint32_t stride, uint64_t seq) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npes) return;
    __threadfence_system();
    __hip_atomic_store(freed + uint64_t(p) * stride, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the pointer tables written from kernel arguments (no copy engine at set-up)
struct PeerTabArgs {
    uint8_t* p[4 * kPeerMaxPes];
};
__global__ void k_peer_tables(PeerTabArgs a, uint8_t** tab, uint32_t n) {
    const uint32_t i = threadIdx.x;
    if (i < n) tab[i] = a.p[i];
}

}  // namespace

struct PeerTransport {
    lmr_transport_t tp;                   // first: the exchange sees an lmr_transport_t
    uint64_t magic = kPeerMagic;
    const lmr_transport_t* base = nullptr;
    int device = 0;
    uint32_t npes = 0, me = 0;
    uint64_t R = 0;                       // records per receive region
    // mailbox
    char name[96] = {0};
    void* shm = nullptr;
    size_t shm_bytes = 0;
    Mailbox mb{};                         // host view
    Mailbox mbd{};                        // device view (registered mapping)
    // receive regions: this PE's [source][parity * 2 + kind] (R x 8 bytes each), and, per peer q,
    // q's regions for this PE as the source, as mapped here
    std::vector<uint8_t*> local;
    std::vector<uint8_t*> mapped;         // [q][parity * 2 + kind]; own entries point into `local`
    uint8_t** d_tab = nullptr;            // [2 parities][idx | vals][npes] device pointer tables
    uint64_t bseq = 0;                    // batches handshaken so far
    uint64_t last_pub[2] = {0, 0};        // sequence number last published into each parity's regions
    uint64_t pushed = 0;                  // chunks pushed (lmr_transport_peer_stats)
};

namespace {

inline size_t flag_index(uint32_t npes, uint32_t q, uint32_t p, int b) {
    return (size_t(q) * npes + p) * 2 + size_t(b);
}


// forwarded collectives (the base transport's): every path other than the push
lmr_status_t peer_alltoall(void* self, const void* send, void* recv, uint64_t bytes, lmr_stream_t s) {
    const PeerTransport* t = static_cast<const PeerTransport*>(self);
    return t->base->alltoall(t->base->self, send, recv, bytes, s);
}
lmr_status_t peer_alltoallv(void* self, const void* send, const uint64_t* sb, const uint64_t* so, void* recv,
                            const uint64_t* rb, const uint64_t* ro, uint32_t unit, lmr_stream_t s) {
    const PeerTransport* t = static_cast<const PeerTransport*>(self);
    return t->base->alltoallv(t->base->self, send, sb, so, recv, rb, ro, unit, s);
}

void peer_teardown(PeerTransport* t) {
    for (size_t i = 0; i < t->mapped.size(); i++)
        if (i / kRegionAllocs != t->me && t->mapped[i]) (void)hipIpcCloseMemHandle(t->mapped[i]);
    if (t->d_tab) (void)hipFree(t->d_tab);
    for (uint8_t* l : t->local)
        if (l) (void)hipFree(l);
    if (t->shm) {
        (void)hipHostUnregister(t->shm);
        munmap(t->shm, t->shm_bytes);
    }
    (void)hipGetLastError();
}

}  // namespace

PeerTransport* peer_of(const lmr_transport_t* tp) {
    if (!tp || !(tp->flags & LMR_TRANSPORT_PEER) || tp->alltoall != peer_alltoall) return nullptr;
    PeerTransport* t = static_cast<PeerTransport*>(tp->self);
    return (t && t->magic == kPeerMagic) ? t : nullptr;
}

uint64_t peer_region_records(const PeerTransport* t) { return t->R; }

lmr_status_t peer_handshake(PeerTransport* t, const int64_t* my_info, std::vector<int64_t>& all) {
    const uint64_t seq = ++t->bseq;
    const int b = int(seq & 1);
    PeSlot* me = &t->mb.slots[t->me];
    for (int i = 0; i < kInfoWords; i++) me->info[b][i] = my_info[i];
    st_rel(&me->bseq[b], seq);
    const double to = peer_timeout_s();
    all.assign(size_t(t->npes) * kInfoWords, 0);
    for (uint32_t p = 0; p < t->npes; p++) {
        PeSlot* s = &t->mb.slots[p];
        if (!host_wait([&] { return ld_acq(&s->bseq[b]) == seq; }, to)) return LMR_E_HIP;
        for (int i = 0; i < kInfoWords; i++) all[size_t(p) * kInfoWords + i] = s->info[b][i];
    }
    return LMR_OK;
}

uint8_t* const* peer_idx_table(const PeerTransport* t, int b) { return t->d_tab + size_t(b) * 2 * t->npes; }
uint8_t* const* peer_vals_table(const PeerTransport* t, int b) { return t->d_tab + (size_t(b) * 2 + 1) * t->npes; }

const uint8_t* peer_recv_idx(const PeerTransport* t, uint32_t src, int b) {
    return t->local[size_t(src) * kRegionAllocs + size_t(b) * 2];
}
const uint8_t* peer_recv_vals(const PeerTransport* t, uint32_t src, int b) {
    return t->local[size_t(src) * kRegionAllocs + size_t(b) * 2 + 1];
}
const int64_t* peer_recv_count(const PeerTransport* t, uint32_t src, int b) {
    return t->mbd.cnt + flag_index(t->npes, t->me, src, b);
}

static uint64_t peer_ticks() { return uint64_t(peer_timeout_s() * 1e8); }   // 100 MHz wall clock

hipError_t peer_wait_freed(PeerTransport* t, int b, uint32_t* err, hipStream_t s) {
    if (t->last_pub[b] == 0) return hipSuccess;            // the parity's regions were never used
    hipLaunchKernelGGL(k_peer_wait, dim3(1), dim3(64), 0, s, t->mbd.freed + flag_index(t->npes, 0, t->me, b),
                       t->npes, uint32_t(2 * t->npes), t->last_pub[b], err, peer_ticks());
    return hipGetLastError();
}

hipError_t peer_publish(PeerTransport* t, int b, const uint32_t* fill, uint64_t seq, hipStream_t s) {
    hipLaunchKernelGGL(k_peer_publish, dim3((t->npes + 63) / 64), dim3(64), 0, s, fill, t->npes,
                       t->mbd.cnt + flag_index(t->npes, 0, t->me, b), t->mbd.pub + flag_index(t->npes, 0, t->me, b),
                       uint32_t(2 * t->npes), seq);
    t->last_pub[b] = seq;
    t->pushed++;
    return hipGetLastError();
}

hipError_t peer_wait_published(PeerTransport* t, int b, uint64_t seq, uint32_t* err, hipStream_t s) {
    hipLaunchKernelGGL(k_peer_wait, dim3(1), dim3(64), 0, s, t->mbd.pub + flag_index(t->npes, t->me, 0, b), t->npes,
                       2u, seq, err, peer_ticks());
    return hipGetLastError();
}

hipError_t peer_mark_free(PeerTransport* t, int b, uint64_t seq, hipStream_t s) {
    hipLaunchKernelGGL(k_peer_free, dim3((t->npes + 63) / 64), dim3(64), 0, s,
                       t->mbd.freed + flag_index(t->npes, t->me, 0, b), t->npes, 2u, seq);
    return hipGetLastError();
}

uint64_t peer_chunk_seq(const PeerTransport* t, uint64_t j) { return (t->bseq << 24) + j + 1; }

}  // namespace lmr

using namespace lmr;

extern "C" {

lmr_status_t lmr_transport_peer_create(const lmr_transport_t* base, const char* job, uint64_t region_records,
                                       int device, lmr_transport_t** out) {
    if (!base || !job || !*job || !out || base->num_pes == 0 || base->num_pes > kPeerMaxPes ||
        base->my_pe >= base->num_pes || strlen(job) > 64 || strchr(job, '/'))
        return LMR_E_INVALID;
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return LMR_E_HIP;
    PeerTransport* t = new PeerTransport();
    t->base = base;
    t->device = device;
    t->npes = base->num_pes;
    t->me = base->my_pe;
    if (region_records == 0) {                             // one default chunk's region
        const uint64_t c = exchange_chunk_records();
        const uint64_t q = (c + t->npes - 1) / t->npes;
        region_records = q + q / 8 + 4096;
    }
    t->R = region_records;
    snprintf(t->name, sizeof t->name, "/lmr_peer_%s", job);
    const double to = peer_timeout_s();
    static const bool dbg = getenv("LMR_PEER_DEBUG") != nullptr;
    const double t_start = now_s();
    auto step = [&](const char* what) {
        if (dbg) fprintf(stderr, "[lmr_peer pe%u %.3f s] %s\n", t->me, now_s() - t_start, what);
    };
    auto fail = [&](lmr_status_t st) {
        peer_teardown(t);
        if (t->me == 0 && t->shm) shm_unlink(t->name);
        delete t;
        return st;
    };
    step("mailbox");
    // ---- the mailbox: PE 0 creates the segment, the others open it
    t->shm_bytes = mailbox_bytes(t->npes);
    int fd = -1;
    if (t->me == 0) {
        shm_unlink(t->name);                                // a stale segment of a killed job
        fd = shm_open(t->name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, off_t(t->shm_bytes)) != 0) {
            if (fd >= 0) close(fd);
            return fail(LMR_E_HIP);
        }
    } else if (!host_wait([&] { return (fd = shm_open(t->name, O_RDWR, 0600)) >= 0; }, to)) {
        return fail(LMR_E_HIP);
    }
    step("opened shm");
    void* m = mmap(nullptr, t->shm_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return fail(LMR_E_HIP);
    t->shm = m;
    t->mb = carve(m, t->npes);
    if (t->me == 0) {
        memset(m, 0, t->shm_bytes);
        t->mb.hdr->magic = kPeerMagic;
        t->mb.hdr->npes = t->npes;
        st_rel(&t->mb.hdr->created, 1);
    } else {
        if (!host_wait([&] { return ld_acq(&t->mb.hdr->created) == 1 && t->mb.hdr->magic == kPeerMagic; }, to) ||
            t->mb.hdr->npes != t->npes)
            return fail(LMR_E_HIP);
    }
    step("mailbox ready");
    // device view of the mailbox (fine-grained: system-scope loads / stores cross GPUs and processes)
    if (hipHostRegister(m, t->shm_bytes, hipHostRegisterMapped) != hipSuccess) {
        t->shm = nullptr;
        munmap(m, t->shm_bytes);
        return fail(LMR_E_HIP);
    }
    void* md = nullptr;
    if (hipHostGetDevicePointer(&md, m, 0) != hipSuccess) return fail(LMR_E_HIP);
    t->mbd = carve(md, t->npes);
    step("registered");
    // ---- receive regions: [source][parity][index | values], R x 8 bytes each
    // memory kind (LMR_PEER_REGION_MEM): uncached by default -- the owner's loads never meet a line
    // its L2 kept from the region's previous use while a peer rewrote it over xGMI -- or "fine"
    // (fine-grained, coherent) on request. Plain (coarse-grained) HBM is not offered: a peer's
    // stores over xGMI do not invalidate the owner's L2, and neither does a kernel-boundary acquire,
    // so the owner could stage stale records; it measured the same only because every run was on one
    // GPU (6.22 / 6.26 / 6.27 ms, profiles/r5/c4/peer_region_mem.txt). Cross-GPU visibility of the
    // two offered kinds is unverified until a multi-GPU run checks it.
    const char* mk = getenv("LMR_PEER_REGION_MEM");
    const unsigned mflags = (mk && mk[0] == 'f') ? hipDeviceMallocFinegrained : hipDeviceMallocUncached;
    t->local.assign(size_t(t->npes) * kRegionAllocs, nullptr);
    for (auto& l : t->local)
        if (hipExtMallocWithFlags(reinterpret_cast<void**>(&l), t->R * 8, mflags) != hipSuccess) return fail(LMR_E_HIP);
    step("regions allocated");
    PeSlot* mine = &t->mb.slots[t->me];
    for (uint32_t src = 0; src < t->npes; src++)
        for (int k = 0; k < kRegionAllocs; k++)
            if (hipIpcGetMemHandle(&mine->handle[src][k], t->local[size_t(src) * kRegionAllocs + k]) != hipSuccess)
                return fail(LMR_E_HIP);
    mine->region_recs = t->R;
    st_rel(&mine->ready, 1);
    step("handles exported");
    for (uint32_t p = 0; p < t->npes; p++) {
        PeSlot* s = &t->mb.slots[p];
        if (!host_wait([&] { return ld_acq(&s->ready) == 1; }, to) || s->region_recs != t->R) return fail(LMR_E_HIP);
    }
    // the PEs map their regions at each other one PE at a time, in PE order, each through its first
    // kernel on the tables (8 processes sharing one GPU that imported at once stalled there)
    for (uint32_t p = 0; p < t->me; p++)
        if (!host_wait([&] { return ld_acq(&t->mb.slots[p].mapped) == 1; }, to)) return fail(LMR_E_HIP);
    t->mapped.assign(size_t(t->npes) * kRegionAllocs, nullptr);
    for (uint32_t q = 0; q < t->npes; q++)
        for (int k = 0; k < kRegionAllocs; k++) {
            uint8_t*& dst = t->mapped[size_t(q) * kRegionAllocs + k];
            if (q == t->me) {
                dst = t->local[size_t(t->me) * kRegionAllocs + k];
                continue;
            }
            void* pp = nullptr;
            if (hipIpcOpenMemHandle(&pp, t->mb.slots[q].handle[t->me][k], hipIpcMemLazyEnablePeerAccess) != hipSuccess)
                return fail(LMR_E_HIP);
            dst = static_cast<uint8_t*>(pp);
        }
    step("peers mapped");
    // pointer tables: destination q's regions for this PE as the source, per parity
    std::vector<uint8_t*> tab(size_t(4) * t->npes);
    for (int b = 0; b < 2; b++)
        for (uint32_t q = 0; q < t->npes; q++) {
            tab[size_t(b) * 2 * t->npes + q] = t->mapped[size_t(q) * kRegionAllocs + size_t(b) * 2];
            tab[(size_t(b) * 2 + 1) * t->npes + q] = t->mapped[size_t(q) * kRegionAllocs + size_t(b) * 2 + 1];
        }
    if (hipMalloc(&t->d_tab, tab.size() * sizeof(uint8_t*)) != hipSuccess) return fail(LMR_E_HIP);
    step("table allocated");
    PeerTabArgs ta{};
    for (size_t i = 0; i < tab.size(); i++) ta.p[i] = tab[i];
    hipLaunchKernelGGL(k_peer_tables, dim3(1), dim3(4 * kPeerMaxPes), 0, nullptr, ta, t->d_tab, uint32_t(tab.size()));
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(nullptr) != hipSuccess) return fail(LMR_E_HIP);
    step("tables");
    // the next PE maps only once this one's first kernel after its imports has completed
    st_rel(&mine->mapped, 1);
    st_rel(&mine->opened, 1);
    for (uint32_t p = 0; p < t->npes; p++)
        if (!host_wait([&] { return ld_acq(&t->mb.slots[p].opened) == 1; }, to)) return fail(LMR_E_HIP);
    step("all opened");
    t->tp.num_pes = t->npes;
    t->tp.my_pe = t->me;
    t->tp.host_buffers = base->host_buffers;
    t->tp.flags = base->flags | LMR_TRANSPORT_PEER;
    t->tp.self = t;
    t->tp.alltoall = peer_alltoall;
    t->tp.alltoallv = peer_alltoallv;
    *out = &t->tp;
    return LMR_OK;
}

lmr_status_t lmr_transport_peer_stats(const lmr_transport_t* tp, uint64_t* batches, uint64_t* pushed_chunks) {
    const PeerTransport* t = peer_of(tp);
    if (!t) return LMR_E_INVALID;
    if (batches) *batches = t->bseq;
    if (pushed_chunks) *pushed_chunks = t->pushed;
    return LMR_OK;
}

lmr_status_t lmr_transport_peer_destroy(lmr_transport_t* tp) {
    PeerTransport* t = peer_of(tp);
    if (!t) return LMR_E_INVALID;
    (void)hipSetDevice(t->device);
    (void)hipDeviceSynchronize();                          // the regions may still be written or read
    // every PE is done with every region before any is unmapped
    st_rel(&t->mb.slots[t->me].closing, 1);
    const double to = peer_timeout_s();
    for (uint32_t p = 0; p < t->npes; p++) (void)host_wait([&] { return ld_acq(&t->mb.slots[p].closing) == 1; }, to);
    const bool owner = t->me == 0;
    char name[96];
    memcpy(name, t->name, sizeof name);
    peer_teardown(t);
    if (owner) shm_unlink(name);
    delete t;
    return LMR_OK;
}

}  // extern "C"
