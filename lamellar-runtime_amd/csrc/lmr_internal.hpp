// lmr_internal.hpp — host-side internals shared by the .hip translation units
// of liblamellar_gpu_ops.so (not part of the C ABI).
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <functional>
#include <vector>
#include "../../include/lamellar_gpu_ops.h"

namespace lmr { struct Prof; }

namespace lmr { struct HostStage; void host_stage_free(HostStage* h); }
namespace lmr { struct StageState; void stage_state_free(StageState* s); void stage_abort(StageState* s); }
namespace lmr { struct XState; void xstate_free(XState* x); }
namespace lmr { struct WinState; void win_state_free(WinState* w); }
namespace lmr { struct WireBufs; void wire_bufs_free(WireBufs* b); }
namespace lmr { struct OrdBufs; void ord_bufs_free(OrdBufs* b); }

struct lmr_ctx {
    int device = 0;
    uint32_t* d_err = nullptr;     // device error word (LMR_ERRBIT_*)
    // tiled-apply / pack workspace (allocated by lmr_ctx_reserve, never on the hot path)
    uint8_t* ws = nullptr;
    uint8_t* ws_alloc = nullptr;   // the allocation ws lies in (hipFree)
    size_t ws_bytes = 0;
    uint64_t rec_cap = 0;          // records one tiled piece may hold
    int num_cus = 256;
    lmr::Prof* prof = nullptr;     // stage timing (lmr_ctx_profile), null when off
    lmr::HostStage* host = nullptr;  // host-buffer ingestion staging (lmr_apply_mvmi_host), lazily made
    lmr::StageState* stage = nullptr;  // staged-apply session (lmr_stage_*), lazily made
    lmr::XState* xch = nullptr;        // multi-PE exchange state (lmr_batch_exchange), lazily made
    bool xdefer_on = false;            // lmr_ctx_exchange_defer
    bool xdefer_open = false;          // the open staged session was left by a deferred exchange
    lmr::WinState* win = nullptr;      // window partition of shards above one tiled window, lazily made
    lmr::WireBufs* wire = nullptr;     // staging of lmr_apply_msg (AM wire format), lazily made
    lmr::OrdBufs* ord = nullptr;       // sort buffers of the ordered apply (n > 1024), see ord_reserve
    // side lane of the tile sweep: the delta pieces of hot tiles run beside the owner tiles
    hipStream_t side = nullptr;
    hipEvent_t side_fork = nullptr, side_join = nullptr;
};

namespace lmr {

// Events that only order kernels on two streams of one device (the side lane) or only time
// kernels (stage profiling) need no system-scope fence; LMR_EVENT_SCOPE=system keeps HIP's
// default one (A/B).
inline bool device_scope_events() {
    static const bool on = [] {
        const char* v = getenv("LMR_EVENT_SCOPE");
        return !(v && v[0] == 's');
    }();
    return on;
}
inline unsigned side_event_flags() {
    return hipEventDisableTiming | (device_scope_events() ? hipEventDisableSystemFence : 0u);
}

// ---- tiling constants (gfx950: 160 KiB LDS per CU; two 64 KiB tiles per CU) ----
constexpr int kTileBytes = 64 * 1024;
constexpr int kMaxTiles = 16384;          // LDS histogram of 64 KiB u32 counters
constexpr int kBinBlock = 1024;           // threads per bin/scatter block
constexpr int kMaxBinBlocks = 1024;       // G: blocks of the bin passes
constexpr int kScanItems = 4096;          // elements per scan block (1024 threads x 4)
constexpr int kMaxPackPes = 512;
constexpr int kMaxWindows = 256;          // tiled windows per shard (lmr_window.hip)
constexpr int kMaxRegions = 32;           // staged-apply regions per session
constexpr int kStageInfoWords = 512;      // staged-apply piece table + per-region totals (u32)
constexpr uint64_t kStageMaxRegion = uint64_t(1) << 30;   // records per staged region
// the one-level ("wide") staged partition (lmr_wide.hip): 128 KiB tiles of LDS words
constexpr int kWideShift8 = 14;           // 8-byte elements per wide tile: 2^14 x 8 B
constexpr int kWideShift4 = 15;           // 1/2/4-byte elements (32-bit LDS words): 2^15 x 4 B
constexpr uint32_t kWideBytes = 128 * 1024;
constexpr uint32_t kWideMaxTiles = 1024;  // 8-byte elements: a shard of at most 2^24 elements
constexpr uint32_t kWideMaxTiles4 = 2048; // 1/2/4-byte elements: at most 2^26 elements
inline int wide_shift(int dtype_b) { return dtype_b == 8 ? kWideShift8 : kWideShift4; }

// ---- stage timing: HIP events around kernel stages (see lmr_ctx_profile) ----
// n: records the stage processes (reported per stage by lmr_ctx_profile_read)
void prof_begin(Prof* p, int stage, hipStream_t s);
void prof_end(Prof* p, int stage, hipStream_t s, uint64_t n);
struct ProfScope {
    Prof* p; int st; hipStream_t s; uint64_t n;
    ProfScope(Prof* p_, int st_, hipStream_t s_, uint64_t n_ = 0) : p(p_), st(st_), s(s_), n(n_) {
        if (p) prof_begin(p, st, s);
    }
    ~ProfScope() { end(); }
    void end() { if (p) prof_end(p, st, s, n); p = nullptr; }
};

// A second stream (and its fork / join events) a launch may run independent work on.
struct SideLane {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
};

// Workspace carve-up of one tiled piece.
struct TiledWs {
    uint32_t* counts;      // [num_tiles * G]
    uint32_t* partials;    // scan block partials
    uint32_t* tile_start;  // [num_tiles + 1]
    uint16_t* bin_lidx;    // [cap]
    uint8_t* bin_val;      // [cap * 8]
    uint32_t* rpos;        // [cap] temp (two-level) or record (one-level) -> binned position
    uint32_t* total;       // [1]
    uint32_t* coarse_off;  // [kMaxTiles/128 * G + 1]  (two-level partition)
    uint32_t* tmp_idx;     // [cap]
    uint8_t* tmp_val;      // [cap * 8]
    uint32_t* qpos;        // [cap] record -> temp position (two-level)
    uint32_t* tile_items;  // [kMaxTiles + 1] work items per tile, then their exclusive scan
    uint32_t* tile_items2; // [kMaxTiles + 1] work items per tile
    uint32_t* plan_partials;
    uint32_t* item_count;  // [1]
    uint8_t* items;        // TileItem[kMaxTiles] owner items, then delta pieces
    uint32_t* rts;         // staged apply: [kMaxRegions][kMaxTiles + 1] tile starts of each region
    uint32_t* sinfo;       // staged apply: piece table (pbase, bstart) + per-region in-bounds totals
    uint32_t* ff;          // count-free partition: bucket and tile fill counters
    uint32_t* runtab;      // staged apply: per fine round, per tile (binned run start, length)
    uint32_t* ptab;        // staged apply: [kMaxRegions][2 * (kMaxCoarse + 1)] piece tables
    uint64_t rt_rounds;    // rounds runtab holds
    uint32_t* crtab;       // staged apply: per coarse round, per bucket (temp run start, length)
    uint64_t crt_rounds;   // rounds crtab holds
    uint32_t* rtot;        // staged apply: [kMaxRegions][kMaxTiles] each region's tile totals
    uint32_t* rfill;       // staged apply: [kMaxRegions][kMaxTiles] each region's fine-pass tile fills
    uint64_t cap;          // records of one tiled piece (bin arrays, position maps)
    uint64_t tmp_cap;      // records the temp arrays (tmp_idx / tmp_val) hold, > cap
    SideLane side;         // the context's side lane (null: everything on the launch stream)
};
size_t tiled_ws_bytes(uint64_t cap);
// largest workspace capacity (records) whose temp slots fit the kernels' uint32 slot math
uint64_t max_rec_cap();
TiledWs carve_tiled_ws(uint8_t* base, uint64_t cap);

// exclusive scan of d[0..m) in place; *d_total = sum (may be null). partials: the
// look-back scratch, scan_scratch_words(m) u32 words, 8-byte aligned, zeroed once when
// allocated (every scan leaves it zeroed). only_if non-null: the launch does nothing
// unless *only_if != 0 when it runs (device-side condition).
uint64_t scan_scratch_words(uint64_t m);
hipError_t scan_exclusive_u32(uint32_t* d, uint64_t m, uint32_t* partials, uint32_t* d_total,
                              hipStream_t s, const uint32_t* only_if = nullptr);

struct ApplyArgs {
    void* shard;
    uint64_t shard_len;
    int kind;
    int op;
    int ret;
    uint64_t cmp_bits;
    uint64_t eps_bits;
    uint32_t* err;
    // records: index k at idx + k*idx_stride (bytes); value at val + k*val_stride,
    // or the scalar `val_bits` when val == nullptr (single value, many indices)
    const uint8_t* idx;
    uint64_t idx_stride;
    const uint8_t* val;
    uint64_t val_stride;
    uint64_t val_bits;
    uint64_t n;
    void* results;   // T per record (ret != NONE)
    uint8_t* ok;     // per record (ret == RESULT)
    Prof* prof;
};

// launchers (dtype-dispatching), defined in lmr_apply.hip
hipError_t launch_apply_direct(int dtype, int index_size, const ApplyArgs& a, hipStream_t s);
hipError_t launch_apply_mvsi(int dtype, const ApplyArgs& a, uint64_t index, hipStream_t s);
// LMR_STRATEGY_ORDERED (lmr_ordered.hip): per element in record order, one atomic block each
hipError_t launch_apply_ordered(lmr_ctx* ctx, int dtype, int index_size, const ApplyArgs& a, hipStream_t s);
constexpr uint64_t kOrderedAuto = 1000;   // AUTO: below this many records (one reference AM at 1 PE)
// sort buffers of the ordered apply: one piece of records (lmr_ctx_create reserves the minimum,
// lmr_ctx_reserve up to the maximum); larger calls run piece after piece
constexpr uint64_t kOrderedMinPiece = uint64_t(1) << 16;
constexpr uint64_t kOrderedMaxPiece = uint64_t(1) << 22;
hipError_t ord_reserve(lmr_ctx* ctx, uint64_t recs);
// tiled apply of SoA/AoS records; returns hipErrorNotSupported when the shard
// is too large for the single-level tile histogram.
hipError_t launch_apply_tiled(int dtype, int index_size, const ApplyArgs& a, const TiledWs& w,
                              hipStream_t s);
bool tiled_supported(int dtype, uint64_t shard_len);
// log2 of the elements of one 64 KiB shard tile
int tile_shift(int dtype);
// elements of one tiled window (kMaxTiles tiles)
uint64_t tiled_window_len(int dtype);
// Shards above one window: partition the records by window, apply each window's
// records with apply_one (its slice of the shard as desc; u32 window-local offsets),
// then results back to input order. Host waits once per piece for the window counts.
using WindowApplyFn = std::function<hipError_t(const lmr_apply_desc_t*, const ApplyArgs&, hipStream_t)>;
// true when the two-level partition's per-(bucket, producer block) segments of an
// n-record piece would be short (< 8192 records) and fixed-size pieces pay
bool piece_partition_pays(int dtype, uint64_t shard_len, uint64_t n);
// true when a one-shot tiled piece of n records (workspace capacity cap) takes the
// count-free partition: order-insensitive integer op, nothing returned
bool free_partition_applies(int dtype, int op, int ret, uint64_t shard_len, uint64_t n, uint64_t cap);

// Staged (deferred) tiled apply: each record stream ("region") is partitioned
// into shard tiles on arrival, all regions are applied in one tile sweep.
struct StageRegion {
    uint64_t base;       // first workspace slot of the region
    uint64_t n;          // records (slots) of the region
    void* results;       // caller's per-record results (arrival order), may be null
    uint8_t* ok;         // caller's per-record Ok flags, may be null
    int op;              // the region's op and operands (mixed sessions: one op phase per run of
    int ret;             // regions with equal op / operands, applied in staging order)
    uint64_t cmp_bits;
    uint64_t eps_bits;
    uint32_t round_base = 0;   // first runtab round of the region (returning regions)
    uint32_t kround = 0;       // the fine pass's LDS round (records)
    uint32_t nrounds = 0;      // runtab rounds reserved for the region (0: no run table)
    uint32_t cround_base = 0;  // first crtab round of the region
    uint32_t ncrounds = 0;     // crtab rounds reserved (producer blocks x rounds per block; 0: none)
    uint32_t rpb = 0;          // coarse rounds per producer block
    uint32_t kcround = 0;      // the coarse pass's LDS round (records)
    uint64_t chunk = 0;        // records per producer block
    // wide sessions (lmr_wide.hip): the region's scanned (tile, block) slices in counts, its
    // per-round tile counts in rpos (u16 offset), producer blocks, the group's binned base
    uint64_t wcnt = 0, wrh = 0;
    uint32_t wg = 0, wbase = 0;
    bool wres = false;         // qpos / round counts kept (a returning region)
};
struct PendingRegion {
    ApplyArgs a;         // the region's records (caller buffers, valid until the region is partitioned)
    int iw;
    const int64_t* n_dev = nullptr;   // count-free only: record count in device memory (a.n: capacity)
};
struct StageSession {
    ApplyArgs a;         // op / kind / shard / ret of the session's current op (record fields unused)
    int dtype = 0;
    int nreg = 0;
    int parted = 0;      // regions [0, parted) are partitioned; [parted, nreg) wait in pend[]
    uint64_t staged = 0; // workspace slots in use
    uint64_t rounds = 0; // runtab rounds in use
    uint64_t crounds = 0;  // crtab rounds in use
    bool free = false;   // count-free regions (stage_free_applies): shared bucket regions, one fine pass
    bool free_armed = false;
    uint32_t free_rows = 0;  // count-free sessions: tile-count rows the coarse launches used
    bool switched = false;  // the op changed with records staged (lmr_stage_op): later phases counted
    bool wide = false;      // counted regions partitioned one-level into 128 KiB tiles (wide_applies)
    bool wide_set = false;  //   decided at the session's first partition
    bool wpack = false;     // wide: packed records (TileArgs::packed: uint2 for 1/2/4-byte values, uint4 for 8-byte)
    uint64_t wcnt = 0;      // wide: count entries in use
    uint64_t wrh = 0;       // wide: round-count entries (u16) in use
    StageRegion reg[kMaxRegions];
    PendingRegion pend[kMaxRegions];
};
// true when a region staged under a different op / operands than `a`'s is pending
bool stage_pending_other_op(const StageSession& s, const ApplyArgs& a);
// true when a staged session of this op takes the count-free regions
bool stage_free_applies(int dtype, int op, int ret, uint64_t shard_len, uint64_t cap);
// add the records of `a` as the next region (caller checks capacity: s.staged + a.n <= workspace
// capacity, a.n <= kStageMaxRegion, s.nreg < kMaxRegions). Regions are only recorded:
// launch_stage_partition partitions every pending region at once (the caller's buffers stay valid
// until then).
hipError_t launch_stage_region(int dtype, int index_size, const ApplyArgs& a, const TiledWs& w,
                               StageSession& s, hipStream_t st);
hipError_t launch_stage_partition(const TiledWs& w, StageSession& s, hipStream_t st);
// a count-free session's region whose record count is in device memory (*n_dev, clamped to a.n,
// the region's capacity), accounted as `expect` records (the exchange's fixed receive regions)
hipError_t launch_stage_region_dev(int dtype, int index_size, const ApplyArgs& a, const int64_t* n_dev,
                                   uint64_t expect, const TiledWs& w, StageSession& s, hipStream_t st);
// apply every staged region in one tile sweep, results back to each region's caller
hipError_t launch_stage_finish(const TiledWs& w, StageSession& s, hipStream_t st);
// the wide path (lmr_wide.hip): applies to shards of <= kWideMaxTiles 128 KiB tiles of 8-byte
// elements (kWideMaxTiles4 for 1/2/4-byte elements) with a workspace whose rpos holds the round
// counts (LMR_WIDE=0 turns it off, LMR_WIDE4=0 for elements below 8 bytes, read per session);
// partition of the pending regions; the
// returning regions' results from binned order back to arrival order after the tile sweep
bool wide_applies(int dtype, uint64_t shard_len, uint64_t cap);
hipError_t wide_partition(const TiledWs& w, StageSession& s, hipStream_t st);
uint8_t* wide_records(const TiledWs& w, const StageSession& s);
hipError_t wide_unpartition(const TiledWs& w, const StageSession& s, const uint8_t* res_bin, const uint8_t* ok_bin,
                            uint32_t num_tiles, hipStream_t st);

// exchange-internal staging (lmr_capi.hip): the context's open session is count-free; a
// region of `cap` records at d_indices / d_vals whose record count is *d_n (device), accounted as
// `expect` records
bool stage_session_free(const lmr_ctx* ctx);
// a session is open / open for this descriptor (shard, element type, kind, op and operands)
bool stage_session_open(const lmr_ctx* ctx);
bool stage_session_of(const lmr_ctx* ctx, const lmr_apply_desc_t& d);
// no session open, or one with no region staged
bool stage_session_empty(const lmr_ctx* ctx);
lmr_status_t stage_soa_dev(lmr_ctx* ctx, const void* d_indices, uint32_t index_size, const void* d_vals,
                           const void* val, uint64_t cap, uint64_t expect, const int64_t* d_n, hipStream_t s);

// the exchange's default chunk (LAMELLAR_EXCHANGE_CHUNK records; lmr_exchange.hip)
uint64_t exchange_chunk_records();

// peer-memory transport (lmr_peer.hip): receive regions of R records per (source, parity) on every
// PE, IPC-mapped; a /dev/shm mailbox of per-chunk counts and sequence numbers
struct PeerTransport;
PeerTransport* peer_of(const lmr_transport_t* tp);               // null unless a peer transport
uint64_t peer_region_records(const PeerTransport* t);
// one host handshake per batch: every PE's 8 info words (all[p * 8 + i]); also advances the batch
// sequence that peer_chunk_seq numbers chunks from
lmr_status_t peer_handshake(PeerTransport* t, const int64_t* my_info, std::vector<int64_t>& all);
uint64_t peer_chunk_seq(const PeerTransport* t, uint64_t j);
uint8_t* const* peer_idx_table(const PeerTransport* t, int b);   // device: destination q's region (this PE the source)
uint8_t* const* peer_vals_table(const PeerTransport* t, int b);
const uint8_t* peer_recv_idx(const PeerTransport* t, uint32_t src, int b);   // this PE's region for `src`
const uint8_t* peer_recv_vals(const PeerTransport* t, uint32_t src, int b);
const int64_t* peer_recv_count(const PeerTransport* t, uint32_t src, int b); // device view of its count
hipError_t peer_wait_freed(PeerTransport* t, int b, uint32_t* err, hipStream_t s);     // parity b's regions reusable
hipError_t peer_publish(PeerTransport* t, int b, const uint32_t* fill, uint64_t seq, hipStream_t s);
hipError_t peer_wait_published(PeerTransport* t, int b, uint64_t seq, uint32_t* err, hipStream_t s);
hipError_t peer_mark_free(PeerTransport* t, int b, uint64_t seq, hipStream_t s);

// pack (lmr_pack.hip)
struct PackArgs {
    lmr_layout_t layout;
    const uint64_t* gidx;
    const uint8_t* vals;     // may be null (SVMI)
    uint32_t val_bytes;
    uint64_t n;
    uint32_t index_size;
    uint8_t* out_idx;
    uint8_t* out_vals;
    uint32_t* out_pos;
    uint64_t* dest_counts;   // [npes]
    uint64_t* dest_offsets;  // [npes + 1]
    uint32_t* err;
    Prof* prof;
    bool stable;             // true: input order within a PE (lmr_pack); false: LDS-staged runs
    // count-free pack only: records past their destination's region go to this list (global
    // index, value) instead of being dropped; ovf_count (device) counts them (null: no list)
    uint64_t* ovf_gidx = nullptr;
    uint8_t* ovf_vals = nullptr;
    uint32_t* ovf_count = nullptr;
    uint64_t ovf_cap = 0;
    // count-free pack only: destination i's region at out_idx_tab[i] / out_vals_tab[i] (device arrays;
    // the peer transport's IPC-mapped receive regions) instead of out_idx / out_vals + i * cap
    uint8_t* const* out_idx_tab = nullptr;
    uint8_t* const* out_vals_tab = nullptr;
    // count-free pack only: `fill` is zero on entry (no memset) and is left zero (the counts kernel
    // clears it after copying it to dest_counts): the exchange's per-chunk pack
    bool fill_zeroed = false;
};
hipError_t launch_pack(const PackArgs& a, uint32_t* counts, uint32_t* partials, uint32_t* total,
                       hipStream_t s);
// count-free unordered pack into fixed per-destination regions of `cap` records (nothing
// returned; dest_counts[i] > cap: region i overflowed: without an overflow list the output is
// incomplete (pack again with launch_pack); with one, region i holds its first cap records and the
// rest are in the list)
hipError_t launch_pack_free(const PackArgs& a, uint32_t* fill, uint32_t cap, hipStream_t s);

// the peer push's bucketed mode (lmr_bucket.hip): the sender packs by (owner, owner coarse bucket
// of 128 tiles) into bucket slices of the owner's receive region, the owner bins each chunk
// straight into fixed per-tile regions of a session swept once
constexpr uint32_t kBucketHdr = 4096;       // bytes of slice counts at the head of a bucketed index region (kBucketMaxKeys u32)
constexpr uint32_t kBucketMaxKeys = 1024;   // (owner, bucket) keys of the sender's pack
constexpr uint32_t kBucketMaxSrc = 16;      // PEs
struct BucketSession {
    bool open = false;
    lmr_apply_desc_t desc{};
    uint32_t T = 0, C = 0;   // the owner's tiles, buckets
    int tpb_log2 = 8;        // log2 of the tiles per bucket (bucket_tpb_log2)
    uint64_t cap_t = 0;      // records per fixed tile region (workspace temp arrays)
    uint64_t staged = 0;     // records expected in the session so far
    uint32_t* tfill = nullptr;   // device [kMaxTiles] tile fills (zero between sessions)
    uint32_t* err = nullptr;
    Prof* prof = nullptr;
};
struct BucketChunk {
    uint32_t S = 0;
    uint32_t cap_b[kBucketMaxSrc] = {};        // source s's slice capacity (records)
    const uint8_t* idx[kBucketMaxSrc] = {};   // source s's index area this chunk (null: nothing from s)
    const uint8_t* val[kBucketMaxSrc] = {};   // null: the scalar sbits[s]
    uint64_t sbits[kBucketMaxSrc] = {};
    uint64_t expect = 0;
};
// buckets of the layout's largest shard (false: the layout / element type cannot take the mode)
int bucket_tpb_log2();
// integer ops whose records commute (any split and order gives the same shard): the mode's ops
bool bucket_op_ok(int dtype, int op);
bool bucket_geometry(const lmr_layout_t& L, int dtype, uint32_t& C, int& cshift);
// records per bucket slice of a receive region of R records (8 bytes each, index and value areas)
uint32_t bucket_slice_cap(uint64_t R, uint32_t C, uint32_t eb);
// the sender's pack of one chunk (a.out_idx_tab / out_vals_tab: the owners' regions; or, with no
// table, a.out_idx / a.out_vals holding the owners' areas back to back, bucket_region_idx_bytes and
// C * cap_b * value bytes apart) and the slice
// counts into the owners' region headers; tot[q]: records written for owner q
hipError_t launch_pack_bucket(const PackArgs& a, uint32_t C, int cshift, uint32_t cap_b, uint32_t* fill,
                              uint32_t* tot, hipStream_t s);
// largest session (records) the fixed tile regions take with headroom
uint64_t bucket_session_limit(const BucketSession& bs);
hipError_t launch_fine_bucket(const BucketChunk& c, const BucketSession& bs, const TiledWs& w, hipStream_t st);
// an owner without a session workspace: the chunk's slices applied with device atomics
hipError_t launch_bucket_direct(const BucketChunk& c, const lmr_apply_desc_t& d, uint32_t C, int cshift, uint32_t* err,
                                hipStream_t st);
// bytes of a bucketed index area: the slice-count header and C slices of cap_b u32 offsets (values:
// C * cap_b * value bytes)
uint64_t bucket_region_idx_bytes(uint32_t C, uint32_t cap_b);
hipError_t launch_bucket_sweep(BucketSession& bs, const TiledWs& w, hipStream_t st);
constexpr int kReduceBlocks = 1024;
hipError_t launch_reduce(int dtype, int op, const void* x, uint64_t n, uint64_t* out, uint8_t* has,
                         void* part, uint8_t* part_has, hipStream_t s);
hipError_t launch_scatter_results(const uint8_t* in, const uint32_t* pos, uint64_t n,
                                  uint32_t elem_bytes, uint8_t* out, const uint8_t* ok_in,
                                  uint8_t* ok_out, Prof* prof, hipStream_t s);
hipError_t apply_windowed(lmr_ctx* ctx, const lmr_apply_desc_t* d, const ApplyArgs& a, int iw, hipStream_t s,
                          const WindowApplyFn& apply_one);

// The index width of an op AM's index_size byte: 1, 2, 4 or 8, and usize (8) for any other value,
// as the generated apply bodies' `_ =>` arm reads them (impl/src/array_ops.rs:867-897).
inline uint32_t am_index_width(uint32_t index_size) {
    return (index_size == 1 || index_size == 2 || index_size == 4) ? index_size : 8u;
}

inline int dtype_bytes(int d) {
    switch (d) {
    case LMR_U8: case LMR_I8: return 1;
    case LMR_U16: case LMR_I16: return 2;
    case LMR_U32: case LMR_I32: case LMR_F32: return 4;
    case LMR_U64: case LMR_I64: case LMR_F64: return 8;
    default: return 0;
    }
}

}  // namespace lmr
