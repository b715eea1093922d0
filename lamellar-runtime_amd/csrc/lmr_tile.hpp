// lmr_tile.hpp — the tile sweep's shared types: work items, per-region ops and the
// arguments of the owner / delta tile kernels (lmr_tile.hip), planned in lmr_apply.hip.
#pragma once
#include "lmr_internal.hpp"

namespace lmr {

// ---- tile work plan --------------------------------------------------------
// Most tiles are one work item in "owner" mode (one workgroup stages the tile
// in LDS, applies every record, writes the tile back). A tile with far more
// records than average (skewed streams, e.g. Zipf 0.99: ~5 % of all records on
// one element) is split into kSplit-record items in "delta" mode when the op
// combines (add/sub/and/or/xor and their fetch forms): each workgroup combines
// its records in an LDS delta tile (identity-initialised), then applies one
// device-scope atomic per touched element; fetch results are the returned base
// combined with the record's LDS prefix — a valid linearisation with each
// workgroup's records applied as one block.
constexpr uint32_t kSplit = 16 * 1024;     // records per delta item (16 per thread)
#ifndef LMR_WAVE_COMBINE
#define LMR_WAVE_COMBINE 1
#endif
constexpr bool kWaveCombine = LMR_WAVE_COMBINE != 0;   // lds_acc_wave in the delta pass (A/B builds: -DLMR_WAVE_COMBINE=0)

struct TileItem { uint32_t tile, lo, hi, mode; };

// a mixed staged session's per-region op (k_tile_owner applies region rg's records with rop[rg])
struct RegionOp {
    int32_t op, ret;
    uint64_t cmp_bits, eps_bits;
};

struct TileArgs {
    void* shard;
    uint64_t shard_len;
    int tile_shift;
    int kind;
    int op;
    int ret;
    uint64_t cmp_bits;
    uint64_t eps_bits;
    uint64_t val_bits;       // scalar value (SVMI)
    bool scalar;
    const TileItem* items;        // one per tile (owner kernel)
    const TileItem* delta;        // delta pieces (delta kernel)
    const uint32_t* delta_count;  // number of delta pieces (device)
    uint32_t num_tiles;
    const uint16_t* bin_lidx;
    const uint8_t* bin_val;
    void* results;           // binned order: [r] (un-partitioned by k_unpartition)
    uint8_t* ok;             // binned order
    uint32_t* err;
    // staged apply: an owner item covers tile t of every region r, records
    // [rts[r * rstride + t], rts[r * rstride + t + 1]); nreg == 0: the item's own [lo, hi)
    const uint32_t* rts;
    uint32_t nreg;
    uint32_t rstride;
    // mixed session (regions of different ops / operands): region rg applied with rop[rg], every
    // region of the tile after the previous one (staging order per element)
    int mixed;
    RegionOp rop[kMaxRegions];
    // the wide path's packed records (1/2/4-byte elements): bin_val holds one uint2 per record,
    // {tile-local index, value bits}, and bin_lidx is unused
    int packed = 0;
};

__host__ __device__ constexpr bool op_combines(int op) {
    return op == LMR_OP_ADD || op == LMR_OP_FETCH_ADD || op == LMR_OP_SUB || op == LMR_OP_FETCH_SUB ||
           op == LMR_OP_AND || op == LMR_OP_FETCH_AND || op == LMR_OP_OR || op == LMR_OP_FETCH_OR ||
           op == LMR_OP_XOR || op == LMR_OP_FETCH_XOR;
}

// k_tile_owner over every tile (+ k_tile_delta over the delta pieces when `delta`, on the
// side lane when there is one: the two kernels touch disjoint tiles and records);
// opt: LMR_OP_ADD / LMR_OP_FETCH_ADD select the specialised kernels, anything else the
// generic op switch
// tile_bytes: kTileBytes, or kWideBytes (the wide staged path's tiles of LDS words)
hipError_t launch_tile_kernels(int dtype, int opt, const TileArgs& t, bool delta, unsigned dgrid, hipStream_t s,
                               const SideLane& side, uint32_t tile_bytes = kTileBytes);

}  // namespace lmr
