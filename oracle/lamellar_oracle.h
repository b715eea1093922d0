/*
 * lamellar_oracle.h — CPU ORACLE FOR TESTS ONLY.
 *
 * This is test infrastructure: a plain-C restatement of pnnl/lamellar-runtime's
 * LamellarArray batched element-op path (index math, IndexSize narrowing, the
 * three pack shapes, the generated apply bodies, result reordering). Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it,
 * and only as the checker / the timed CPU baseline. The product path
 * (liblamellar_gpu_ops.so) never links or calls it.
 *
 * Parity pinning: the reference is Rust and cannot be built here (no cargo,
 * no vendored crates, no network — SURVEY.md §8(c)); it holds no golden
 * vectors. The oracle is pinned against the reference's own known-answer
 * tests (tests/array/...), restated in tests/test_oracle_known_answers.py.
 *
 * Every function cites the reference file:line it restates.
 */
#ifndef LAMELLAR_ORACLE_H
#define LAMELLAR_ORACLE_H

#include "../include/lamellar_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- layout / index math: src/array/unsafe.rs ---- */
int      orc_layout_new(lmr_layout_t* L, uint64_t array_size, uint32_t num_pes,
                        uint32_t my_pe, uint32_t distribution);                 /* :178-274 */
int      orc_layout_sub(const lmr_layout_t* parent, uint64_t start, uint64_t end,
                        lmr_layout_t* out);                                     /* :1259-1290 */
int      orc_full_pe_and_offset(const lmr_layout_t* L, uint64_t index,
                                uint64_t* pe, uint64_t* offset);               /* :1610-1647 */
int      orc_pe_for_dist_index(const lmr_layout_t* L, uint64_t index, uint64_t* pe); /* :1651-1673 */
int      orc_pe_full_offset_for_dist_index(const lmr_layout_t* L, uint64_t pe,
                                           uint64_t index, uint64_t* off);     /* :1677-1705 */
int      orc_pe_sub_offset_for_dist_index(const lmr_layout_t* L, uint64_t pe,
                                          uint64_t index, uint64_t* off);      /* :1708-1736 */
int      orc_pe_and_offset(const lmr_layout_t* L, uint64_t index,
                           uint64_t* pe, uint64_t* offset);                     /* :1207-1223 */
uint64_t orc_global_start_index_for_pe(const lmr_layout_t* L, uint64_t pe);    /* :1878-1886 */
int      orc_start_index_for_pe(const lmr_layout_t* L, uint64_t pe, uint64_t* out); /* :1889-1941 */
uint64_t orc_num_elems_pe(const lmr_layout_t* L, uint64_t pe);                 /* :1966-2016 */
uint64_t orc_local_slice_start(const lmr_layout_t* L, uint64_t pe);            /* :2023-2066 */
uint32_t orc_index_size(const lmr_layout_t* L);       /* unsafe/operations.rs:56-75, :300-304 */
uint32_t orc_record_bytes(uint32_t index_size, uint32_t dtype);  /* IdxVal repr(C), operations.rs:213-219 */
uint32_t orc_record_val_offset(uint32_t index_size, uint32_t dtype);
uint32_t orc_dtype_bytes(uint32_t dtype);
uint32_t orc_op_ret_kind(uint32_t op);                /* which handle each op builder returns */
int      orc_op_supported(uint32_t kind, uint32_t dtype, uint32_t op); /* src/array.rs:207-220 */

/* ---- apply of one op buffer (one AM's exec body): impl/src/array_ops.rs ----
 * `slice` is the (sub)array's local slice on the applying PE.
 * results: T per record for LMR_RET_VALS / LMR_RET_RESULT; ok: 1 = Ok, 0 = Err (RESULT only).
 * Records are applied sequentially in buffer order. Return: first error status. */
int orc_apply_mvmi(void* slice, uint64_t slice_len, uint32_t kind, uint32_t dtype,
                   uint32_t op, const void* cmp, const void* eps,
                   const void* idx_vals, uint64_t nbytes, uint32_t index_size,
                   void* results, uint8_t* ok);                 /* :863-899, 1041-1079, 1226-1264 */
int orc_apply_svmi(void* slice, uint64_t slice_len, uint32_t kind, uint32_t dtype,
                   uint32_t op, const void* cmp, const void* eps, const void* val,
                   const void* indices, uint64_t nbytes, uint32_t index_size,
                   void* results, uint8_t* ok);                 /* :929-967, 1109-1149, 1297-1343 */
int orc_apply_mvsi(void* slice, uint64_t slice_len, uint32_t kind, uint32_t dtype,
                   uint32_t op, const void* cmp, const void* eps,
                   const void* vals, uint64_t nbytes, uint64_t index,
                   void* results, uint8_t* ok);                 /* :999-1008, 1178-1190, 1378-1390 */

/* ---- pack: src/array/unsafe/operations.rs ----
 * One op buffer ("AM") descriptor, emitted in generation order: chunk by
 * chunk (operations.rs:462-480), inside a chunk a buffer is flushed when it
 * reaches bytes_per_batch (:759) and the partial buffers are flushed in PE
 * order at the end of the chunk (:779-797). */
typedef struct {
    uint32_t pe;
    uint32_t _pad;
    uint64_t byte_off;   /* into the bytes output */
    uint64_t nbytes;
    uint64_t nrec;
    uint64_t res_off;    /* into res_pos: input positions j of this buffer's records */
} orc_am_t;

uint64_t orc_num_chunks(uint64_t len, uint64_t batch_op_threads);             /* operations.rs:455-480 */
int64_t orc_pack_mvmi(const lmr_layout_t* L, uint32_t dtype, const uint64_t* gidx,
                      const void* vals, uint64_t n, uint32_t index_size,
                      uint64_t am_size_threshold, uint64_t batch_op_threads,
                      orc_am_t* ams, uint64_t max_ams, uint8_t* bytes, uint64_t bytes_cap,
                      uint64_t* res_pos, int* status);          /* :663-811 */
int64_t orc_pack_svmi(const lmr_layout_t* L, const uint64_t* gidx, uint64_t n,
                      uint32_t index_size, uint64_t am_size_threshold,
                      uint64_t batch_op_threads, orc_am_t* ams, uint64_t max_ams,
                      uint8_t* bytes, uint64_t bytes_cap, uint64_t* res_pos,
                      int* status);                             /* :479-587 */

/* ---- whole batch op, every PE simulated in one address space ----
 * pe_slices[p] = PE p's local slice of the (sub)array described by L.
 * Shape selection as initiate_batch_* (unsafe/operations.rs:290-477):
 * i_len==v_len==1 -> single, v_len>1 && i_len==1 -> MVSI, v_len==1 && i_len>1 -> SVMI,
 * both >1 -> MVMI (lengths must match: LMR_E_LENGTH otherwise).
 * Application order: input order (one valid linearisation of the reference). */
int orc_batch_op(const lmr_layout_t* L, void* const* pe_slices, uint32_t kind,
                 uint32_t dtype, uint32_t op, const void* cmp, const void* eps,
                 const uint64_t* gidx, uint64_t i_len, const void* vals, uint64_t v_len,
                 void* results, uint8_t* ok);

/* ---- reductions (impl/src/array_reduce.rs; UnsafeArray::reduce, unsafe.rs:1414-1557) ----
 * orc_reduce: one PE's step, `local_data().iter().reduce(op)` (array_reduce.rs:82-88) — a
 * sequential left fold with the closures of :283-319 (`acc + val`, `acc * val` wrapping as
 * release-mode Rust; `if a > b {a} else {b}`; `if a < b {a} else {b}`). *has = 0 for an
 * empty slice (None). op: 0 sum, 1 prod, 2 max, 3 min.
 * orc_reduce_tree: the cross-PE tree of :90-107 over per-PE (has, value) pairs: [lo, hi]
 * splits at mid = (lo + hi) / 2, a None side is the identity, op(left, right) otherwise. */
void orc_reduce(uint32_t dtype, uint32_t op, const void* data, uint64_t n, void* out, uint8_t* has);
void orc_reduce_tree(uint32_t dtype, uint32_t op, const void* vals, const uint8_t* has, uint32_t npes,
                     void* out, uint8_t* out_has);

/* ---- per-record step and the linearisability checker (linearize.c) ----
 * orc_elem_step: one record applied to a register copy of an element (the
 * semantics of apply_elem above): new state, returned bits, Ok flag.
 * orc_check_linearizable: for every element of one slice, is there a serial order
 * of that element's records (idx[k] == element) that reproduces each record's
 * returned value (rets, element-sized; NULL = not checked) and Ok flag (oks, NULL =
 * not checked) and ends at final_slice[element]? vals: n values, or one (v_len == 1).
 * Records with idx >= slice_len are ignored. Returns 0 = linearisable, 1 = not (the
 * element in *bad_elem), 2 = undecided within max_nodes branch steps, < 0 = error. */
int orc_elem_step(uint32_t kind, uint32_t dtype, uint32_t op, uint64_t state_bits, uint64_t val_bits,
                  const void* cmp, const void* eps, uint64_t* new_bits, uint64_t* ret_bits, uint8_t* ok);
int orc_check_linearizable(uint32_t kind, uint32_t dtype, uint32_t op, const void* cmp, const void* eps,
                           const void* init_slice, const void* final_slice, uint64_t slice_len,
                           const uint64_t* idx, uint64_t n, const void* vals, uint64_t v_len,
                           const void* rets, const uint8_t* oks, uint64_t max_nodes,
                           uint64_t* bad_elem);

/* result reorder: ArrayFetchBatchOpHandle (operations/handle.rs:315-317) */
void orc_scatter_results(const void* res_in, const uint64_t* res_pos, uint64_t n,
                         uint32_t elem_bytes, void* res_out);

#ifdef __cplusplus
}
#endif
#endif
