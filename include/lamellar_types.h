/*
 * lamellar_types.h — plain-C vocabulary shared by the MI355X batched element-op
 * library (liblamellar_gpu_ops.so) and its CPU oracle (oracle/).
 *
 * Every enum below restates a type of pnnl/lamellar-runtime's LamellarArray
 * batched element-op path; the numeric values are the reference's declaration
 * order so a Rust `as u32` cast of the reference enum is the C value.
 *
 * No HIP, torch or C++ types appear here: Rust (bindgen / hand-written
 * `extern "C"`), ctypes and the C oracle all include this file unchanged.
 */
#ifndef LAMELLAR_TYPES_H
#define LAMELLAR_TYPES_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes. The reference panics in these situations; the C ABI returns
 * a code instead (SURVEY.md §8(b) "Errors").
 *   LMR_E_OOB       global index >= array len   (src/array/unsafe/operations.rs:523-526, 716-719)
 *   LMR_E_DIVZERO   integer div/rem by zero     (Rust panics in release too)
 *   LMR_E_OVERFLOW  integer MIN / -1, MIN % -1  (Rust panics in release too)
 *   LMR_E_UNSUPPORTED op not generated for (kind, T)  (impl/src/array_ops.rs:648,758,807 `unreachable!`)
 */
typedef enum {
    LMR_OK = 0,
    LMR_E_INVALID = 1,
    LMR_E_OOB = 2,
    LMR_E_DIVZERO = 3,
    LMR_E_OVERFLOW = 4,
    LMR_E_UNSUPPORTED = 5,
    LMR_E_HIP = 6,
    LMR_E_WORKSPACE = 7,
    LMR_E_LENGTH = 8
} lmr_status_t;

/* Device error word bits (OR-ed by kernels; read back with lmr_ctx_error). */
#define LMR_ERRBIT_OOB         0x1u
#define LMR_ERRBIT_DIVZERO     0x2u
#define LMR_ERRBIT_OVERFLOW    0x4u
#define LMR_ERRBIT_UNSUPPORTED 0x8u
#define LMR_ERRBIT_TRANSPORT   0x10u   /* a peer-transport wait timed out (a PE never arrived) */

/* Element types with a device path. usize/isize are 64-bit on every target the
 * reference supports, so they map to U64/I64. u128/i128/bool are out of scope
 * (no 128-bit device atomics; SURVEY.md §8(a')). */
typedef enum {
    LMR_U8 = 0, LMR_U16 = 1, LMR_U32 = 2, LMR_U64 = 3,
    LMR_I8 = 4, LMR_I16 = 5, LMR_I32 = 6, LMR_I64 = 7,
    LMR_F32 = 8, LMR_F64 = 9,
    LMR_NUM_DTYPES = 10
} lmr_dtype_t;

/* ArrayOpCmd<T> in declaration order — src/array/operations.rs:86-114. */
typedef enum {
    LMR_OP_ADD = 0, LMR_OP_FETCH_ADD = 1,
    LMR_OP_SUB = 2, LMR_OP_FETCH_SUB = 3,
    LMR_OP_MUL = 4, LMR_OP_FETCH_MUL = 5,
    LMR_OP_DIV = 6, LMR_OP_FETCH_DIV = 7,
    LMR_OP_REM = 8, LMR_OP_FETCH_REM = 9,
    LMR_OP_AND = 10, LMR_OP_FETCH_AND = 11,
    LMR_OP_OR = 12, LMR_OP_FETCH_OR = 13,
    LMR_OP_XOR = 14, LMR_OP_FETCH_XOR = 15,
    LMR_OP_STORE = 16, LMR_OP_LOAD = 17,
    LMR_OP_SWAP = 18, LMR_OP_PUT = 19, LMR_OP_GET = 20,
    LMR_OP_COMPARE_EXCHANGE = 21, LMR_OP_COMPARE_EXCHANGE_EPS = 22,
    LMR_OP_SHL = 23, LMR_OP_FETCH_SHL = 24,
    LMR_OP_SHR = 25, LMR_OP_FETCH_SHR = 26,
    LMR_NUM_OPS = 27
} lmr_opcmd_t;

/* BatchReturnType — src/array/unsafe/operations.rs:850-854. */
typedef enum {
    LMR_RET_NONE = 0,    /* ArrayBatchOpHandle           */
    LMR_RET_VALS = 1,    /* ArrayFetchBatchOpHandle<T>   -> Vec<T>          */
    LMR_RET_RESULT = 2   /* ArrayResultBatchOpHandle<T>  -> Vec<Result<T,T>> */
} lmr_ret_kind_t;

/* Distribution — src/array.rs:247-252. */
typedef enum { LMR_DIST_BLOCK = 0, LMR_DIST_CYCLIC = 1 } lmr_distribution_t;

/* Built-in array reductions (impl/src/array_reduce.rs:283-319: "sum", "prod",
 * "max", "min"; src/array/unsafe.rs:1414-1557). */
typedef enum { LMR_REDUCE_SUM = 0, LMR_REDUCE_PROD = 1, LMR_REDUCE_MAX = 2, LMR_REDUCE_MIN = 3 } lmr_reduce_op_t;

/* Array kinds that carry the op path (src/array/atomic.rs:28-41, 524-533;
 * impl/src/array_ops.rs:546-572). On the device every kind applies each record
 * atomically per element; the kind only changes the CompareExchangeEps return
 * value (NativeAtomic returns Ok(new) on an exact match,
 * impl/src/array_ops.rs:391-395) and which ops exist (ReadOnly: load only). */
typedef enum {
    LMR_KIND_UNSAFE = 0,
    LMR_KIND_NATIVE_ATOMIC = 1,   /* AtomicArray<u8..u64,i8..i64> */
    LMR_KIND_GENERIC_ATOMIC = 2,  /* AtomicArray<f32,f64>          */
    LMR_KIND_LOCAL_LOCK = 3,
    LMR_KIND_GLOBAL_LOCK = 4,
    LMR_KIND_READ_ONLY = 5
} lmr_array_kind_t;

/* Index width of packed records — IndexSize, src/array/unsafe/operations.rs:47-86.
 * The value is the byte width (1, 2, 4, 8); U64 and Usize are both 8. */

/* Layout of a (sub)array — the fields of UnsafeArrayInner that index math
 * reads (src/array/unsafe.rs:107-116). `sub` = 1 for a sub_array view. */
typedef struct {
    uint32_t distribution;         /* lmr_distribution_t */
    uint32_t num_pes;
    uint32_t my_pe;
    uint32_t sub;
    uint64_t orig_elem_per_pe;
    uint64_t orig_remaining_elems;
    uint64_t offset;               /* relative to size of T */
    uint64_t size;                 /* relative to size of T */
} lmr_layout_t;

#ifdef __cplusplus
}
#endif
#endif /* LAMELLAR_TYPES_H */
