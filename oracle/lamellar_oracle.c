/*
 * lamellar_oracle.c — CPU ORACLE FOR TESTS ONLY (see lamellar_oracle.h).
 *
 * Plain-C restatement of pnnl/lamellar-runtime's batched element-op path.
 * Integer arithmetic wraps (release profile, Cargo.toml:83-87 has no
 * overflow-checks); division/remainder by zero and MIN/-1 are reported as
 * status codes where Rust panics; float `%` is fmod (Rust `%` on f32/f64).
 */
#include "lamellar_oracle.h"
#include <math.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* layout: src/array/unsafe.rs                                         */
/* ------------------------------------------------------------------ */

/* UnsafeArray::async_new (unsafe.rs:178-274): full_array_size = max(len, num_pes),
 * elem_per_pe = full / npes, remaining = full % npes; when len < npes the array
 * is returned as sub_array(0..len). */
int orc_layout_new(lmr_layout_t* L, uint64_t array_size, uint32_t num_pes,
                   uint32_t my_pe, uint32_t distribution) {
    if (!L || num_pes == 0 || my_pe >= num_pes || distribution > 1) return LMR_E_INVALID;
    uint64_t full = array_size > num_pes ? array_size : num_pes;
    memset(L, 0, sizeof(*L));
    L->distribution = distribution;
    L->num_pes = num_pes;
    L->my_pe = my_pe;
    L->orig_elem_per_pe = full / num_pes;
    L->orig_remaining_elems = full % num_pes;
    L->offset = 0;
    L->size = full;
    L->sub = 0;
    if (full != array_size) {
        lmr_layout_t tmp = *L;
        return orc_layout_sub(&tmp, 0, array_size, L);
    }
    return LMR_OK;
}

/* sub_array (unsafe.rs:1259-1290): offset += start; size = end - start; sub = true */
int orc_layout_sub(const lmr_layout_t* p, uint64_t start, uint64_t end, lmr_layout_t* out) {
    if (!p || !out || end > p->size || start > end) return LMR_E_INVALID;
    lmr_layout_t L = *p;
    L.offset += start;
    L.size = end - start;
    L.sub = 1;
    *out = L;
    return LMR_OK;
}

/* full_pe_and_offset_for_global_index (unsafe.rs:1610-1647) */
int orc_full_pe_and_offset(const lmr_layout_t* L, uint64_t index, uint64_t* pe, uint64_t* off) {
    if (!(L->size > index)) return 0;
    uint64_t g = index;
    if (L->distribution == LMR_DIST_BLOCK) {
        uint64_t rem_index = L->orig_remaining_elems * (L->orig_elem_per_pe + 1);
        if (g < rem_index) {
            uint64_t p = g / (L->orig_elem_per_pe + 1);
            *pe = p;
            *off = g - p * (L->orig_elem_per_pe + 1);
        } else {
            uint64_t t = g - rem_index;
            uint64_t tp = t / L->orig_elem_per_pe;
            *pe = L->orig_remaining_elems + tp;
            *off = t - tp * L->orig_elem_per_pe;
        }
    } else {
        *pe = g % L->num_pes;
        *off = g / L->num_pes;
    }
    return 1;
}

/* pe_for_dist_index (unsafe.rs:1651-1673) */
int orc_pe_for_dist_index(const lmr_layout_t* L, uint64_t index, uint64_t* pe) {
    if (!(L->size > index)) return 0;
    uint64_t g = index + L->offset;
    if (L->distribution == LMR_DIST_BLOCK) {
        uint64_t rem_index = L->orig_remaining_elems * (L->orig_elem_per_pe + 1);
        if (g < rem_index) *pe = g / (L->orig_elem_per_pe + 1);
        else *pe = L->orig_remaining_elems + (g - rem_index) / L->orig_elem_per_pe;
    } else {
        *pe = g % L->num_pes;
    }
    return 1;
}

/* pe_full_offset_for_dist_index (unsafe.rs:1677-1705) */
int orc_pe_full_offset_for_dist_index(const lmr_layout_t* L, uint64_t pe, uint64_t index,
                                      uint64_t* off) {
    uint64_t g = L->offset + index;
    if (L->distribution == LMR_DIST_BLOCK) {
        uint64_t rem_index = L->orig_remaining_elems * (L->orig_elem_per_pe + 1);
        if (g < rem_index) {
            *off = g - pe * (L->orig_elem_per_pe + 1);
        } else {
            uint64_t t = g - rem_index;
            uint64_t tp = t / L->orig_elem_per_pe;
            *off = t - tp * L->orig_elem_per_pe;
        }
        return 1;
    }
    if (g % L->num_pes == pe) { *off = index / L->num_pes; return 1; }
    return 0;
}

/* pe_sub_offset_for_dist_index (unsafe.rs:1708-1736) */
int orc_pe_sub_offset_for_dist_index(const lmr_layout_t* L, uint64_t pe, uint64_t index,
                                     uint64_t* off) {
    uint64_t start_pe;
    if (!orc_pe_for_dist_index(L, 0, &start_pe)) return 0;
    if (L->distribution == LMR_DIST_BLOCK) {
        if (start_pe == pe) {
            if (index < L->size) { *off = index; return 1; }
            return 0;
        }
        return orc_pe_full_offset_for_dist_index(L, pe, index, off);
    }
    if ((index + L->offset) % L->num_pes == pe) { *off = index / L->num_pes; return 1; }
    return 0;
}

/* UnsafeArray::pe_and_offset_for_global_index (unsafe.rs:1207-1223) */
int orc_pe_and_offset(const lmr_layout_t* L, uint64_t index, uint64_t* pe, uint64_t* off) {
    if (L->sub) {
        if (!orc_pe_for_dist_index(L, index, pe)) return 0;
        return orc_pe_sub_offset_for_dist_index(L, *pe, index, off);
    }
    return orc_full_pe_and_offset(L, index, pe, off);
}

/* global_start_index_for_pe (unsafe.rs:1878-1886) */
uint64_t orc_global_start_index_for_pe(const lmr_layout_t* L, uint64_t pe) {
    if (L->distribution == LMR_DIST_BLOCK) {
        uint64_t gs = L->orig_elem_per_pe * pe;
        return gs + (pe < L->orig_remaining_elems ? pe : L->orig_remaining_elems);
    }
    return pe;
}

/* start_index_for_pe (unsafe.rs:1889-1941) */
int orc_start_index_for_pe(const lmr_layout_t* L, uint64_t pe, uint64_t* out) {
    if (L->distribution == LMR_DIST_BLOCK) {
        uint64_t gs = orc_global_start_index_for_pe(L, pe);
        if (gs >= L->offset) {
            uint64_t start = gs - L->offset;
            if (start < L->size) { *out = start; return 1; }
            return 0;
        }
        uint64_t ge = gs + L->orig_elem_per_pe;
        if (pe < L->orig_remaining_elems) ge += 1;
        if (L->offset < ge) { *out = 0; return 1; }
        return 0;
    }
    uint64_t start_pe;
    if (orc_pe_for_dist_index(L, 0, &start_pe)) {
        uint64_t tl = L->size < L->num_pes ? L->size : L->num_pes;
        for (uint64_t i = 0; i < tl; i++)
            if ((i + start_pe) % L->num_pes == pe) { *out = i; return 1; }
    }
    return 0;
}

/* num_elems_pe (unsafe.rs:1966-2016) */
uint64_t orc_num_elems_pe(const lmr_layout_t* L, uint64_t pe) {
    if (L->distribution == LMR_DIST_BLOCK) {
        uint64_t si, ei;
        if (!orc_start_index_for_pe(L, pe, &si)) return 0;
        if (!orc_start_index_for_pe(L, pe + 1, &ei)) ei = L->size;
        return ei - si;
    }
    uint64_t start_pe, end_pe;
    if (!orc_pe_for_dist_index(L, 0, &start_pe)) return 0;
    if (!orc_pe_for_dist_index(L, L->size - 1, &end_pe)) return 0; /* reference panics */
    uint64_t n = L->size / L->num_pes;
    if (L->size % L->num_pes != 0) {
        if (start_pe <= end_pe) {
            if (pe >= start_pe && pe <= end_pe) n += 1;
        } else {
            if (pe >= start_pe || pe <= end_pe) n += 1;
        }
    }
    return n;
}

/* local_as_mut_slice start offset within PE `pe`'s full shard (unsafe.rs:2023-2066) */
uint64_t orc_local_slice_start(const lmr_layout_t* L, uint64_t pe) {
    if (L->distribution == LMR_DIST_BLOCK) {
        uint64_t start_pe;
        if (!orc_pe_for_dist_index(L, 0, &start_pe)) return 0;
        if (pe == start_pe) return L->offset - orc_global_start_index_for_pe(L, pe);
        return 0;
    }
    uint64_t g = L->offset;
    return g / L->num_pes + ((pe >= g % L->num_pes) ? 0 : 1);
}

/* IndexSize::from(max local len) with LAMELLAR_ARRAY_INDEX_SIZE=dynamic
 * (unsafe/operations.rs:56-75; max over PEs :300-304). */
uint32_t orc_index_size(const lmr_layout_t* L) {
    uint64_t m = 0;
    for (uint64_t p = 0; p < L->num_pes; p++) {
        uint64_t n = orc_num_elems_pe(L, p);
        if (n > m) m = n;
    }
    if (m <= 0xFFull) return 1;
    if (m <= 0xFFFFull) return 2;
    if (m <= 0xFFFFFFFFull) return 4;
    return 8;
}

uint32_t orc_dtype_bytes(uint32_t dtype) {
    switch (dtype) {
    case LMR_U8: case LMR_I8: return 1;
    case LMR_U16: case LMR_I16: return 2;
    case LMR_U32: case LMR_I32: case LMR_F32: return 4;
    case LMR_U64: case LMR_I64: case LMR_F64: return 8;
    default: return 0;
    }
}

static uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

/* #[repr(C)] struct IdxVal<I,T>{index: I, val: T} (operations.rs:213-219):
 * val at round_up(sizeof I, align T), size rounded to max(align I, align T). */
uint32_t orc_record_val_offset(uint32_t index_size, uint32_t dtype) {
    return (uint32_t)round_up(index_size, orc_dtype_bytes(dtype));
}
uint32_t orc_record_bytes(uint32_t index_size, uint32_t dtype) {
    uint32_t tb = orc_dtype_bytes(dtype);
    uint32_t a = index_size > tb ? index_size : tb;
    return (uint32_t)round_up(orc_record_val_offset(index_size, dtype) + tb, a);
}

/* Which handle each op builder returns (operations/{arithmetic,bitwise,access,
 * compare_exchange,read_only,shift}.rs): fetch_*, load, get, swap -> Vals;
 * compare_exchange(_epsilon) -> Result; the rest -> None. */
uint32_t orc_op_ret_kind(uint32_t op) {
    switch (op) {
    case LMR_OP_FETCH_ADD: case LMR_OP_FETCH_SUB: case LMR_OP_FETCH_MUL:
    case LMR_OP_FETCH_DIV: case LMR_OP_FETCH_REM: case LMR_OP_FETCH_AND:
    case LMR_OP_FETCH_OR: case LMR_OP_FETCH_XOR: case LMR_OP_LOAD:
    case LMR_OP_SWAP: case LMR_OP_GET: case LMR_OP_FETCH_SHL: case LMR_OP_FETCH_SHR:
        return LMR_RET_VALS;
    case LMR_OP_COMPARE_EXCHANGE: case LMR_OP_COMPARE_EXCHANGE_EPS:
        return LMR_RET_RESULT;
    default:
        return LMR_RET_NONE;
    }
}

/* Op availability per (kind, T): src/array.rs:207-220 with the OpType lists of
 * impl/src/array_ops.rs:1503-1533. Integers: ReadOnly, Access, Arithmetic,
 * CompExEps, Bitwise, Shift, CompEx. Floats: ReadOnly, Access, Arithmetic,
 * CompExEps. ReadOnlyArray: ReadOnly only. */
int orc_op_supported(uint32_t kind, uint32_t dtype, uint32_t op) {
    if (dtype >= LMR_NUM_DTYPES || op >= LMR_NUM_OPS) return 0;
    if (kind == LMR_KIND_READ_ONLY) return op == LMR_OP_LOAD;
    int is_float = (dtype == LMR_F32 || dtype == LMR_F64);
    if (!is_float) return 1;
    switch (op) {
    case LMR_OP_AND: case LMR_OP_FETCH_AND: case LMR_OP_OR: case LMR_OP_FETCH_OR:
    case LMR_OP_XOR: case LMR_OP_FETCH_XOR: case LMR_OP_COMPARE_EXCHANGE:
    case LMR_OP_SHL: case LMR_OP_FETCH_SHL: case LMR_OP_SHR: case LMR_OP_FETCH_SHR:
        return 0;
    default:
        return 1;
    }
}

/* ------------------------------------------------------------------ */
/* element apply: impl/src/array_ops.rs:327-545                         */
/* ------------------------------------------------------------------ */
/* One record applied to one element, sequentially. NativeAtomic semantics
 * (array_ops.rs:327-458, native_atomic.rs:29-113) and the generic/lock/unsafe
 * semantics (:480-545) coincide when applied one at a time except for
 * CompareExchangeEps (:391-419 vs :521-535), which is the only place `kind`
 * matters. */

#define INT_APPLY(NAME, T, UT, WT, IS_SIGNED, BITS, MINV)                                  \
static int apply_##NAME(T* a, T v, uint32_t op, uint32_t kind, T cmp, T eps,              \
                        T* res, uint8_t* ok) {                                             \
    T old = *a;                                                                            \
    *res = old;                                                                            \
    switch (op) {                                                                          \
    case LMR_OP_ADD: case LMR_OP_FETCH_ADD: *a = (T)(UT)((UT)old + (UT)v); break;          \
    case LMR_OP_SUB: case LMR_OP_FETCH_SUB: *a = (T)(UT)((UT)old - (UT)v); break;          \
    case LMR_OP_MUL: case LMR_OP_FETCH_MUL:                                                \
        *a = (T)(UT)((WT)(UT)old * (WT)(UT)v); break;                                      \
    case LMR_OP_DIV: case LMR_OP_FETCH_DIV:                                                \
        if (v == 0) return LMR_E_DIVZERO;                                                  \
        if (IS_SIGNED && old == (T)(MINV) && v == (T)-1) return LMR_E_OVERFLOW;            \
        *a = (T)(old / v); break;                                                          \
    case LMR_OP_REM: case LMR_OP_FETCH_REM:                                                \
        if (v == 0) return LMR_E_DIVZERO;                                                  \
        if (IS_SIGNED && old == (T)(MINV) && v == (T)-1) return LMR_E_OVERFLOW;            \
        *a = (T)(old % v); break;                                                          \
    case LMR_OP_AND: case LMR_OP_FETCH_AND: *a = (T)(old & v); break;                      \
    case LMR_OP_OR: case LMR_OP_FETCH_OR: *a = (T)(old | v); break;                        \
    case LMR_OP_XOR: case LMR_OP_FETCH_XOR: *a = (T)(old ^ v); break;                      \
    case LMR_OP_STORE: case LMR_OP_PUT: *a = v; break;                                     \
    case LMR_OP_LOAD: case LMR_OP_GET: break;                                              \
    case LMR_OP_SWAP: *a = v; break;                                                       \
    case LMR_OP_COMPARE_EXCHANGE:                                                          \
        if (old == cmp) { *a = v; *ok = 1; *res = cmp; } else { *ok = 0; }                 \
        break;                                                                             \
    case LMR_OP_COMPARE_EXCHANGE_EPS:                                                      \
        if (kind == LMR_KIND_NATIVE_ATOMIC) {                                              \
            /* array_ops.rs:391-419: exact match returns Ok(val); otherwise CAS while  \
               (orig.abs_diff(old) as T) < eps and return Ok(orig) */                   \
            if (old == cmp) { *a = v; *ok = 1; *res = v; }                                 \
            else {                                                                         \
                UT d = (old > cmp) ? (UT)((UT)old - (UT)cmp) : (UT)((UT)cmp - (UT)old);    \
                if ((T)d < eps) { *a = v; *ok = 1; *res = old; } else { *ok = 0; }         \
            }                                                                              \
        } else {                                                                           \
            /* array_ops.rs:521-535 */                                                     \
            int same = (cmp > old) ? ((T)(UT)((UT)cmp - (UT)old) < eps)                    \
                                   : ((T)(UT)((UT)old - (UT)cmp) < eps);                   \
            if (same) { *a = v; *ok = 1; *res = cmp; } else { *ok = 0; }                   \
        }                                                                                  \
        break;                                                                             \
    case LMR_OP_SHL: case LMR_OP_FETCH_SHL:                                                \
        *a = (T)(UT)((WT)(UT)old << ((unsigned)(UT)v & (BITS - 1))); break;                \
    case LMR_OP_SHR: case LMR_OP_FETCH_SHR:                                                \
        *a = (T)(old >> ((unsigned)(UT)v & (BITS - 1))); break;                            \
    default: return LMR_E_UNSUPPORTED;                                                     \
    }                                                                                      \
    return LMR_OK;                                                                         \
}

INT_APPLY(u8, uint8_t, uint8_t, uint32_t, 0, 8, 0)
INT_APPLY(u16, uint16_t, uint16_t, uint32_t, 0, 16, 0)
INT_APPLY(u32, uint32_t, uint32_t, uint64_t, 0, 32, 0)
INT_APPLY(u64, uint64_t, uint64_t, uint64_t, 0, 64, 0)
INT_APPLY(i8, int8_t, uint8_t, uint32_t, 1, 8, INT8_MIN)
INT_APPLY(i16, int16_t, uint16_t, uint32_t, 1, 16, INT16_MIN)
INT_APPLY(i32, int32_t, uint32_t, uint64_t, 1, 32, INT32_MIN)
INT_APPLY(i64, int64_t, uint64_t, uint64_t, 1, 64, INT64_MIN)

#define FLT_APPLY(NAME, T, FMOD)                                                           \
static int apply_##NAME(T* a, T v, uint32_t op, uint32_t kind, T cmp, T eps,              \
                        T* res, uint8_t* ok) {                                             \
    (void)kind;                                                                            \
    T old = *a;                                                                            \
    *res = old;                                                                            \
    switch (op) {                                                                          \
    case LMR_OP_ADD: case LMR_OP_FETCH_ADD: *a = old + v; break;                           \
    case LMR_OP_SUB: case LMR_OP_FETCH_SUB: *a = old - v; break;                           \
    case LMR_OP_MUL: case LMR_OP_FETCH_MUL: *a = old * v; break;                           \
    case LMR_OP_DIV: case LMR_OP_FETCH_DIV: *a = old / v; break;                           \
    case LMR_OP_REM: case LMR_OP_FETCH_REM: *a = FMOD(old, v); break;                      \
    case LMR_OP_STORE: case LMR_OP_PUT: *a = v; break;                                     \
    case LMR_OP_LOAD: case LMR_OP_GET: break;                                              \
    case LMR_OP_SWAP: *a = v; break;                                                       \
    case LMR_OP_COMPARE_EXCHANGE_EPS: {                                                    \
        /* generic kinds only (f32/f64 are GenericAtomic): array_ops.rs:521-535 */        \
        int same = (cmp > old) ? ((cmp - old) < eps) : ((old - cmp) < eps);                \
        if (same) { *a = v; *ok = 1; *res = cmp; } else { *ok = 0; }                       \
        break; }                                                                           \
    default: return LMR_E_UNSUPPORTED;                                                     \
    }                                                                                      \
    return LMR_OK;                                                                         \
}

FLT_APPLY(f32, float, fmodf)
FLT_APPLY(f64, double, fmod)

/* Apply one record to slice[index]; `val`, `cmp`, `eps` and `res` point at
 * element-sized storage of `dtype`. */
static int apply_elem(void* slice, uint64_t index, uint32_t kind, uint32_t dtype, uint32_t op,
                      const void* val, const void* cmp, const void* eps, void* res, uint8_t* ok) {
#define CASE(D, NAME, T)                                                                   \
    case D: {                                                                              \
        T v, c = 0, e = 0, r;                                                              \
        memcpy(&v, val, sizeof(T));                                                        \
        if (cmp) memcpy(&c, cmp, sizeof(T));                                               \
        if (eps) memcpy(&e, eps, sizeof(T));                                               \
        int st = apply_##NAME(((T*)slice) + index, v, op, kind, c, e, &r, ok);             \
        if (res) memcpy(res, &r, sizeof(T));                                               \
        return st;                                                                         \
    }
    switch (dtype) {
    CASE(LMR_U8, u8, uint8_t) CASE(LMR_U16, u16, uint16_t)
    CASE(LMR_U32, u32, uint32_t) CASE(LMR_U64, u64, uint64_t)
    CASE(LMR_I8, i8, int8_t) CASE(LMR_I16, i16, int16_t)
    CASE(LMR_I32, i32, int32_t) CASE(LMR_I64, i64, int64_t)
    CASE(LMR_F32, f32, float) CASE(LMR_F64, f64, double)
    default: return LMR_E_UNSUPPORTED;
    }
#undef CASE
}

int orc_elem_step(uint32_t kind, uint32_t dtype, uint32_t op, uint64_t state_bits, uint64_t val_bits,
                  const void* cmp, const void* eps, uint64_t* new_bits, uint64_t* ret_bits, uint8_t* ok) {
    const uint32_t eb = orc_dtype_bytes(dtype);
    uint8_t elem[8] = {0}, val[8] = {0}, res[8] = {0};
    memcpy(elem, &state_bits, eb);          /* little endian: the low eb bytes */
    memcpy(val, &val_bits, eb);
    *ok = 0;
    const int st = apply_elem(elem, 0, kind, dtype, op, val, cmp, eps, res, ok);
    *new_bits = 0;
    *ret_bits = 0;
    memcpy(new_bits, elem, eb);
    memcpy(ret_bits, res, eb);
    return st;
}

static uint64_t read_index(const uint8_t* p, uint32_t index_size) {
    switch (index_size) {
    case 1: return p[0];
    case 2: { uint16_t x; memcpy(&x, p, 2); return x; }
    case 4: { uint32_t x; memcpy(&x, p, 4); return x; }
    default: { uint64_t x; memcpy(&x, p, 8); return x; }
    }
}

static void write_index(uint8_t* p, uint32_t index_size, uint64_t v) {
    switch (index_size) {
    case 1: p[0] = (uint8_t)v; break;
    case 2: { uint16_t x = (uint16_t)v; memcpy(p, &x, 2); break; }
    case 4: { uint32_t x = (uint32_t)v; memcpy(p, &x, 4); break; }
    default: memcpy(p, &v, 8); break;
    }
}

static int keep_first(int st, int s2) { return st != LMR_OK ? st : s2; }

/* The `_` arm of every generated match is `unreachable!` (array_ops.rs:648,758,807):
 * an op outside the (kind, T) table is reported before touching the slice. */
static int check_op(uint32_t kind, uint32_t dtype, uint32_t op) {
    return orc_op_supported(kind, dtype, op) ? LMR_OK : LMR_E_UNSUPPORTED;
}

/* multi_val_multi_idx exec bodies (array_ops.rs:863-899 none, 1041-1079 result,
 * 1226-1264 fetch): reinterpret the bytes as &[IdxVal<I,T>] by index_size and loop. */
int orc_apply_mvmi(void* slice, uint64_t slice_len, uint32_t kind, uint32_t dtype,
                   uint32_t op, const void* cmp, const void* eps,
                   const void* idx_vals, uint64_t nbytes, uint32_t index_size,
                   void* results, uint8_t* ok) {
    int st = check_op(kind, dtype, op);
    if (st) return st;
    uint32_t rb = orc_record_bytes(index_size, dtype), vo = orc_record_val_offset(index_size, dtype);
    uint32_t tb = orc_dtype_bytes(dtype);
    uint64_t n = nbytes / rb;
    const uint8_t* p = (const uint8_t*)idx_vals;
    for (uint64_t k = 0; k < n; k++) {
        uint64_t idx = read_index(p + k * rb, index_size);
        if (idx >= slice_len) { st = keep_first(st, LMR_E_OOB); continue; }
        uint8_t o = 0;
        int s2 = apply_elem(slice, idx, kind, dtype, op, p + k * rb + vo, cmp, eps,
                            results ? (uint8_t*)results + k * tb : NULL, &o);
        if (ok) ok[k] = o;
        st = keep_first(st, s2);
    }
    return st;
}

/* single_val_multi_idx exec bodies (array_ops.rs:929-967, 1109-1149, 1297-1343) */
int orc_apply_svmi(void* slice, uint64_t slice_len, uint32_t kind, uint32_t dtype,
                   uint32_t op, const void* cmp, const void* eps, const void* val,
                   const void* indices, uint64_t nbytes, uint32_t index_size,
                   void* results, uint8_t* ok) {
    int st = check_op(kind, dtype, op);
    if (st) return st;
    uint32_t tb = orc_dtype_bytes(dtype);
    uint64_t n = nbytes / index_size;
    const uint8_t* p = (const uint8_t*)indices;
    for (uint64_t k = 0; k < n; k++) {
        uint64_t idx = read_index(p + k * index_size, index_size);
        if (idx >= slice_len) { st = keep_first(st, LMR_E_OOB); continue; }
        uint8_t o = 0;
        int s2 = apply_elem(slice, idx, kind, dtype, op, val, cmp, eps,
                            results ? (uint8_t*)results + k * tb : NULL, &o);
        if (ok) ok[k] = o;
        st = keep_first(st, s2);
    }
    return st;
}

/* multi_val_single_idx exec bodies (array_ops.rs:999-1008, 1178-1190, 1378-1390):
 * the lock is taken once and the values are applied in order. */
int orc_apply_mvsi(void* slice, uint64_t slice_len, uint32_t kind, uint32_t dtype,
                   uint32_t op, const void* cmp, const void* eps,
                   const void* vals, uint64_t nbytes, uint64_t index,
                   void* results, uint8_t* ok) {
    int st = check_op(kind, dtype, op);
    if (st) return st;
    uint32_t tb = orc_dtype_bytes(dtype);
    uint64_t n = nbytes / tb;
    if (n && index >= slice_len) return LMR_E_OOB;
    const uint8_t* p = (const uint8_t*)vals;
    for (uint64_t k = 0; k < n; k++) {
        uint8_t o = 0;
        int s2 = apply_elem(slice, index, kind, dtype, op, p + k * tb, cmp, eps,
                            results ? (uint8_t*)results + k * tb : NULL, &o);
        if (ok) ok[k] = o;
        st = keep_first(st, s2);
    }
    return st;
}

/* ------------------------------------------------------------------ */
/* pack: src/array/unsafe/operations.rs                                 */
/* ------------------------------------------------------------------ */

/* OpInput::as_op_input chunk count (operations.rs:455-480): len < 1000 -> 1,
 * else batch_op_threads chunks of len/num plus a remainder chunk of len % (len/num). */
uint64_t orc_num_chunks(uint64_t len, uint64_t batch_op_threads) {
    if (len == 0) return 0;
    uint64_t num = len < 1000 ? 1 : (batch_op_threads ? batch_op_threads : 1);
    uint64_t per = len / num;
    return num + ((len % per) > 0 ? 1 : 0);
}

static void chunk_bounds(uint64_t len, uint64_t threads, uint64_t c, uint64_t* s, uint64_t* e) {
    uint64_t num = len < 1000 ? 1 : (threads ? threads : 1);
    uint64_t per = len / num;
    if (c < num) { *s = c * per; *e = (c + 1) * per; }
    else { *s = num * per; *e = len; }
}

typedef struct {
    orc_am_t* ams; uint64_t max_ams; int64_t n_ams;
    uint8_t* bytes; uint64_t cap; uint64_t used;
    uint64_t* res_pos; uint64_t res_used;
} pack_out_t;

/* Flush one per-PE buffer as an op buffer (an AM in the reference). */
static int emit_am(pack_out_t* o, uint32_t pe, const uint8_t* buf, uint64_t nbytes,
                   const uint64_t* pos, uint64_t nrec) {
    if ((uint64_t)o->n_ams >= o->max_ams || o->used + nbytes > o->cap) return LMR_E_WORKSPACE;
    orc_am_t* a = &o->ams[o->n_ams++];
    a->pe = pe; a->_pad = 0; a->byte_off = o->used; a->nbytes = nbytes; a->nrec = nrec;
    a->res_off = o->res_used;
    memcpy(o->bytes + o->used, buf, nbytes);
    memcpy(o->res_pos + o->res_used, pos, nrec * sizeof(uint64_t));
    o->used += nbytes; o->res_used += nrec;
    return LMR_OK;
}

#include <stdlib.h>

/* multi_val_multi_index (unsafe/operations.rs:663-811) and
 * one_val_multi_indices (:479-587): rec_bytes = sizeof(IdxVal<I,T>) (MVMI) or
 * index_size (SVMI); num_per_batch = ceil(threshold / rec_bytes) (:488-489, 679-681). */
static int64_t pack_common(const lmr_layout_t* L, uint32_t dtype, const uint64_t* gidx,
                           const void* vals, uint64_t n, uint32_t index_size,
                           uint64_t thr, uint64_t threads, int svmi, orc_am_t* ams,
                           uint64_t max_ams, uint8_t* bytes, uint64_t cap,
                           uint64_t* res_pos, int* status) {
    uint32_t tb = svmi ? 0 : orc_dtype_bytes(dtype);
    uint32_t rb = svmi ? index_size : orc_record_bytes(index_size, dtype);
    uint32_t vo = svmi ? 0 : orc_record_val_offset(index_size, dtype);
    uint64_t num_per_batch = (uint64_t)ceilf((float)thr / (float)rb);
    if (num_per_batch == 0) num_per_batch = 1;
    uint64_t bytes_per_batch = num_per_batch * rb;
    uint32_t npes = L->num_pes;
    pack_out_t o = {ams, max_ams, 0, bytes, cap, 0, res_pos, 0};
    *status = LMR_OK;
    uint8_t* buf = (uint8_t*)malloc((size_t)npes * bytes_per_batch);
    uint64_t* pos = (uint64_t*)malloc((size_t)npes * num_per_batch * sizeof(uint64_t));
    uint64_t* fill = (uint64_t*)calloc(npes, sizeof(uint64_t));
    if (!buf || !pos || !fill) { free(buf); free(pos); free(fill); *status = LMR_E_WORKSPACE; return -1; }
    uint64_t nchunks = orc_num_chunks(n, threads);
    for (uint64_t c = 0; c < nchunks; c++) {
        uint64_t s, e;
        chunk_bounds(n, threads, c, &s, &e);
        memset(fill, 0, npes * sizeof(uint64_t));
        for (uint64_t j = s; j < e; j++) {
            uint64_t pe, off;
            if (!orc_pe_and_offset(L, gidx[j], &pe, &off)) {
                if (*status == LMR_OK) *status = LMR_E_OOB;   /* reference panics here */
                continue;
            }
            uint8_t* r = buf + pe * bytes_per_batch + fill[pe] * rb;
            memset(r, 0, rb);                 /* padding bytes: zero (reference leaves them as-is) */
            write_index(r, index_size, off);
            if (!svmi) memcpy(r + vo, (const uint8_t*)vals + j * tb, tb);
            pos[pe * num_per_batch + fill[pe]] = j;
            fill[pe]++;
            if (fill[pe] * rb >= bytes_per_batch) {
                int st = emit_am(&o, (uint32_t)pe, buf + pe * bytes_per_batch, fill[pe] * rb,
                                 pos + pe * num_per_batch, fill[pe]);
                if (st) { *status = st; goto done; }
                fill[pe] = 0;
            }
        }
        for (uint32_t pe = 0; pe < npes; pe++) {
            if (fill[pe] > 0) {
                int st = emit_am(&o, pe, buf + (uint64_t)pe * bytes_per_batch, fill[pe] * rb,
                                 pos + (uint64_t)pe * num_per_batch, fill[pe]);
                if (st) { *status = st; goto done; }
            }
        }
    }
done:
    free(buf); free(pos); free(fill);
    return o.n_ams;
}

int64_t orc_pack_mvmi(const lmr_layout_t* L, uint32_t dtype, const uint64_t* gidx,
                      const void* vals, uint64_t n, uint32_t index_size,
                      uint64_t am_size_threshold, uint64_t batch_op_threads,
                      orc_am_t* ams, uint64_t max_ams, uint8_t* bytes, uint64_t bytes_cap,
                      uint64_t* res_pos, int* status) {
    return pack_common(L, dtype, gidx, vals, n, index_size, am_size_threshold,
                       batch_op_threads, 0, ams, max_ams, bytes, bytes_cap, res_pos, status);
}

int64_t orc_pack_svmi(const lmr_layout_t* L, const uint64_t* gidx, uint64_t n,
                      uint32_t index_size, uint64_t am_size_threshold,
                      uint64_t batch_op_threads, orc_am_t* ams, uint64_t max_ams,
                      uint8_t* bytes, uint64_t bytes_cap, uint64_t* res_pos, int* status) {
    return pack_common(L, LMR_U8, gidx, NULL, n, index_size, am_size_threshold,
                       batch_op_threads, 1, ams, max_ams, bytes, bytes_cap, res_pos, status);
}

/* ------------------------------------------------------------------ */
/* whole batch                                                           */
/* ------------------------------------------------------------------ */

int orc_batch_op(const lmr_layout_t* L, void* const* pe_slices, uint32_t kind,
                 uint32_t dtype, uint32_t op, const void* cmp, const void* eps,
                 const uint64_t* gidx, uint64_t i_len, const void* vals, uint64_t v_len,
                 void* results, uint8_t* ok) {
    int st = check_op(kind, dtype, op);
    if (st) return st;
    if (i_len == 0 || v_len == 0) return LMR_OK;           /* "no vals no indices" :345-347 */
    if (i_len > 1 && v_len > 1 && i_len != v_len) return LMR_E_LENGTH;
    uint32_t tb = orc_dtype_bytes(dtype);
    uint64_t n = i_len > v_len ? i_len : v_len;
    const uint8_t* vp = (const uint8_t*)vals;
    for (uint64_t j = 0; j < n; j++) {
        uint64_t g = (i_len == 1) ? gidx[0] : gidx[j];
        const uint8_t* v = (v_len == 1) ? vp : vp + j * tb;
        uint64_t pe, off;
        if (!orc_pe_and_offset(L, g, &pe, &off)) { st = keep_first(st, LMR_E_OOB); continue; }
        uint8_t o = 0;
        int s2 = apply_elem(pe_slices[pe], off, kind, dtype, op, v, cmp, eps,
                            results ? (uint8_t*)results + j * tb : NULL, &o);
        if (ok) ok[j] = o;
        st = keep_first(st, s2);
    }
    return st;
}

/* ---- reductions: array_reduce.rs:82-88 (per-PE fold), :90-107 (cross-PE tree), :283-319 (ops) */
#define RED_STEP(T, UT, a, b, op)                                                        \
    ((op) == 0 ? (T)((UT)(a) + (UT)(b)) : (op) == 1 ? (T)((UT)(a) * (UT)(b))            \
     : (op) == 2 ? ((a) > (b) ? (a) : (b)) : ((a) < (b) ? (a) : (b)))
#define FRED_STEP(a, b, op)                                                              \
    ((op) == 0 ? (a) + (b) : (op) == 1 ? (a) * (b) : (op) == 2 ? ((a) > (b) ? (a) : (b)) \
     : ((a) < (b) ? (a) : (b)))

static void red_combine(uint32_t dtype, uint32_t op, void* acc, const void* v) {
    switch (dtype) {
#define RC(CODE, T, UT) case CODE: { T a, b; memcpy(&a, acc, sizeof a); memcpy(&b, v, sizeof b); \
        T r = RED_STEP(T, UT, a, b, op); memcpy(acc, &r, sizeof r); break; }
    RC(LMR_U8, uint8_t, uint8_t) RC(LMR_U16, uint16_t, uint16_t) RC(LMR_U32, uint32_t, uint32_t)
    RC(LMR_U64, uint64_t, uint64_t) RC(LMR_I8, int8_t, uint8_t) RC(LMR_I16, int16_t, uint16_t)
    RC(LMR_I32, int32_t, uint32_t) RC(LMR_I64, int64_t, uint64_t)
#undef RC
    case LMR_F32: { float a, b; memcpy(&a, acc, 4); memcpy(&b, v, 4); float r = FRED_STEP(a, b, op); memcpy(acc, &r, 4); break; }
    case LMR_F64: { double a, b; memcpy(&a, acc, 8); memcpy(&b, v, 8); double r = FRED_STEP(a, b, op); memcpy(acc, &r, 8); break; }
    default: break;
    }
}

void orc_reduce(uint32_t dtype, uint32_t op, const void* data, uint64_t n, void* out, uint8_t* has) {
    const size_t eb = orc_dtype_bytes(dtype);
    *has = n > 0;
    if (!n) return;
    memcpy(out, data, eb);
    for (uint64_t k = 1; k < n; k++) red_combine(dtype, op, out, (const uint8_t*)data + k * eb);
}

static int red_tree(uint32_t dtype, uint32_t op, const uint8_t* vals, const uint8_t* has, uint32_t lo,
                    uint32_t hi, uint8_t* out) {
    const size_t eb = orc_dtype_bytes(dtype);
    if (lo == hi) {
        if (has[lo]) memcpy(out, vals + lo * eb, eb);
        return has[lo] != 0;
    }
    const uint32_t mid = (lo + hi) / 2;
    uint8_t r[8];
    const int hl = red_tree(dtype, op, vals, has, lo, mid, out);
    const int hr = red_tree(dtype, op, vals, has, mid + 1, hi, r);
    if (!hl) { if (hr) memcpy(out, r, eb); return hr; }
    if (hr) red_combine(dtype, op, out, r);
    return 1;
}

void orc_reduce_tree(uint32_t dtype, uint32_t op, const void* vals, const uint8_t* has, uint32_t npes,
                     void* out, uint8_t* out_has) {
    *out_has = npes ? (uint8_t)red_tree(dtype, op, (const uint8_t*)vals, has, 0, npes - 1, (uint8_t*)out) : 0;
}

void orc_scatter_results(const void* res_in, const uint64_t* res_pos, uint64_t n,
                         uint32_t elem_bytes, void* res_out) {
    for (uint64_t k = 0; k < n; k++)
        memcpy((uint8_t*)res_out + res_pos[k] * elem_bytes,
               (const uint8_t*)res_in + k * elem_bytes, elem_bytes);
}
