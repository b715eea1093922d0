/*
 * cpu_baseline.c — CPU BASELINE FOR bench.py ONLY (see cpu_baseline.h).
 */
#define _GNU_SOURCE
#include "cpu_baseline.h"
#include "lamellar_oracle.h"
#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

typedef struct {
    uint32_t dtype, op, index_size, rb, vo, tb;
    void* shard;
    uint64_t shard_len;
    const uint64_t* gidx;
    const uint8_t* vals;
    const uint8_t* val;
    uint64_t n;
    uint64_t num_per_batch;
    uint8_t* bytes;        /* n records */
    uint8_t* locks;        /* per element, floats only */
    uint64_t cmp_bits;     /* compare_exchange(current) */
    void* results;
    /* op buffers: [buf_start[b], buf_start[b+1]) record ranges */
    uint64_t* buf_start;
    uint64_t n_bufs;
    uint64_t next_buf;     /* work counter */
    int status;
    uint32_t nchunks;
    uint64_t chunk_lo[1024], chunk_hi[1024];
} job_t;

typedef struct { job_t* j; uint32_t id; } targ_t;

/* pack one chunk: 1 PE, so records keep input order and op buffers are
 * consecutive runs of num_per_batch records inside the chunk. */
static void* pack_thread(void* p) {
    targ_t* t = (targ_t*)p;
    job_t* j = t->j;
    for (uint64_t k = j->chunk_lo[t->id]; k < j->chunk_hi[t->id]; k++) {
        uint64_t idx = j->gidx[k];
        uint8_t* r = j->bytes + k * j->rb;
        if (idx >= j->shard_len) { j->status = LMR_E_OOB; idx = 0; }
        switch (j->index_size) {
        case 1: r[0] = (uint8_t)idx; break;
        case 2: { uint16_t x = (uint16_t)idx; memcpy(r, &x, 2); break; }
        case 4: { uint32_t x = (uint32_t)idx; memcpy(r, &x, 4); break; }
        default: memcpy(r, &idx, 8); break;
        }
        memcpy(r + j->vo, j->vals ? j->vals + k * j->tb : j->val, j->tb);
    }
    return NULL;
}

#define CAS_LOOP(T, EXPR)                                                                  \
    do {                                                                                   \
        T old = __atomic_load_n(a, __ATOMIC_SEQ_CST), nw;                                  \
        for (;;) {                                                                         \
            nw = (T)(EXPR);                                                                \
            if (__atomic_compare_exchange_n(a, &old, nw, 0, __ATOMIC_SEQ_CST,              \
                                            __ATOMIC_SEQ_CST)) break;                      \
            sched_yield();                                                                 \
        }                                                                                  \
        res = old;                                                                         \
    } while (0)

#define NATIVE_APPLY(NAME, T, UT, WT)                                                      \
static T native_##NAME(T* a, T v, uint32_t op, uint64_t cmp_bits) {                        \
    T res = 0;                                                                             \
    switch (op) {                                                                          \
    case LMR_OP_COMPARE_EXCHANGE: {                                                        \
        /* array_ops.rs:387-390: compare_exchange(current, new) -> Ok(current) / Err(actual) */ \
        T cur; memcpy(&cur, &cmp_bits, sizeof(T));                                          \
        T exp = cur;                                                                       \
        __atomic_compare_exchange_n(a, &exp, v, 0, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);   \
        res = exp; break; }                                                                \
    case LMR_OP_ADD: case LMR_OP_FETCH_ADD: res = __atomic_fetch_add(a, v, __ATOMIC_SEQ_CST); break; \
    case LMR_OP_SUB: case LMR_OP_FETCH_SUB: res = __atomic_fetch_sub(a, v, __ATOMIC_SEQ_CST); break; \
    case LMR_OP_AND: case LMR_OP_FETCH_AND: res = __atomic_fetch_and(a, v, __ATOMIC_SEQ_CST); break; \
    case LMR_OP_OR: case LMR_OP_FETCH_OR: res = __atomic_fetch_or(a, v, __ATOMIC_SEQ_CST); break; \
    case LMR_OP_XOR: case LMR_OP_FETCH_XOR: res = __atomic_fetch_xor(a, v, __ATOMIC_SEQ_CST); break; \
    case LMR_OP_MUL: case LMR_OP_FETCH_MUL: CAS_LOOP(T, (UT)((WT)(UT)old * (WT)(UT)v)); break; \
    case LMR_OP_SWAP: case LMR_OP_STORE: case LMR_OP_PUT:                                  \
        res = __atomic_exchange_n(a, v, __ATOMIC_SEQ_CST); break;                          \
    case LMR_OP_LOAD: case LMR_OP_GET: res = __atomic_load_n(a, __ATOMIC_SEQ_CST); break;  \
    default: res = __atomic_fetch_add(a, v, __ATOMIC_SEQ_CST); break;                      \
    }                                                                                      \
    return res;                                                                            \
}

NATIVE_APPLY(u8, uint8_t, uint8_t, uint32_t)
NATIVE_APPLY(u16, uint16_t, uint16_t, uint32_t)
NATIVE_APPLY(u32, uint32_t, uint32_t, uint64_t)
NATIVE_APPLY(u64, uint64_t, uint64_t, uint64_t)
NATIVE_APPLY(i8, int8_t, uint8_t, uint32_t)
NATIVE_APPLY(i16, int16_t, uint16_t, uint32_t)
NATIVE_APPLY(i32, int32_t, uint32_t, uint64_t)
NATIVE_APPLY(i64, int64_t, uint64_t, uint64_t)

#define GENERIC_APPLY(NAME, T, FMOD)                                                       \
static T generic_##NAME(T* a, uint8_t* lock, T v, uint32_t op) {                           \
    while (__atomic_test_and_set(lock, __ATOMIC_ACQUIRE)) sched_yield();                   \
    T old = *a;                                                                            \
    switch (op) {                                                                          \
    case LMR_OP_ADD: case LMR_OP_FETCH_ADD: *a = old + v; break;                           \
    case LMR_OP_SUB: case LMR_OP_FETCH_SUB: *a = old - v; break;                           \
    case LMR_OP_MUL: case LMR_OP_FETCH_MUL: *a = old * v; break;                           \
    case LMR_OP_DIV: case LMR_OP_FETCH_DIV: *a = old / v; break;                           \
    case LMR_OP_REM: case LMR_OP_FETCH_REM: *a = FMOD(old, v); break;                      \
    case LMR_OP_SWAP: case LMR_OP_STORE: case LMR_OP_PUT: *a = v; break;                   \
    default: break;                                                                        \
    }                                                                                      \
    __atomic_clear(lock, __ATOMIC_RELEASE);                                                \
    return old;                                                                            \
}

GENERIC_APPLY(f32, float, fmodf)
GENERIC_APPLY(f64, double, fmod)

static void* apply_thread(void* p) {
    job_t* j = ((targ_t*)p)->j;
    const int ret = orc_op_ret_kind(j->op) != LMR_RET_NONE && j->results;
    for (;;) {
        uint64_t b = __atomic_fetch_add(&j->next_buf, 1, __ATOMIC_RELAXED);
        if (b >= j->n_bufs) break;
        for (uint64_t k = j->buf_start[b]; k < j->buf_start[b + 1]; k++) {
            const uint8_t* r = j->bytes + k * j->rb;
            uint64_t idx = 0;
            memcpy(&idx, r, j->index_size);
            const uint8_t* vp = r + j->vo;
#define DO(D, NAME, T)                                                                     \
            case D: { T v; memcpy(&v, vp, sizeof(T));                                      \
                T o = native_##NAME((T*)j->shard + idx, v, j->op, j->cmp_bits);            \
                if (ret) { ((T*)j->results)[k] = o; } break; }
#define DOF(D, NAME, T)                                                                    \
            case D: { T v; memcpy(&v, vp, sizeof(T));                                      \
                T o = generic_##NAME((T*)j->shard + idx, j->locks + idx, v, j->op);        \
                if (ret) { ((T*)j->results)[k] = o; } break; }
            switch (j->dtype) {
            DO(LMR_U8, u8, uint8_t) DO(LMR_U16, u16, uint16_t) DO(LMR_U32, u32, uint32_t)
            DO(LMR_U64, u64, uint64_t) DO(LMR_I8, i8, int8_t) DO(LMR_I16, i16, int16_t)
            DO(LMR_I32, i32, int32_t) DO(LMR_I64, i64, int64_t)
            DOF(LMR_F32, f32, float) DOF(LMR_F64, f64, double)
            default: break;
            }
#undef DO
#undef DOF
        }
    }
    return NULL;
}

int cpu_baseline_run(uint32_t dtype, uint32_t op, void* shard, uint64_t shard_len,
                     const uint64_t* gidx, const void* vals, const void* val, uint64_t n,
                     uint32_t threads, uint64_t am_size_threshold, const void* cmp, void* results,
                     cpu_times_t* out) {
    if (threads == 0) threads = 1;
    if (threads > 1024) threads = 1024;
    job_t* j = (job_t*)calloc(1, sizeof(job_t));
    if (!j) return LMR_E_WORKSPACE;
    lmr_layout_t L;
    orc_layout_new(&L, shard_len, 1, 0, LMR_DIST_BLOCK);
    j->dtype = dtype; j->op = op;
    j->index_size = orc_index_size(&L);
    j->tb = orc_dtype_bytes(dtype);
    j->rb = orc_record_bytes(j->index_size, dtype);
    j->vo = orc_record_val_offset(j->index_size, dtype);
    j->shard = shard; j->shard_len = shard_len; j->gidx = gidx;
    j->vals = (const uint8_t*)vals; j->val = (const uint8_t*)val; j->n = n;
    j->results = results;
    if (cmp) memcpy(&j->cmp_bits, cmp, j->tb);
    j->num_per_batch = (uint64_t)ceilf((float)am_size_threshold / (float)j->rb);
    if (j->num_per_batch == 0) j->num_per_batch = 1;
    j->bytes = (uint8_t*)malloc(n * j->rb + 1);
    if (dtype == LMR_F32 || dtype == LMR_F64) j->locks = (uint8_t*)calloc(shard_len, 1);
    /* chunking (operations.rs:455-480) with batch_op_threads = max(1, T/4) */
    uint32_t packers = threads / 4 ? threads / 4 : 1;
    uint64_t nch = orc_num_chunks(n, packers);
    if (nch > 1024) nch = 1024;
    j->nchunks = (uint32_t)nch;
    uint64_t num = n < 1000 ? 1 : packers, per = num ? n / num : n;
    for (uint64_t c = 0; c < nch; c++) {
        j->chunk_lo[c] = c < num ? c * per : num * per;
        j->chunk_hi[c] = c < num ? (c + 1) * per : n;
    }
    /* op buffers: consecutive num_per_batch runs inside each chunk */
    uint64_t maxb = n / j->num_per_batch + nch + 2;
    j->buf_start = (uint64_t*)malloc((maxb + 1) * sizeof(uint64_t));
    if (!j->bytes || !j->buf_start || ((dtype == LMR_F32 || dtype == LMR_F64) && !j->locks)) {
        free(j->bytes); free(j->buf_start); free(j->locks); free(j);
        return LMR_E_WORKSPACE;
    }
    uint64_t nb = 0;
    for (uint64_t c = 0; c < nch; c++)
        for (uint64_t s = j->chunk_lo[c]; s < j->chunk_hi[c]; s += j->num_per_batch)
            j->buf_start[nb++] = s;
    j->buf_start[nb] = n;
    j->n_bufs = nb;

    pthread_t* th = (pthread_t*)malloc((threads + nch) * sizeof(pthread_t));
    targ_t* ta = (targ_t*)malloc((threads + nch) * sizeof(targ_t));
    double t0 = now_s();
    for (uint32_t c = 0; c < j->nchunks; c++) { ta[c].j = j; ta[c].id = c; pthread_create(&th[c], NULL, pack_thread, &ta[c]); }
    for (uint32_t c = 0; c < j->nchunks; c++) pthread_join(th[c], NULL);
    double t1 = now_s();
    j->next_buf = 0;
    for (uint32_t c = 0; c < threads; c++) { ta[c].j = j; ta[c].id = c; pthread_create(&th[c], NULL, apply_thread, &ta[c]); }
    for (uint32_t c = 0; c < threads; c++) pthread_join(th[c], NULL);
    double t2 = now_s();
    if (out) { out->pack_s = t1 - t0; out->apply_s = t2 - t1; out->total_s = t2 - t0; out->n_buffers = nb; }
    int st = j->status;
    free(th); free(ta); free(j->bytes); free(j->buf_start); free(j->locks); free(j);
    return st;
}
