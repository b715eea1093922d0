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

/* ------------------------------------------------------------------------------------
 * C4: P PEs on one node exchanging op buffers through shared memory, as the
 * shmem lamellae does (lamellar_run.sh:31-40 starts one process per PE). Each PE is a group
 * of threads here (every PE's memory is visible to every other, like the /dev/shm
 * segments); per PE:
 *  - packers (max(1, T/4) chunks, operations.rs:462-480) map each global index to (PE,
 *    offset) (unsafe.rs:1610-1647) and append IdxVal records to per-destination op buffers
 *    of am_size_threshold bytes (unsafe/operations.rs:663-811), allocated in the sender's
 *    own segment; a full buffer is sent: to the PE itself it is queued as is (the dst == src
 *    shortcut, registered_active_message.rs:150-154), to another PE a CmdMsg {addr, size,
 *    hash} goes into the destination's command queue with the additive checksum of the
 *    bytes (command_queues.rs:26-35, 63-94, 725-807);
 *  - every thread of the PE, once its packing is done, serves the PE's queue: a remote
 *    buffer is copied out of the sender's segment and its checksum verified (get_data,
 *    command_queues.rs:996-1021, 1395-1531), then its records are applied with SeqCst
 *    atomics (the NativeAtomic apply above).
 * The step ends when every PE has applied every buffer addressed to it.
 * ------------------------------------------------------------------------------------ */
typedef struct {
    const uint8_t* addr;
    uint64_t bytes;
    uint64_t hash;       /* 0 for the dst == src shortcut (no copy, no check) */
} cmd_msg_t;

typedef struct {
    pthread_mutex_t mu;
    cmd_msg_t* q;
    uint64_t head, tail, cap;
} cmd_queue_t;

typedef struct mpe_s mpe_t;
typedef struct {
    mpe_t* m;
    uint32_t pe;
    uint8_t* seg;             /* this PE's segment: op buffers are carved from it */
    uint64_t seg_used;        /* bump pointer (atomic) */
    uint64_t seg_cap;
    void* shard;
    cmd_queue_t queue;
    const uint64_t* gidx;
    const uint8_t* vals;
    uint64_t n;
    uint32_t packers;
} mpe_pe_t;

struct mpe_s {
    uint32_t npes, tpe, dtype, op, index_size, rb, vo, tb;
    lmr_layout_t L;
    uint64_t per_batch;       /* records per op buffer */
    mpe_pe_t* pe;
    uint32_t packers_left;    /* atomic: packing threads still running, over all PEs */
    uint64_t sent, applied;   /* atomic buffer counts */
    int status;
};

typedef struct { mpe_t* m; uint32_t pe, t; } mpe_arg_t;

static uint64_t add_hash(const uint8_t* p, uint64_t len) {
    uint64_t s = 0, w;
    uint64_t k = 0;
    for (; k + 8 <= len; k += 8) { memcpy(&w, p + k, 8); s += w; }
    for (; k < len; k++) s += p[k];
    return s;
}

static void q_push(cmd_queue_t* q, cmd_msg_t c) {
    pthread_mutex_lock(&q->mu);
    if (q->tail == q->cap) {
        uint64_t nc = q->cap ? 2 * q->cap : 1024;
        cmd_msg_t* nq = (cmd_msg_t*)realloc(q->q, nc * sizeof(cmd_msg_t));
        if (nq) { q->q = nq; q->cap = nc; }
    }
    if (q->tail < q->cap) q->q[q->tail++] = c;
    pthread_mutex_unlock(&q->mu);
}

static int q_pop(cmd_queue_t* q, cmd_msg_t* c) {
    int got = 0;
    pthread_mutex_lock(&q->mu);
    if (q->head < q->tail) { *c = q->q[q->head++]; got = 1; }
    pthread_mutex_unlock(&q->mu);
    return got;
}

static void mpe_send(mpe_t* m, uint32_t src, uint32_t dst, const uint8_t* buf, uint64_t bytes) {
    cmd_msg_t c = {buf, bytes, src == dst ? 0 : add_hash(buf, bytes)};
    __atomic_fetch_add(&m->sent, 1, __ATOMIC_SEQ_CST);
    q_push(&m->pe[dst].queue, c);
}

static void mpe_apply_buf(mpe_t* m, mpe_pe_t* P, const uint8_t* recs, uint64_t bytes) {
    const uint64_t nr = bytes / m->rb;
    for (uint64_t k = 0; k < nr; k++) {
        const uint8_t* r = recs + k * m->rb;
        uint64_t idx = 0;
        memcpy(&idx, r, m->index_size);
        const uint8_t* vp = r + m->vo;
#define MDO(D, NAME, T) case D: { T v; memcpy(&v, vp, sizeof(T)); (void)native_##NAME((T*)P->shard + idx, v, m->op, 0); break; }
        switch (m->dtype) {
        MDO(LMR_U8, u8, uint8_t) MDO(LMR_U16, u16, uint16_t) MDO(LMR_U32, u32, uint32_t)
        MDO(LMR_U64, u64, uint64_t) MDO(LMR_I8, i8, int8_t) MDO(LMR_I16, i16, int16_t)
        MDO(LMR_I32, i32, int32_t) MDO(LMR_I64, i64, int64_t)
        default: break;
        }
#undef MDO
    }
}

static void* mpe_thread(void* p) {
    mpe_arg_t* a = (mpe_arg_t*)p;
    mpe_t* m = a->m;
    mpe_pe_t* P = &m->pe[a->pe];
    const uint64_t bb = m->per_batch * m->rb;
    if (a->t < P->packers) {
        /* pack chunk t of this PE's input (operations.rs:462-480) */
        const uint64_t per = P->n / P->packers;
        const uint64_t lo = a->t * per, hi = (a->t + 1 == P->packers) ? P->n : lo + per;
        uint8_t** cur = (uint8_t**)calloc(m->npes, sizeof(uint8_t*));
        uint64_t* fill = (uint64_t*)calloc(m->npes, sizeof(uint64_t));
        for (uint64_t k = lo; k < hi; k++) {
            uint64_t pe = 0, off = 0;
            if (!orc_pe_and_offset(&m->L, P->gidx[k], &pe, &off)) { m->status = LMR_E_OOB; continue; }
            if (!cur[pe]) {
                const uint64_t at = __atomic_fetch_add(&P->seg_used, bb, __ATOMIC_RELAXED);
                if (at + bb > P->seg_cap) { m->status = LMR_E_WORKSPACE; continue; }
                cur[pe] = P->seg + at;
                fill[pe] = 0;
            }
            uint8_t* r = cur[pe] + fill[pe] * m->rb;
            memcpy(r, &off, m->index_size);
            memcpy(r + m->vo, P->vals + k * m->tb, m->tb);
            if (++fill[pe] == m->per_batch) {
                mpe_send(m, a->pe, (uint32_t)pe, cur[pe], bb);
                cur[pe] = NULL;
            }
        }
        for (uint32_t pe = 0; pe < m->npes; pe++)
            if (cur[pe] && fill[pe]) mpe_send(m, a->pe, pe, cur[pe], fill[pe] * m->rb);
        free(cur);
        free(fill);
        __atomic_fetch_sub(&m->packers_left, 1, __ATOMIC_SEQ_CST);
    }
    /* serve this PE's command queue until every buffer of every PE is applied */
    uint8_t* local = (uint8_t*)malloc(bb);
    for (;;) {
        cmd_msg_t c;
        if (q_pop(&P->queue, &c)) {
            const uint8_t* src = c.addr;
            if (c.hash) {                                   /* remote: get_data + checksum */
                memcpy(local, c.addr, c.bytes);
                if (add_hash(local, c.bytes) != c.hash) m->status = LMR_E_INVALID;
                src = local;
            }
            mpe_apply_buf(m, P, src, c.bytes);
            __atomic_fetch_add(&m->applied, 1, __ATOMIC_SEQ_CST);
            continue;
        }
        if (__atomic_load_n(&m->packers_left, __ATOMIC_SEQ_CST) == 0 &&
            __atomic_load_n(&m->applied, __ATOMIC_SEQ_CST) == __atomic_load_n(&m->sent, __ATOMIC_SEQ_CST))
            break;
        sched_yield();
    }
    free(local);
    return NULL;
}

int cpu_baseline_multi_pe(uint32_t dtype, uint32_t op, uint32_t npes, uint32_t threads_per_pe, uint64_t array_len,
                          void* const* shards, const uint64_t* const* gidx, const void* const* vals, uint64_t n_per_pe,
                          uint64_t am_size_threshold, cpu_times_t* out) {
    if (npes == 0 || npes > 64 || threads_per_pe == 0 || dtype >= LMR_F32 || orc_op_ret_kind(op) != LMR_RET_NONE)
        return LMR_E_INVALID;
    mpe_t* m = (mpe_t*)calloc(1, sizeof(mpe_t));
    if (!m) return LMR_E_WORKSPACE;
    m->npes = npes; m->tpe = threads_per_pe; m->dtype = dtype; m->op = op;
    orc_layout_new(&m->L, array_len, npes, 0, LMR_DIST_BLOCK);
    m->index_size = orc_index_size(&m->L);
    m->tb = orc_dtype_bytes(dtype);
    m->rb = orc_record_bytes(m->index_size, dtype);
    m->vo = orc_record_val_offset(m->index_size, dtype);
    m->per_batch = (uint64_t)ceilf((float)am_size_threshold / (float)m->rb);
    if (m->per_batch == 0) m->per_batch = 1;
    m->pe = (mpe_pe_t*)calloc(npes, sizeof(mpe_pe_t));
    const uint32_t packers = threads_per_pe / 4 ? threads_per_pe / 4 : 1;
    int st = LMR_OK;
    for (uint32_t p = 0; p < npes && m->pe; p++) {
        mpe_pe_t* P = &m->pe[p];
        P->m = m; P->pe = p; P->shard = shards[p]; P->gidx = gidx[p];
        P->vals = (const uint8_t*)vals[p]; P->n = n_per_pe;
        P->packers = n_per_pe < 1000 ? 1 : packers;
        /* every packer may leave one partial buffer per destination */
        P->seg_cap = (n_per_pe / m->per_batch + (uint64_t)P->packers * npes + 2) * m->per_batch * m->rb;
        P->seg = (uint8_t*)malloc(P->seg_cap);
        pthread_mutex_init(&P->queue.mu, NULL);
        if (!P->seg) st = LMR_E_WORKSPACE;
        m->packers_left += P->packers;
    }
    const uint32_t nt = npes * threads_per_pe;
    pthread_t* th = (pthread_t*)malloc(nt * sizeof(pthread_t));
    mpe_arg_t* ta = (mpe_arg_t*)malloc(nt * sizeof(mpe_arg_t));
    if (!m->pe || !th || !ta) st = LMR_E_WORKSPACE;
    if (st == LMR_OK) {
        const double t0 = now_s();
        for (uint32_t i = 0; i < nt; i++) {
            ta[i].m = m; ta[i].pe = i / threads_per_pe; ta[i].t = i % threads_per_pe;
            pthread_create(&th[i], NULL, mpe_thread, &ta[i]);
        }
        for (uint32_t i = 0; i < nt; i++) pthread_join(th[i], NULL);
        const double t1 = now_s();
        if (out) { out->pack_s = 0; out->apply_s = t1 - t0; out->total_s = t1 - t0; out->n_buffers = m->sent; }
        st = m->status;
    }
    for (uint32_t p = 0; m->pe && p < npes; p++) {
        free(m->pe[p].seg);
        free(m->pe[p].queue.q);
        pthread_mutex_destroy(&m->pe[p].queue.mu);
    }
    free(th); free(ta); free(m->pe); free(m);
    return st;
}
