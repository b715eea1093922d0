/*
 * linearize.c — CPU ORACLE FOR TESTS ONLY: linearisability checker.
 *
 * The reference applies the records of concurrently running op AMs with one
 * SeqCst RMW or CAS loop per record (NativeAtomic, impl/src/array_ops.rs:327-458,
 * src/array/native_atomic.rs:29-113), under a per-element mutex (GenericAtomic,
 * src/array/generic_atomic.rs:286-293) or under a shard lock per AM (LocalLock,
 * array_ops.rs:557-560), and promises no order between records
 * (src/array/operations/arithmetic.rs:57-58). What every kind guarantees is that
 * each element sees its records one at a time: the returned old values (fetch_*,
 * swap, load), the Result<T,T> of compare_exchange(_epsilon) and the final value
 * must be those of SOME serial order of that element's records. This file checks
 * exactly that, per element, for a batch applied to one slice.
 *
 * Method: a depth-first search over serial orders. At state s the candidates are
 * the unused records whose step from s (orc_elem_step, the oracle's own per-record
 * semantics) returns their recorded value and Ok flag. A record that returns the
 * state it ran at fits at that one state only; if it leaves it unchanged it is taken
 * at once and never branched on. Other records (compare_exchange_epsilon successes,
 * ops returning nothing) may fit at several states, as a no-op at one and a change at
 * another, so they are only branched on as changes; any left over when the final
 * value is reached must fit as a no-op at some visited state. Among state-changing
 * candidates only one per
 * distinct value is tried. Records are found through a hash of their returned
 * value; the search gives up after `max_nodes` branch steps (reported apart).
 * When every record of an element returns the state it ran at (fetch_*, swap,
 * load, compare_exchange, failed compare_exchange_epsilon) the question is exactly
 * whether an Eulerian trail exists over the edges (returned value -> next state),
 * which is decided in linear time instead (euler()).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "lamellar_oracle.h"

/* One record applied to a register copy of an element: new state, returned bits, Ok flag.
 * Returns LMR_OK or the error status of the step (division by zero, ...). */
int orc_elem_step(uint32_t kind, uint32_t dtype, uint32_t op, uint64_t state_bits, uint64_t val_bits,
                  const void* cmp, const void* eps, uint64_t* new_bits, uint64_t* ret_bits, uint8_t* ok);

static uint64_t mask_of(uint32_t eb) { return eb >= 8 ? ~0ull : ((1ull << (8 * eb)) - 1ull); }

static uint64_t load_bits(const void* base, uint64_t i, uint32_t eb) {
    uint64_t x = 0;
    memcpy(&x, (const uint8_t*)base + i * eb, eb);
    return x;
}

typedef struct {
    uint32_t kind, dtype, op, eb;
    const void *cmp, *eps;
    int ret_kind;                  /* 0 none, 1 vals, 2 result */
    /* records of the element being checked */
    uint32_t m;
    const uint64_t* v;             /* [m] value bits */
    const uint64_t* r;             /* [m] returned bits (ret_kind > 0) */
    const uint8_t* ok;             /* [m] ok flags (ret_kind == 2) */
    uint8_t* used;                 /* [m] */
    /* hash of records by returned bits: head[h], next[j] */
    uint32_t hcap;
    int32_t* head;
    int32_t* next;
    /* records whose returned value does not name the state they ran at
       (compare_exchange successes, nothing returned): scanned linearly */
    int32_t* other;
    uint32_t nother;
    uint64_t nodes, max_nodes;
    uint32_t tried_cap;            /* entries of the tried stack (levels may re-try a record) */
} Ctx;

static uint32_t hash64(uint64_t x, uint32_t cap) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)(x & (cap - 1));
}

/* does record j step from state s with its recorded result? -> new state in *ns */
static int fits(const Ctx* c, uint32_t j, uint64_t s, uint64_t* ns) {
    uint64_t nb = 0, rb = 0;
    uint8_t okf = 0;
    if (orc_elem_step(c->kind, c->dtype, c->op, s, c->v[j], c->cmp, c->eps, &nb, &rb, &okf) != LMR_OK) return 0;
    const uint64_t mk = mask_of(c->eb);
    if (c->ret_kind >= 1 && ((rb ^ c->r[j]) & mk)) return 0;
    if (c->ret_kind == 2 && (okf != 0) != (c->ok[j] != 0)) return 0;
    *ns = nb & mk;
    return 1;
}

/* whether the recorded return value of record j is the state it ran at (then the
   hash of returned values finds it): fetch_* / swap / load, compare_exchange (Ok
   carries `current`, which is the state it matched; Err the state it saw) and the
   Err of compare_exchange_epsilon (its Ok carries current / new / old by kind) */
static int ret_is_state(const Ctx* c, uint32_t j) {
    if (c->ret_kind == 0) return 0;
    if (c->ret_kind == 1 || c->op == LMR_OP_COMPARE_EXCHANGE) return 1;
    return c->ok[j] == 0;
}

/* When every record returns the state it ran at, record j can only run at state r_j
 * and moves it to to_j = step(r_j, v_j): a serial order is exactly an Eulerian trail
 * over the edges r_j -> to_j from the initial to the final value. Decided exactly in
 * linear time: every vertex balanced once a virtual edge final -> init is added, and
 * every edge in the weakly connected component of init. 1 = yes, 0 = no. */
static uint32_t uf_find(uint32_t* p, uint32_t x) {
    while (p[x] != x) { p[x] = p[p[x]]; x = p[x]; }
    return x;
}

static int euler(const Ctx* c, uint64_t init, uint64_t final_bits, uint64_t* keys, int32_t* ids,
                 uint32_t hcap, int64_t* bal, uint32_t* parent, uint32_t* from, uint32_t* to) {
    const uint64_t mk = mask_of(c->eb);
    uint32_t nv = 0;
    for (uint32_t h = 0; h < hcap; h++) ids[h] = -1;
#define VID(X, OUT)                                                                        \
    do {                                                                                   \
        const uint64_t key_ = (X);                                                         \
        uint32_t h_ = hash64(key_, hcap);                                                  \
        while (ids[h_] >= 0 && keys[h_] != key_) h_ = (h_ + 1) & (hcap - 1);               \
        if (ids[h_] < 0) { ids[h_] = (int32_t)nv; keys[h_] = key_; bal[nv] = 0; parent[nv] = nv; nv++; } \
        (OUT) = (uint32_t)ids[h_];                                                         \
    } while (0)
    uint32_t vi, vf;
    VID(init & mk, vi);
    VID(final_bits & mk, vf);
    for (uint32_t j = 0; j < c->m; j++) {
        uint64_t ns;
        if (!fits(c, j, c->r[j], &ns)) return 0;            /* cannot return r_j from state r_j */
        VID(c->r[j], from[j]);
        VID(ns, to[j]);
    }
#undef VID
    bal[vf] += 1; bal[vi] -= 1;                              /* virtual edge final -> init */
    parent[uf_find(parent, vf)] = uf_find(parent, vi);
    for (uint32_t j = 0; j < c->m; j++) {
        bal[from[j]] += 1;
        bal[to[j]] -= 1;
        const uint32_t a = uf_find(parent, from[j]), b = uf_find(parent, to[j]);
        if (a != b) parent[a] = b;
    }
    const uint32_t root = uf_find(parent, vi);
    for (uint32_t v = 0; v < nv; v++)
        if (bal[v] != 0 || uf_find(parent, v) != root) return 0;
    return 1;
}

typedef struct { uint64_t state; uint32_t trail_len; uint32_t tried_len; } Frame;

/* every record the trail has not used leaves some visited state unchanged there
   (so it can be inserted at that point of the order) */
static int placeable_rest(const Ctx* c, const Frame* stack, uint32_t sp, uint64_t s, uint32_t tl) {
    if (tl == c->m) return 1;
    for (uint32_t j = 0; j < c->m; j++) {
        if (c->used[j]) continue;
        uint64_t ns;
        int ok = fits(c, j, s, &ns) && ns == s;
        for (uint32_t f = 0; !ok && f < sp; f++)
            ok = fits(c, j, stack[f].state, &ns) && ns == stack[f].state;
        if (!ok) return 0;
    }
    return 1;
}

/* Iterative DFS; each level owns the range [tried_len, tr) of values it has tried.
 * 1 = linearisable, 0 = not, -1 = gave up (node budget). */
static int search(Ctx* c, uint64_t init, uint64_t final_bits, uint32_t* trail, uint32_t* tried,
                   Frame* stack) {
    const uint64_t mk = mask_of(c->eb);
    uint64_t s = init & mk;
    uint32_t tl = 0, sp = 0, tr = 0;
    int entering = 1;
    for (;;) {
        if (entering) {
            int progress = 1;
            while (progress) {
                progress = 0;
                for (int32_t j = c->head[hash64(s, c->hcap)]; j >= 0; j = c->next[j]) {
                    uint64_t ns;
                    if (c->used[j] || !ret_is_state(c, (uint32_t)j) || !fits(c, (uint32_t)j, s, &ns) || ns != s)
                        continue;
                    c->used[j] = 1; trail[tl++] = (uint32_t)j; progress = 1;
                }
            }
            /* records of the `other` list are not absorbed on the way: one that is a no-op
               here may be needed elsewhere as a state change (compare_exchange_epsilon with
               |new - current| < eps fits both at `current` and at `new`). Any of them left
               unused at the end is placed as a no-op at a visited state, if one fits. */
            if (s == (final_bits & mk) && placeable_rest(c, stack, sp, s, tl)) return 1;
            stack[sp].state = s;
            stack[sp].trail_len = tl;
            stack[sp].tried_len = tr;
            sp++;
            entering = 0;
        }
        /* try the next untried state-changing candidate of the top level */
        Frame* f = &stack[sp - 1];
        s = f->state;
        while (tl > f->trail_len) c->used[trail[--tl]] = 0;   /* undo the previous pick's subtree */
        int32_t pick = -1;
        uint64_t pick_ns = 0;
        if (tl < c->m) {
            for (int pass = 0; pass < 2 && pick < 0; pass++) {
                int32_t j = pass == 0 ? c->head[hash64(s, c->hcap)] : -1;
                uint32_t q = 0;
                for (;;) {
                    int32_t cur;
                    if (pass == 0) { if (j < 0) break; cur = j; j = c->next[j]; }
                    else { if (q >= c->nother) break; cur = c->other[q++]; }
                    uint64_t ns;
                    if (c->used[cur] || (pass == 0 && !ret_is_state(c, (uint32_t)cur))) continue;
                    if (!fits(c, (uint32_t)cur, s, &ns) || ns == s) continue;
                    int dup = 0;
                    for (uint32_t t = f->tried_len; t < tr; t++)
                        if (c->v[tried[t]] == c->v[cur]) { dup = 1; break; }
                    if (dup) continue;
                    pick = cur; pick_ns = ns;
                    break;
                }
            }
        }
        if (pick < 0) {                     /* level exhausted: pop it */
            tr = f->tried_len;
            sp--;
            if (sp == 0) return 0;
            /* the parent's tried list must not include entries of this popped level:
               they were appended after the parent's own pick, so keep the parent's
               range up to (and including) its pick */
            continue;
        }
        if (++c->nodes > c->max_nodes || tr >= c->tried_cap) return -1;
        /* this level's tried range is [f->tried_len, tr); deeper levels append after it,
           and are truncated back to tr when they pop */
        tried[tr++] = (uint32_t)pick;
        c->used[pick] = 1;
        trail[tl++] = (uint32_t)pick;
        s = pick_ns;
        entering = 1;
    }
}

int orc_check_linearizable(uint32_t kind, uint32_t dtype, uint32_t op, const void* cmp, const void* eps,
                           const void* init_slice, const void* final_slice, uint64_t slice_len,
                           const uint64_t* idx, uint64_t n, const void* vals, uint64_t v_len,
                           const void* rets, const uint8_t* oks, uint64_t max_nodes,
                           uint64_t* bad_elem) {
    const uint32_t eb = orc_dtype_bytes(dtype);
    if (!eb) return -2;
    int ret_kind = (int)orc_op_ret_kind(op);
    if (!rets) ret_kind = 0;
    if (ret_kind == 2 && !oks) ret_kind = 1;
    /* CSR of records by element */
    uint32_t* cnt = calloc(slice_len + 1, sizeof(uint32_t));
    uint32_t* ord = malloc((n ? n : 1) * sizeof(uint32_t));
    if (!cnt || !ord) { free(cnt); free(ord); return -2; }
    for (uint64_t k = 0; k < n; k++)
        if (idx[k] < slice_len) cnt[idx[k] + 1]++;
    for (uint64_t e = 0; e < slice_len; e++) cnt[e + 1] += cnt[e];
    uint32_t* fill = malloc((slice_len + 1) * sizeof(uint32_t));
    memcpy(fill, cnt, (slice_len + 1) * sizeof(uint32_t));
    for (uint64_t k = 0; k < n; k++)
        if (idx[k] < slice_len) ord[fill[idx[k]]++] = (uint32_t)k;
    free(fill);
    uint32_t mmax = 0;
    for (uint64_t e = 0; e < slice_len; e++)
        if (cnt[e + 1] - cnt[e] > mmax) mmax = cnt[e + 1] - cnt[e];
    uint32_t hcap = 16;
    while (hcap < 2 * mmax) hcap <<= 1;
    uint64_t* v = malloc((mmax + 1) * 8);
    uint64_t* r = malloc((mmax + 1) * 8);
    uint8_t* okv = malloc(mmax + 1);
    uint8_t* used = malloc(mmax + 1);
    int32_t* head = malloc(hcap * sizeof(int32_t));
    int32_t* next = malloc((mmax + 1) * sizeof(int32_t));
    int32_t* other = malloc((mmax + 1) * sizeof(int32_t));
    uint32_t* trail = malloc((mmax + 1) * sizeof(uint32_t));
    const uint32_t tried_cap = 4 * (mmax + 1) + 64;
    uint32_t* tried = malloc((size_t)tried_cap * sizeof(uint32_t));
    Frame* stack = malloc((mmax + 2) * sizeof(Frame));
    uint32_t ecap = 16;
    while (ecap < 4 * (mmax + 2)) ecap <<= 1;
    uint64_t* ekeys = malloc((size_t)ecap * 8);
    int32_t* eids = malloc((size_t)ecap * sizeof(int32_t));
    int64_t* ebal = malloc((size_t)(2 * mmax + 4) * 8);
    uint32_t* epar = malloc((size_t)(2 * mmax + 4) * 4);
    uint32_t* efrom = malloc((size_t)(mmax + 1) * 4);
    uint32_t* eto = malloc((size_t)(mmax + 1) * 4);
    int result = 0;
    if (!v || !r || !okv || !used || !head || !next || !other || !trail || !tried || !stack || !ekeys || !eids ||
        !ebal || !epar || !efrom || !eto) {
        result = -2;
        goto done;
    }
    Ctx c;
    memset(&c, 0, sizeof(c));
    c.kind = kind; c.dtype = dtype; c.op = op; c.eb = eb; c.cmp = cmp; c.eps = eps;
    c.ret_kind = ret_kind; c.v = v; c.r = r; c.ok = okv; c.used = used;
    c.hcap = hcap; c.head = head; c.next = next; c.other = other; c.max_nodes = max_nodes;
    c.tried_cap = tried_cap;
    const uint64_t mk = mask_of(eb);
    for (uint64_t e = 0; e < slice_len; e++) {
        const uint32_t m = cnt[e + 1] - cnt[e];
        const uint64_t init = load_bits(init_slice, e, eb), fin = load_bits(final_slice, e, eb);
        if (m == 0) {
            if ((init ^ fin) & mk) { result = 1; *bad_elem = e; goto done; }
            continue;
        }
        c.m = m;
        c.nother = 0;
        c.nodes = 0;
        uint32_t hc = 16;
        while (hc < 2 * m) hc <<= 1;
        c.hcap = hc;
        for (uint32_t h = 0; h < hc; h++) head[h] = -1;
        for (uint32_t q = 0; q < m; q++) {
            const uint32_t k = ord[cnt[e] + q];
            v[q] = load_bits(vals, v_len == 1 ? 0 : k, eb) & mk;
            r[q] = ret_kind ? (load_bits(rets, k, eb) & mk) : 0;
            okv[q] = (ret_kind == 2) ? oks[k] : 0;
            used[q] = 0;
        }
        for (uint32_t q = m; q-- > 0;) {
            if (ret_is_state(&c, q)) {
                const uint32_t h = hash64(r[q], hc);
                next[q] = head[h];
                head[h] = (int32_t)q;
            } else {
                other[c.nother++] = (int32_t)q;
            }
        }
        uint32_t ec = 16;
        while (ec < 4 * (m + 2)) ec <<= 1;
        const int st = (c.ret_kind > 0 && c.nother == 0)
                           ? euler(&c, init, fin, ekeys, eids, ec, ebal, epar, efrom, eto)
                           : search(&c, init, fin, trail, tried, stack);
        if (st != 1) { result = st == 0 ? 1 : 2; *bad_elem = e; goto done; }
    }
done:
    free(cnt); free(ord); free(v); free(r); free(okv); free(used); free(head); free(next); free(other);
    free(trail); free(tried); free(stack); free(ekeys); free(eids); free(ebal); free(epar); free(efrom); free(eto);
    return result;
}
