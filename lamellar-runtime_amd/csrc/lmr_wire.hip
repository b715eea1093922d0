// lmr_wire.hip — the reference's op-AM wire format on the owner side (host code).
//
// lmr_am_decode / lmr_am_encode : one op AM struct (bincode legacy, the serde derives of
//                                 impl/src/array_ops.rs:855-997 and the array handles)
// lmr_msg_parse                 : a lamellae message, single AM or batched
//                                 (registered_active_message.rs:227-257, 443-497;
//                                 simple_batcher.rs:276-304)
// lmr_reply_encode              : the Vec<T> / Vec<Result<T,T>> a returning AM sends back
// lmr_apply_msg                 : every op AM of a message applied on the device, small
//                                 AMs of one message aggregated into one record stream per
//                                 (shard, op, operands, value) -- the batcher's counterpart
// Layouts are documented in include/lamellar_gpu_ops.h (AM wire format).
#include <string.h>
#include <vector>
#include <algorithm>
#include "../../include/lamellar_gpu_ops.h"
#include "lmr_internal.hpp"

namespace lmr {

namespace {

// fixed parts (bytes): Option<SerializeHeader> 1 + 2 + 4; AmHeader 4 + 8 + 16;
// DataHeader 8 + 16 + 8; UnitHeader 16; __NetworkDarc 8 + 4 + 8 + 8

struct Reader {
    const uint8_t* p;
    uint64_t len, pos = 0;
    bool ok = true;
    bool need(uint64_t n) {
        if (!ok || pos + n > len || pos + n < pos) ok = false;
        return ok;
    }
    uint64_t uint(int bytes) {
        if (!need(uint64_t(bytes))) return 0;
        uint64_t v = 0;
        memcpy(&v, p + pos, size_t(bytes));          // little endian host
        pos += uint64_t(bytes);
        return v;
    }
    void skip(uint64_t n) { if (need(n)) pos += n; }
};

struct Writer {
    uint8_t* p;
    uint64_t cap, pos = 0;
    void uint(uint64_t v, int bytes) {
        if (p && pos + uint64_t(bytes) <= cap) memcpy(p + pos, &v, size_t(bytes));
        pos += uint64_t(bytes);
    }
    void bytes(const void* src, uint64_t n) {
        if (p && src && pos + n <= cap) memcpy(p + pos, src, size_t(n));
        pos += n;
    }
};

bool valid_kind(uint32_t k) { return k <= LMR_KIND_READ_ONLY; }
bool has_lock_darc(uint32_t k) {
    return k == LMR_KIND_GENERIC_ATOMIC || k == LMR_KIND_LOCAL_LOCK || k == LMR_KIND_GLOBAL_LOCK;
}

void read_darc(Reader& r, lmr_net_darc_t& d) {
    d.inner_addr = r.uint(8);
    d.backend = uint32_t(r.uint(4));
    d.reserved_ = 0;
    d.orig_world_pe = r.uint(8);
    d.orig_team_pe = r.uint(8);
}
void write_darc(Writer& w, const lmr_net_darc_t& d) {
    w.uint(d.inner_addr, 8);
    w.uint(d.backend, 4);
    w.uint(d.orig_world_pe, 8);
    w.uint(d.orig_team_pe, 8);
}

// UnsafeArray<T> { inner: UnsafeArrayInner, phantom } (phantom: zero bytes)
void read_unsafe(Reader& r, lmr_am_view_t& v) {
    read_darc(r, v.data);
    v.distribution = uint32_t(r.uint(4));
    v.orig_elem_per_pe = r.uint(8);
    v.orig_remaining_elems = r.uint(8);
    v.elem_size = r.uint(8);
    v.offset = r.uint(8);
    v.size = r.uint(8);
    v.sub = uint32_t(r.uint(1));
}
void write_unsafe(Writer& w, const lmr_am_view_t& v) {
    write_darc(w, v.data);
    w.uint(v.distribution, 4);
    w.uint(v.orig_elem_per_pe, 8);
    w.uint(v.orig_remaining_elems, 8);
    w.uint(v.elem_size, 8);
    w.uint(v.offset, 8);
    w.uint(v.size, 8);
    w.uint(v.sub ? 1 : 0, 1);
}

}  // namespace

struct WireBufs {
    void* h = nullptr;                  // pinned staging: records in, results out
    size_t hcap = 0;
    void* d = nullptr;
    size_t dcap = 0;
};

void wire_bufs_free(WireBufs* b) {
    if (!b) return;                                  // (lmr_ctx_destroy has drained the device)
    if (b->h) (void)hipHostFree(b->h);
    if (b->d) (void)hipFree(b->d);
    delete b;
}

}  // namespace lmr

using namespace lmr;

extern "C" {

lmr_status_t lmr_am_decode(const uint8_t* body, uint64_t len, uint32_t shape, uint32_t kind, uint32_t dtype,
                           lmr_am_view_t* out) {
    if (!body || !out || shape > LMR_SHAPE_MVSI || !valid_kind(kind) || dtype >= LMR_NUM_DTYPES) return LMR_E_INVALID;
    lmr_am_view_t v;
    memset(&v, 0, sizeof(v));
    v.shape = shape;
    v.kind = kind;
    v.dtype = dtype;
    v.native_type = 0xFFFFFFFFu;
    const int eb = dtype_bytes(int(dtype));
    Reader r{body, len};
    // data: the array handle
    if (has_lock_darc(kind)) read_darc(r, v.lock);
    read_unsafe(r, v);
    if (kind == LMR_KIND_NATIVE_ATOMIC) v.native_type = uint32_t(r.uint(4));
    // op: ArrayOpCmd<T> (u32 tag, CompareExchange(T), CompareExchangeEps(T, T))
    v.op = uint32_t(r.uint(4));
    if (v.op >= LMR_NUM_OPS) return LMR_E_INVALID;
    if (v.op == LMR_OP_COMPARE_EXCHANGE) v.cmp_bits = r.uint(eb);
    if (v.op == LMR_OP_COMPARE_EXCHANGE_EPS) {
        v.cmp_bits = r.uint(eb);
        v.eps_bits = r.uint(eb);
    }
    if (shape == LMR_SHAPE_SVMI) v.val_bits = r.uint(eb);
    const uint64_t nb = r.uint(8);                       // serde_bytes: u64 length + bytes
    v.recs_offset = r.pos;
    v.recs_bytes = nb;
    r.skip(nb);
    if (shape == LMR_SHAPE_MVSI) v.index = r.uint(8);
    else v.index_size = uint32_t(r.uint(1));
    if (!r.ok) return LMR_E_LENGTH;
    if (shape != LMR_SHAPE_MVSI) v.index_size = am_index_width(v.index_size);   // `_ =>`: usize records
    v.body_bytes = r.pos;
    *out = v;
    return LMR_OK;
}

lmr_status_t lmr_am_encode(const lmr_am_view_t* v, const void* recs, uint8_t* out, uint64_t cap, uint64_t* written) {
    if (!v || !written || v->shape > LMR_SHAPE_MVSI || !valid_kind(v->kind) || v->dtype >= LMR_NUM_DTYPES ||
        v->op >= LMR_NUM_OPS || (v->recs_bytes && !recs))
        return LMR_E_INVALID;
    const int eb = dtype_bytes(int(v->dtype));
    Writer w{out, cap};
    if (has_lock_darc(v->kind)) write_darc(w, v->lock);
    write_unsafe(w, *v);
    if (v->kind == LMR_KIND_NATIVE_ATOMIC) w.uint(v->native_type, 4);
    w.uint(v->op, 4);
    if (v->op == LMR_OP_COMPARE_EXCHANGE) w.uint(v->cmp_bits, eb);
    if (v->op == LMR_OP_COMPARE_EXCHANGE_EPS) {
        w.uint(v->cmp_bits, eb);
        w.uint(v->eps_bits, eb);
    }
    if (v->shape == LMR_SHAPE_SVMI) w.uint(v->val_bits, eb);
    w.uint(v->recs_bytes, 8);
    w.bytes(recs, v->recs_bytes);
    if (v->shape == LMR_SHAPE_MVSI) w.uint(v->index, 8);
    else w.uint(v->index_size, 1);
    *written = w.pos;
    return (out && w.pos <= cap) ? LMR_OK : LMR_E_LENGTH;
}

lmr_status_t lmr_msg_parse(const uint8_t* msg, uint64_t len, lmr_am_resolver_t resolve, void* user,
                           lmr_msg_entry_t* entries, uint32_t cap, uint32_t* n) {
    if (!msg || !n) return LMR_E_INVALID;
    *n = 0;
    Reader r{msg, len};
    if (r.uint(1) != 1) return LMR_E_INVALID;            // Option<SerializeHeader>: Some
    const uint32_t src = uint32_t(r.uint(2));
    const uint32_t mcmd = uint32_t(r.uint(4));
    if (!r.ok) return LMR_E_LENGTH;
    uint32_t cnt = 0;
    auto add = [&](const lmr_msg_entry_t& e) -> bool {
        if (cnt < cap && entries) entries[cnt] = e;
        cnt++;
        return true;
    };
    // one [header][body] entry of command c at r.pos
    auto entry = [&](uint32_t c) -> lmr_status_t {
        lmr_msg_entry_t e;
        memset(&e, 0, sizeof(e));
        e.cmd = c;
        e.src = src;
        if (c == LMR_CMD_AM || c == LMR_CMD_RETURN_AM) {
            e.am_id = int32_t(uint32_t(r.uint(4)));
            e.team_addr = r.uint(8);
            e.req_id = r.uint(8);
            e.req_sub_id = r.uint(8);
            if (!r.ok) return LMR_E_LENGTH;
            uint64_t fb = 0;
            const int rc = resolve ? resolve(user, c, e.am_id, msg + r.pos, len - r.pos, &e.shape, &e.kind, &e.dtype, &fb)
                                   : 2;
            if (rc == 1) {                               // a ReturnAm / user AM, sized by the runtime
                if (fb > len - r.pos) return LMR_E_LENGTH;
                e.shape = LMR_SHAPE_FOREIGN;
                e.kind = e.dtype = 0;
                e.body_offset = r.pos;
                e.body_bytes = fb;
                r.skip(fb);
                add(e);
                return LMR_OK;
            }
            if (rc != 0 || c == LMR_CMD_RETURN_AM || e.shape > LMR_SHAPE_MVSI)
                return LMR_E_UNSUPPORTED;                // unknown: its serialized size is unknown here
            lmr_am_view_t v;
            lmr_status_t st = lmr_am_decode(msg + r.pos, len - r.pos, e.shape, e.kind, e.dtype, &v);
            if (st != LMR_OK) return st;
            e.body_offset = r.pos;
            e.body_bytes = v.body_bytes;
            r.skip(v.body_bytes);
        } else if (c == LMR_CMD_DATA) {
            const uint64_t size = r.uint(8);
            e.req_id = r.uint(8);
            e.req_sub_id = r.uint(8);
            const uint64_t darcs = r.uint(8);
            r.skip(darcs);
            e.body_offset = r.pos;
            e.body_bytes = size;
            r.skip(size);
        } else if (c == LMR_CMD_UNIT) {
            e.req_id = r.uint(8);
            e.req_sub_id = r.uint(8);
            e.body_offset = r.pos;
        } else {
            return LMR_E_INVALID;
        }
        if (!r.ok) return LMR_E_LENGTH;
        add(e);
        return LMR_OK;
    };
    lmr_status_t st = LMR_OK;
    if (mcmd == LMR_CMD_BATCHED) {
        while (st == LMR_OK && r.pos < len) {
            const uint32_t c = uint32_t(r.uint(4));
            if (!r.ok) return LMR_E_LENGTH;
            if (c == LMR_CMD_BATCHED) return LMR_E_INVALID;   // simple_batcher.rs:299-301
            st = entry(c);
        }
    } else {
        st = entry(mcmd);
    }
    *n = cnt;
    if (st != LMR_OK) return st;
    return cnt > cap ? LMR_E_LENGTH : LMR_OK;
}

uint64_t lmr_reply_bytes(uint32_t dtype, uint32_t ret_kind, uint64_t n) {
    if (dtype >= LMR_NUM_DTYPES) return 0;
    const uint64_t eb = uint64_t(dtype_bytes(int(dtype)));
    if (ret_kind == LMR_RET_VALS) return 8 + n * eb;
    if (ret_kind == LMR_RET_RESULT) return 8 + n * (4 + eb);
    return 0;
}

lmr_status_t lmr_reply_encode(uint32_t dtype, uint32_t ret_kind, uint64_t n, const void* results, const uint8_t* oks,
                              uint8_t* out, uint64_t cap) {
    if (dtype >= LMR_NUM_DTYPES || (ret_kind != LMR_RET_VALS && ret_kind != LMR_RET_RESULT) || !out ||
        (n && !results) || (ret_kind == LMR_RET_RESULT && n && !oks))
        return LMR_E_INVALID;
    if (cap < lmr_reply_bytes(dtype, ret_kind, n)) return LMR_E_LENGTH;
    const uint64_t eb = uint64_t(dtype_bytes(int(dtype)));
    Writer w{out, cap};
    w.uint(n, 8);
    const uint8_t* res = static_cast<const uint8_t*>(results);
    if (ret_kind == LMR_RET_VALS) {
        w.bytes(res, n * eb);
    } else {
        for (uint64_t k = 0; k < n; k++) {
            w.uint(oks[k] ? 0 : 1, 4);                     // Result::Ok = 0, Err = 1
            w.bytes(res + k * eb, eb);
        }
    }
    return LMR_OK;
}

namespace {

struct AmJob {
    uint32_t entry;
    lmr_am_view_t v;
    lmr_shard_t sh;
    uint64_t n;            // records
    uint32_t group;
    uint64_t pos;          // first record inside its group
};

struct Group {
    lmr_apply_desc_t desc;
    uint32_t shape;        // MVSI: one job per group
    uint64_t index;        // MVSI index
    bool scalar;           // SVMI: one value for every record
    uint64_t val_bits;
    uint64_t n = 0;
    uint64_t h_idx = 0, h_val = 0, h_res = 0, h_ok = 0;   // offsets in the staging buffers
};

inline uint64_t al8(uint64_t x) { return (x + 7) & ~uint64_t(7); }

uint64_t load_le(const uint8_t* p, int bytes) {
    uint64_t v = 0;
    memcpy(&v, p, size_t(bytes));
    return v;
}

}  // namespace

lmr_status_t lmr_apply_msg(lmr_ctx_t* ctx, const uint8_t* msg, uint64_t len, lmr_am_resolver_t resolve,
                           lmr_shard_resolver_t shards, void* user, uint8_t* replies, uint64_t reply_cap,
                           uint64_t* reply_offs, uint64_t* reply_lens, uint32_t max_entries, uint32_t* n_entries,
                           lmr_stream_t stream) {
    if (!ctx || !msg || !resolve || !shards || !n_entries) return LMR_E_INVALID;
    uint32_t ne = 0;
    lmr_status_t st = lmr_msg_parse(msg, len, resolve, user, nullptr, 0, &ne);
    if (st != LMR_OK && st != LMR_E_LENGTH) return st;
    *n_entries = ne;
    if (ne > max_entries) return LMR_E_LENGTH;
    std::vector<lmr_msg_entry_t> ent(ne);
    st = lmr_msg_parse(msg, len, resolve, user, ent.data(), ne, &ne);
    if (st != LMR_OK) return st;
    if (reply_offs)
        for (uint32_t e = 0; e < ne; e++) reply_offs[e] = ~uint64_t(0);
    if (reply_lens)
        for (uint32_t e = 0; e < ne; e++) reply_lens[e] = 0;
    // ---- decode, resolve shards, group
    std::vector<AmJob> jobs;
    std::vector<Group> groups;
    for (uint32_t e = 0; e < ne; e++) {
        if (ent[e].cmd != LMR_CMD_AM || ent[e].shape == LMR_SHAPE_FOREIGN) continue;
        AmJob j;
        j.entry = e;
        st = lmr_am_decode(msg + ent[e].body_offset, len - ent[e].body_offset, ent[e].shape, ent[e].kind,
                           ent[e].dtype, &j.v);
        if (st != LMR_OK) return st;
        memset(&j.sh, 0, sizeof(j.sh));
        if (shards(user, &j.v, &j.sh) != 0 || !j.sh.shard) continue;
        if (!lmr_op_supported(j.v.kind, j.v.dtype, j.v.op)) return LMR_E_UNSUPPORTED;
        const uint32_t eb = uint32_t(dtype_bytes(int(j.v.dtype)));
        if (j.v.shape == LMR_SHAPE_MVMI) {
            const uint32_t rb = lmr_record_bytes(j.v.index_size, j.v.dtype);
            if (!rb || j.v.recs_bytes % rb) return LMR_E_LENGTH;
            j.n = j.v.recs_bytes / rb;
        } else if (j.v.shape == LMR_SHAPE_SVMI) {
            if (j.v.recs_bytes % j.v.index_size) return LMR_E_LENGTH;
            j.n = j.v.recs_bytes / j.v.index_size;
        } else {
            if (j.v.recs_bytes % eb) return LMR_E_LENGTH;
            j.n = j.v.recs_bytes / eb;
        }
        lmr_apply_desc_t d;
        memset(&d, 0, sizeof(d));
        d.shard = j.sh.shard;
        d.shard_len = j.sh.shard_len;
        d.kind = j.v.kind;
        d.dtype = j.v.dtype;
        d.op = j.v.op;
        d.strategy = j.sh.strategy;
        d.cmp_bits = j.v.cmp_bits;
        d.eps_bits = j.v.eps_bits;
        const bool scalar = j.v.shape == LMR_SHAPE_SVMI;
        uint32_t g = uint32_t(groups.size());
        if (j.v.shape != LMR_SHAPE_MVSI) {
            for (uint32_t q = 0; q < groups.size(); q++) {
                const Group& G = groups[q];
                if (G.shape != LMR_SHAPE_MVSI && G.desc.shard == d.shard && G.desc.shard_len == d.shard_len &&
                    G.desc.kind == d.kind && G.desc.dtype == d.dtype && G.desc.op == d.op &&
                    G.desc.strategy == d.strategy && G.desc.cmp_bits == d.cmp_bits && G.desc.eps_bits == d.eps_bits &&
                    G.scalar == scalar && (!scalar || G.val_bits == j.v.val_bits)) {
                    g = q;
                    break;
                }
            }
        }
        if (g == groups.size()) {
            Group G;
            G.desc = d;
            G.shape = j.v.shape;
            G.index = j.v.index;
            G.scalar = scalar;
            G.val_bits = scalar ? j.v.val_bits : 0;
            groups.push_back(G);
        }
        j.group = g;
        j.pos = groups[g].n;
        groups[g].n += j.n;
        jobs.push_back(j);
    }
    if (jobs.empty()) return LMR_OK;
    // ---- staging layout: [idx u64 | vals] per group, then [results | oks] per group
    uint64_t in_bytes = 0, out_bytes = 0;
    for (Group& G : groups) {
        const uint64_t eb = uint64_t(dtype_bytes(int(G.desc.dtype)));
        G.h_idx = in_bytes;
        if (G.shape != LMR_SHAPE_MVSI) in_bytes += al8(G.n * 8);
        G.h_val = in_bytes;
        if (!G.scalar) in_bytes += al8(G.n * eb);
        const uint32_t rk = lmr_op_ret_kind(G.desc.op);
        G.h_res = out_bytes;
        if (rk != LMR_RET_NONE) out_bytes += al8(G.n * eb);
        G.h_ok = out_bytes;
        if (rk == LMR_RET_RESULT) out_bytes += al8(G.n);
    }
    // replies: offsets in entry order
    uint64_t rtot = 0;
    for (const AmJob& j : jobs) {
        const uint32_t rk = lmr_op_ret_kind(j.v.op);
        if (rk == LMR_RET_NONE) continue;
        if (reply_offs) reply_offs[j.entry] = rtot;
        if (reply_lens) reply_lens[j.entry] = lmr_reply_bytes(j.v.dtype, rk, j.n);
        rtot += lmr_reply_bytes(j.v.dtype, rk, j.n);
    }
    if (rtot && (!replies || !reply_offs || rtot > reply_cap)) return LMR_E_LENGTH;
    if (!ctx->wire) ctx->wire = new WireBufs();
    WireBufs* B = ctx->wire;
    (void)hipSetDevice(ctx->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uint64_t need = in_bytes + out_bytes + 64;
    if (B->hcap < need || B->dcap < need) {
        if (hipStreamSynchronize(s) != hipSuccess) return LMR_E_HIP;
        if (B->hcap < need) {
            if (B->h) (void)hipHostFree(B->h);
            B->h = nullptr;
            B->hcap = 0;
            if (hipHostMalloc(&B->h, need + need / 4, hipHostMallocDefault) != hipSuccess) return LMR_E_HIP;
            B->hcap = need + need / 4;
        }
        if (B->dcap < need) {
            if (B->d) (void)hipFree(B->d);
            B->d = nullptr;
            B->dcap = 0;
            if (hipMalloc(&B->d, need + need / 4) != hipSuccess) return LMR_E_HIP;
            B->dcap = need + need / 4;
        }
    }
    // the previous call's copies out of the staging buffer are complete (every return after
    // its first copy waited for the stream); fill records
    uint8_t* H = static_cast<uint8_t*>(B->h);
    uint8_t* D = static_cast<uint8_t*>(B->d);
    for (const AmJob& j : jobs) {
        const Group& G = groups[j.group];
        const int eb = dtype_bytes(int(j.v.dtype));
        const uint8_t* recs = msg + ent[j.entry].body_offset + j.v.recs_offset;
        uint64_t* hidx = reinterpret_cast<uint64_t*>(H + G.h_idx) + j.pos;
        uint8_t* hval = H + G.h_val + j.pos * uint64_t(eb);
        if (j.v.shape == LMR_SHAPE_MVMI) {
            const uint32_t rb = lmr_record_bytes(j.v.index_size, j.v.dtype);
            const uint32_t vo = lmr_record_val_offset(j.v.index_size, j.v.dtype);
            for (uint64_t k = 0; k < j.n; k++) {
                hidx[k] = load_le(recs + k * rb, int(j.v.index_size));
                memcpy(hval + k * uint64_t(eb), recs + k * rb + vo, size_t(eb));
            }
        } else if (j.v.shape == LMR_SHAPE_SVMI) {
            for (uint64_t k = 0; k < j.n; k++) hidx[k] = load_le(recs + k * j.v.index_size, int(j.v.index_size));
        } else {
            memcpy(H + G.h_val, recs, size_t(j.n * uint64_t(eb)));
        }
    }
    // from the first queued copy on, every return waits for the stream: the next call refills H
    struct SyncOnExit {
        hipStream_t s;
        bool armed = true;
        ~SyncOnExit() { if (armed) (void)hipStreamSynchronize(s); }
    } drain{s};
    if (in_bytes && hipMemcpyAsync(D, H, in_bytes, hipMemcpyHostToDevice, s) != hipSuccess) return LMR_E_HIP;
    uint8_t* Dout = D + in_bytes;
    for (const Group& G : groups) {
        if (G.n == 0) continue;
        const uint32_t rk = lmr_op_ret_kind(G.desc.op);
        void* dres = rk != LMR_RET_NONE ? Dout + G.h_res : nullptr;
        uint8_t* dok = rk == LMR_RET_RESULT ? Dout + G.h_ok : nullptr;
        if (G.shape == LMR_SHAPE_MVSI) {
            st = lmr_apply_mvsi(ctx, &G.desc, D + G.h_val, G.n, G.index, dres, dok, stream);
        } else {
            const uint64_t vb = G.val_bits;
            st = lmr_apply_soa(ctx, &G.desc, D + G.h_idx, 8, G.scalar ? nullptr : D + G.h_val, G.scalar ? &vb : nullptr,
                               G.n, dres, dok, stream);
        }
        if (st != LMR_OK) return st;
    }
    if (out_bytes && hipMemcpyAsync(H + in_bytes, Dout, out_bytes, hipMemcpyDeviceToHost, s) != hipSuccess)
        return LMR_E_HIP;
    drain.armed = false;
    if (hipStreamSynchronize(s) != hipSuccess) return LMR_E_HIP;
    // ---- replies
    const uint8_t* Hout = H + in_bytes;
    for (const AmJob& j : jobs) {
        const uint32_t rk = lmr_op_ret_kind(j.v.op);
        if (rk == LMR_RET_NONE) continue;
        const Group& G = groups[j.group];
        const uint64_t eb = uint64_t(dtype_bytes(int(j.v.dtype)));
        const uint64_t off = reply_offs[j.entry];
        st = lmr_reply_encode(j.v.dtype, rk, j.n, Hout + G.h_res + j.pos * eb,
                              rk == LMR_RET_RESULT ? Hout + G.h_ok + j.pos : nullptr, replies + off, reply_cap - off);
        if (st != LMR_OK) return st;
    }
    return LMR_OK;
}

}  // extern "C"
