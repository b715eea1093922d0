"""Messages from the running runtime applied on the device (lmr_apply_msg): one batched
lamellae message of 220 small op AMs (MVMI / SVMI / MVSI, four ops, three arrays, plus
Data and Unit entries, a user AM and a ReturnAm) encoded by oracle/wire.py, applied with the AMs of one (array, op,
operands) aggregated into one record stream, replies decoded and checked: final states
against the oracle (order-insensitive ops), returned values against the linearizability
checker (order-dependent ops), and the launch count against the number of groups."""
import numpy as np
import pytest
import torch

from oracle import wire
from test_gpu_parity import to_dev

pytestmark = pytest.mark.gpu

U64, F64, U32 = 3, 9, 2


def _handle(inner):
    return dict(data=wire.net_darc(inner, 1, 0, 0), distribution=0, orig_elem_per_pe=1 << 20, orig_remaining_elems=0,
                elem_size=1, offset=0, size=1 << 20, sub=False, lock=wire.net_darc(inner + 1, 1, 0, 0), native_type=8)


def _le(vals, n):
    return b"".join(int(v).to_bytes(n, "little") for v in vals)


def test_batched_message_of_small_ams(world, orc):
    k = world.team().kernels
    rng = np.random.default_rng(2024)
    LA, LB, LC = 26000, 400, 2000
    a0 = rng.integers(0, 2**40, LA).astype(np.uint64)
    b0 = rng.integers(-100, 100, LB).astype(np.float64)
    c0 = rng.integers(0, 4, LC).astype(np.uint32)
    shards = {0xA000: (to_dev(a0), LA), 0xB000: (to_dev(b0), LB), 0xC000: (to_dev(c0), LC)}
    reg = {201: (wire.SHAPE_MVMI, wire.KIND_NATIVE, U64), 202: (wire.SHAPE_SVMI, wire.KIND_NATIVE, U64),
           203: (wire.SHAPE_MVSI, wire.KIND_GENERIC, F64), 204: (wire.SHAPE_MVMI, wire.KIND_GENERIC, F64),
           205: (wire.SHAPE_MVMI, wire.KIND_NATIVE, U32), 206: (wire.SHAPE_SVMI, wire.KIND_NATIVE, U32)}
    entries, meta = [], []          # meta[e] = (am_id, idx, vals) of entry e (None: Data / Unit)

    def am(am_id, inner, shape, eb, op, idx, vals, iw=4, cmp_bits=0, val_bits=0, index=0):
        kind = reg[am_id][1]
        if shape == wire.SHAPE_MVMI:
            recs = wire.idx_vals(iw, eb, idx, vals)
        elif shape == wire.SHAPE_SVMI:
            recs = _le(idx, iw)
        else:
            recs = _le(vals, eb)
        body = wire.am_body(shape, kind, eb, _handle(inner), op, recs, cmp_bits=cmp_bits, index_size=iw,
                            val_bits=val_bits, index=index)
        entries.append(("am", am_id, 0x77, len(entries), 0, body))
        meta.append((am_id, idx, vals))

    f64bits = lambda x: np.asarray(x, dtype=np.float64).view(np.uint64)
    adds = []
    for j in range(60):
        i = rng.integers(0, 25000, 50)
        v = rng.integers(0, 2**40, 50).astype(np.uint64)
        am(201, 0xA000, wire.SHAPE_MVMI, 8, 0, i, v)
        adds.append((i, v))
        if j == 10:
            entries.append(("data", 5, 1, b"\x00" * 8, b"x" * 40))
            meta.append(None)
    for j in range(60):
        am(202, 0xA000, wire.SHAPE_SVMI, 8, 1, rng.integers(25000, 25500, 40), None, val_bits=3)
    for j in range(10):
        vals = rng.integers(-8, 8, 20).astype(np.float64)
        am(203, 0xB000, wire.SHAPE_MVSI, 8, 0, None, f64bits(vals), index=int(rng.integers(0, 50)))
        meta[-1] = (203, meta[-1][2], vals)
    entries.append(("unit", 6, 2))
    meta.append(None)
    # a user AM and a ReturnAm among the op AMs (simple_batcher.rs:276-304): the resolver sizes
    # them (the runtime's deserializer would), the library steps over them and leaves them be
    entries.append(("am", 300, 0x77, 9000, 0, bytes(range(45))))
    meta.append(None)
    entries.append(("return_am", 301, 0x77, 9001, 0, bytes(19)))
    meta.append(None)
    for j in range(30):
        vals = rng.integers(-8, 8, 30).astype(np.float64)
        am(204, 0xB000, wire.SHAPE_MVMI, 8, 1, rng.integers(100, 300, 30), f64bits(vals))
        meta[-1] = (204, meta[-1][1], vals)
    for j in range(30):
        am(205, 0xC000, wire.SHAPE_MVMI, 4, 18, 2 * rng.integers(0, LC // 2, 25), rng.integers(0, 9, 25))
    for j in range(30):
        am(206, 0xC000, wire.SHAPE_SVMI, 4, 21, 2 * rng.integers(0, LC // 2, 25) + 1, None, cmp_bits=0, val_bits=7)
    msg = wire.message_batched(1, entries)

    def shard_of(v):
        t, n = shards[v.data.inner_addr]
        return t, n, 0
    k.profile(True)
    k.profile_read(reset=True)
    try:
        replies = k.apply_msg(msg, lambda am_id: {300: 45, 301: 19}.get(am_id, reg.get(am_id)), shard_of)
        stages = k.profile_read(reset=True)
    finally:
        k.profile(False)
    assert k.errors() == 0
    # aggregation: one apply per (array, op, operands, value) group, one per MVSI AM; groups
    # below 1000 records (204, 205, 206) take the ordered path (AUTO), the others direct atomics
    assert stages["direct"][1] == 2 and stages["ordered"][1] == 3, stages
    assert stages["mvsi"][1] == 10, stages
    A = shards[0xA000][0].cpu().numpy().view(np.uint64)
    B = shards[0xB000][0].cpu().numpy().view(np.float64)
    C = shards[0xC000][0].cpu().numpy().view(np.uint32)

    def gather(am_id, scalar=None):
        idx, vals, rets, oks = [], [], [], []
        for e, m in enumerate(meta):
            if m is None or m[0] != am_id:
                continue
            eb = 8 if reg[am_id][2] != U32 else 4
            rk = 2 if am_id == 206 else 1
            r, o = wire.decode_reply(eb, rk, replies[e]) if (e in replies) else (None, None)
            n = len(m[1]) if m[1] is not None else len(m[2])
            idx.append(np.asarray(m[1], dtype=np.uint64))
            vals.append(np.full(n, scalar) if scalar is not None else np.asarray(m[2]))
            if r is not None:
                assert len(r) == n
                rets.append(r)
            if o is not None:
                oks.append(o)
        cat = lambda x: np.concatenate(x) if x else None
        return cat(idx), cat(vals), cat(rets), cat(oks)

    # A[0:25000): adds (order-insensitive): exact
    ref = a0.copy()
    for i, v in adds:
        np.add.at(ref, i.astype(np.int64), v)
    assert np.array_equal(A[:25000], ref[:25000])
    # A[25000:25500): fetch_add(3) olds -> one serial order per element
    i, v, r, _ = gather(202, scalar=3)
    sl = slice(25000, 25500)
    st, bad = orc.check_linearizable(1, U64, np.uint64, 1, a0[sl], A[sl], i - 25000, v.astype(np.uint64), r)
    assert st == 0, bad
    # B MVSI blocks (small integers: exact in any order), B fetch_add olds
    refb = b0.copy()
    for e, m in enumerate(meta):
        if m is None or m[0] != 203:
            continue
        body_index = entries[e][5]
        index = int.from_bytes(body_index[-8:], "little")
        refb[index] += m[2].sum()
    assert np.array_equal(B[:100], refb[:100])
    i, v, r, _ = gather(204)
    st, bad = orc.check_linearizable(2, F64, np.float64, 1, b0[100:300], B[100:300], i - 100, v,
                                     r.view(np.float64))
    assert st == 0, bad
    # C: swaps on even elements, compare_exchange(current 0) -> 7 on odd ones
    i, v, r, _ = gather(205)
    ev = np.arange(0, LC, 2)
    st, bad = orc.check_linearizable(1, U32, np.uint32, 18, c0[ev], C[ev], i // 2, v.astype(np.uint32),
                                     r.astype(np.uint32))
    assert st == 0, bad
    i, v, r, o = gather(206, scalar=7)
    od = np.arange(1, LC, 2)
    st, bad = orc.check_linearizable(1, U32, np.uint32, 21, c0[od], C[od], (i - 1) // 2, v.astype(np.uint32),
                                     r.astype(np.uint32), o, current=np.uint32(0))
    assert st == 0, bad
    # replies exist exactly for the returning AMs
    ret_ids = {202, 204, 205, 206}
    assert set(replies) == {e for e, m in enumerate(meta) if m is not None and m[0] in ret_ids}
