"""AM wire format (include/lamellar_gpu_ops.h, "AM wire format"): the library's decoder,
encoder, message parser and reply encoder against the independent Python restatement in
oracle/wire.py. Host code only (no GPU). Wire-format parity is unpinned (no reference
fixture holds serialized bytes): these tests pin the library to the restated serde layout."""
import ctypes

import numpy as np
import pytest

from oracle import wire

DT = {"u8": (0, 1), "u16": (1, 2), "u32": (2, 4), "u64": (3, 8), "i8": (4, 1), "i16": (5, 2), "i32": (6, 4),
      "i64": (7, 8), "f32": (8, 4), "f64": (9, 8)}
LMR_E_INVALID, LMR_E_UNSUPPORTED, LMR_E_LENGTH = 1, 5, 8


def _handle(rng, kind):
    h = dict(data=wire.net_darc(int(rng.integers(1, 2**48)), 1, 3, 2), distribution=int(rng.integers(0, 2)),
             orig_elem_per_pe=int(rng.integers(1, 2**40)), orig_remaining_elems=int(rng.integers(0, 8)),
             elem_size=1, offset=int(rng.integers(0, 1000)), size=int(rng.integers(1, 2**40)),
             sub=bool(rng.integers(0, 2)), lock=wire.net_darc(int(rng.integers(1, 2**48)), 1, 3, 2),
             native_type=int(rng.integers(0, 10)))
    return h


def _recs(rng, shape, iw, eb, n):
    if shape == wire.SHAPE_MVMI:
        return wire.idx_vals(iw, eb, rng.integers(0, 2**(8 * iw - 1), n), rng.integers(0, 2**(8 * eb - 1), n))
    if shape == wire.SHAPE_SVMI:
        return b"".join(int(x).to_bytes(iw, "little") for x in rng.integers(0, 2**(8 * iw - 1), n))
    return b"".join(int(x).to_bytes(eb, "little") for x in rng.integers(0, 2**(8 * eb - 1), n))


def _view(capi, buf, shape, kind, code):
    from lamellar_runtime_amd import _capi
    v = _capi.lmr_am_view_t()
    raw = (ctypes.c_uint8 * max(len(buf), 1)).from_buffer_copy(buf if buf else b"\0")
    st = capi.lmr_am_decode(raw, len(buf), shape, kind, code, ctypes.byref(v))
    return st, v


def test_record_layout_matches_library(capi):
    for iw in (1, 2, 4, 8):
        for name, (code, eb) in DT.items():
            assert (capi.lmr_record_bytes(iw, code), capi.lmr_record_val_offset(iw, code)) == \
                wire.record_layout(iw, eb), (iw, name)


@pytest.mark.parametrize("shape", [wire.SHAPE_MVMI, wire.SHAPE_SVMI, wire.SHAPE_MVSI], ids=["mvmi", "svmi", "mvsi"])
@pytest.mark.parametrize("kind", range(6), ids=["unsafe", "native", "generic", "locallock", "globallock", "readonly"])
def test_am_decode_encode_roundtrip(capi, shape, kind):
    rng = np.random.default_rng(11 + 7 * shape + kind)
    for name, (code, eb) in DT.items():
        for op in (0, 1, 18, 21, 22, 26):
            h = _handle(rng, kind)
            iw = int(rng.choice([1, 2, 4, 8]))
            n = int(rng.integers(0, 40))
            recs = _recs(rng, shape, iw, eb, n)
            cmp_bits, eps_bits = int(rng.integers(0, 2**(8 * eb - 1))), int(rng.integers(0, 2**(8 * eb - 1)))
            val_bits, index = int(rng.integers(0, 2**(8 * eb - 1))), int(rng.integers(0, 2**40))
            body = wire.am_body(shape, kind, eb, h, op, recs, cmp_bits, eps_bits, iw, val_bits, index)
            st, v = _view(capi, body + b"trailing", shape, kind, code)
            assert st == 0, (name, op, st)
            assert v.body_bytes == len(body)
            assert (v.op, v.shape, v.kind, v.dtype) == (op, shape, kind, code)
            assert v.data.inner_addr == int.from_bytes(h["data"][:8], "little") and v.data.orig_world_pe == 3
            assert (v.distribution, v.orig_elem_per_pe, v.orig_remaining_elems, v.offset, v.size, v.sub) == \
                (h["distribution"], h["orig_elem_per_pe"], h["orig_remaining_elems"], h["offset"], h["size"],
                 int(h["sub"]))
            if kind in (wire.KIND_GENERIC, wire.KIND_LOCAL_LOCK, wire.KIND_GLOBAL_LOCK):
                assert v.lock.inner_addr == int.from_bytes(h["lock"][:8], "little")
            assert v.native_type == (h["native_type"] if kind == wire.KIND_NATIVE else 0xFFFFFFFF)
            assert v.cmp_bits == (cmp_bits if op in (21, 22) else 0)
            assert v.eps_bits == (eps_bits if op == 22 else 0)
            assert bytes(body[v.recs_offset:v.recs_offset + v.recs_bytes]) == recs
            if shape == wire.SHAPE_MVSI:
                assert v.index == index
            else:
                assert v.index_size == iw
            if shape == wire.SHAPE_SVMI:
                assert v.val_bits == val_bits
            # the encoder reproduces the bytes
            out = (ctypes.c_uint8 * (len(body) + 16))()
            wr = ctypes.c_uint64()
            rb = (ctypes.c_uint8 * max(len(recs), 1)).from_buffer_copy(recs if recs else b"\0")
            assert capi.lmr_am_encode(ctypes.byref(v), rb, out, len(out), ctypes.byref(wr)) == 0
            assert wr.value == len(body) and bytes(out)[:len(body)] == body
            # too small an output: LENGTH with the needed size
            assert capi.lmr_am_encode(ctypes.byref(v), rb, out, 3, ctypes.byref(wr)) == LMR_E_LENGTH
            assert wr.value == len(body)
            # truncated body
            st, _ = _view(capi, body[:-1], shape, kind, code)
            assert st == LMR_E_LENGTH


def test_am_decode_rejects_bad_fields(capi):
    h = _handle(np.random.default_rng(1), wire.KIND_NATIVE)
    body = wire.am_body(wire.SHAPE_MVMI, wire.KIND_NATIVE, 8, h, 40, b"", index_size=4)
    assert _view(capi, body, wire.SHAPE_MVMI, wire.KIND_NATIVE, 3)[0] == LMR_E_INVALID     # op tag
    body = wire.am_body(wire.SHAPE_MVMI, wire.KIND_NATIVE, 8, h, 0, b"", index_size=3)
    st, v = _view(capi, body, wire.SHAPE_MVMI, wire.KIND_NATIVE, 3)                       # index width 3:
    assert st == 0 and v.index_size == 8                                                  # usize (`_ =>`)
    assert _view(capi, body, 3, wire.KIND_NATIVE, 3)[0] == LMR_E_INVALID                   # shape
    assert _view(capi, body, 0, 6, 3)[0] == LMR_E_INVALID                                  # kind


REG = {101: (wire.SHAPE_MVMI, wire.KIND_NATIVE, 3), 102: (wire.SHAPE_SVMI, wire.KIND_GENERIC, 9),
       103: (wire.SHAPE_MVSI, wire.KIND_LOCAL_LOCK, 2)}


USER = {}          # am_id -> serialized body size of a non-op AM (the runtime's deserializer knows it)


def _resolver():
    from lamellar_runtime_amd import _capi

    def res(_user, _cmd, am_id, _body, _avail, shape, kind, dtype, body_bytes):
        if am_id in USER:
            body_bytes[0] = USER[am_id]
            return 1
        if am_id not in REG:
            return 2
        shape[0], kind[0], dtype[0] = REG[am_id]
        return 0
    return _capi.AM_RESOLVER_FN(res)


def _parse(capi, msg, cap=64):
    from lamellar_runtime_amd import _capi
    res = _resolver()
    ents = (_capi.lmr_msg_entry_t * cap)()
    n = ctypes.c_uint32()
    raw = (ctypes.c_uint8 * len(msg)).from_buffer_copy(msg)
    st = capi.lmr_msg_parse(raw, len(msg), res, None, ents, cap, ctypes.byref(n))
    return st, [ents[i] for i in range(min(n.value, cap))], n.value


def _bodies(rng):
    out = []
    for am_id, (shape, kind, code) in REG.items():
        eb = [e for c, e in DT.values() if c == code][0]
        recs = _recs(rng, shape, 4, eb, int(rng.integers(1, 30)))
        out.append((am_id, wire.am_body(shape, kind, eb, _handle(rng, kind), 1, recs, index_size=4,
                                        val_bits=5, index=77)))
    return out


def test_msg_parse_single_am(capi):
    rng = np.random.default_rng(5)
    am_id, body = _bodies(rng)[0]
    msg = wire.message_single(6, am_id, 0xABC, 42, 7, body)
    st, ents, n = _parse(capi, msg)
    assert st == 0 and n == 1
    e = ents[0]
    assert (e.cmd, e.src, e.am_id, e.team_addr, e.req_id, e.req_sub_id) == (0, 6, am_id, 0xABC, 42, 7)
    assert (e.shape, e.kind, e.dtype) == REG[am_id]
    assert e.body_offset == 7 + 28 and e.body_bytes == len(body)


def test_msg_parse_batched_with_data_and_unit(capi):
    rng = np.random.default_rng(6)
    bodies = _bodies(rng)
    entries = []
    for j in range(5):
        am_id, body = bodies[j % len(bodies)]
        entries.append(("am", am_id, 0x10 + j, 100 + j, j, body))
        if j == 1:
            entries.append(("data", 9, 1, b"\x01" * 12, b"payload!" * 3))
        if j == 3:
            entries.append(("unit", 11, 2))
    msg = wire.message_batched(3, entries)
    st, ents, n = _parse(capi, msg)
    assert st == 0 and n == len(entries)
    off = 7
    for e, spec in zip(ents, entries):
        off += 4
        if spec[0] == "am":
            assert (e.cmd, e.am_id, e.team_addr, e.req_id, e.req_sub_id) == (0,) + spec[1:5]
            assert e.body_offset == off + 28 and e.body_bytes == len(spec[5])
            off += 28 + len(spec[5])
        elif spec[0] == "data":
            assert (e.cmd, e.req_id, e.req_sub_id) == (2, 9, 1)
            assert bytes(msg[e.body_offset:e.body_offset + e.body_bytes]) == spec[4]
            off += 32 + len(spec[3]) + len(spec[4])
        else:
            assert (e.cmd, e.req_id, e.req_sub_id) == (3, 11, 2)
            off += 16
    assert off == len(msg)
    # too small an entry array: LENGTH, the count still reported
    st, _, n2 = _parse(capi, msg, cap=2)
    assert st == LMR_E_LENGTH and n2 == len(entries)


def test_msg_parse_user_and_return_ams(capi):
    """A batched message as the SimpleBatcher builds it (simple_batcher.rs:276-304): op AMs
    mixed with user AMs and ReturnAms (sized by the resolver, reported as LMR_SHAPE_FOREIGN),
    Data and Unit entries; every entry parsed in order."""
    rng = np.random.default_rng(8)
    bodies = _bodies(rng)
    USER.clear()
    USER.update({500: 37, 501: 0, 502: 200})
    entries = [("am", bodies[0][0], 1, 10, 0, bodies[0][1]),
               ("am", 500, 2, 11, 0, bytes(rng.integers(0, 256, 37, dtype=np.uint8))),
               ("return_am", 502, 3, 12, 1, bytes(200)),
               ("unit", 13, 0),
               ("am", 501, 4, 14, 0, b""),
               ("am", bodies[1][0], 5, 15, 0, bodies[1][1]),
               ("data", 16, 2, b"", b"zz")]
    msg = wire.message_batched(4, entries)
    try:
        st, ents, n = _parse(capi, msg)
    finally:
        USER.clear()
    assert st == 0 and n == len(entries)
    assert [e.cmd for e in ents] == [0, 0, 1, 3, 0, 0, 2]
    assert [e.shape for e in ents[:3]] == [REG[bodies[0][0]][0], 3, 3] and ents[4].shape == 3
    assert (ents[1].am_id, ents[1].body_bytes, ents[2].am_id, ents[2].body_bytes) == (500, 37, 502, 200)
    assert bytes(msg[ents[1].body_offset:ents[1].body_offset + 37]) == entries[1][5]
    assert ents[5].body_bytes == len(bodies[1][1]) and ents[5].shape == REG[bodies[1][0]][0]
    # a foreign AM claiming more bytes than the message holds
    USER[500] = 10 ** 6
    try:
        assert _parse(capi, msg)[0] == LMR_E_LENGTH
    finally:
        USER.clear()


def test_msg_parse_errors(capi):
    rng = np.random.default_rng(7)
    am_id, body = _bodies(rng)[0]
    # a return AM the resolver does not size / an unknown AM: its size is unknown here
    msg = wire.message_batched(0, [("return_am", am_id, 1, 2, 3, body)])
    assert _parse(capi, msg)[0] == LMR_E_UNSUPPORTED
    assert _parse(capi, wire.message_single(0, 999, 1, 2, 3, body))[0] == LMR_E_UNSUPPORTED
    # nested batch, missing header, truncation
    bad = wire.ser_header(0, wire.CMD_BATCHED) + (4).to_bytes(4, "little")
    assert _parse(capi, bad)[0] == LMR_E_INVALID
    assert _parse(capi, b"\x00" + wire.message_single(0, am_id, 1, 2, 3, body)[1:])[0] == LMR_E_INVALID
    assert _parse(capi, wire.message_single(0, am_id, 1, 2, 3, body)[:-1])[0] == LMR_E_LENGTH


@pytest.mark.parametrize("name", ["u8", "i16", "u32", "f32", "u64", "f64"])
def test_reply_encode(capi, name):
    code, eb = DT[name]
    rng = np.random.default_rng(code)
    n = 37
    bits = rng.integers(0, 2**(8 * eb - 1), n).astype(np.uint64)
    res = np.frombuffer(b"".join(int(b).to_bytes(eb, "little") for b in bits), dtype=np.uint8).copy()
    oks = rng.integers(0, 2, n).astype(np.uint8)
    for rk in (1, 2):
        nb = capi.lmr_reply_bytes(code, rk, n)
        assert nb == 8 + n * (eb if rk == 1 else 4 + eb)
        out = np.zeros(nb, dtype=np.uint8)
        assert capi.lmr_reply_encode(code, rk, n, res.ctypes.data, oks.ctypes.data, out.ctypes.data, nb) == 0
        v, o = wire.decode_reply(eb, rk, out.tobytes())
        assert np.array_equal(v, bits)
        if rk == 2:
            assert np.array_equal(o, oks)
        assert capi.lmr_reply_encode(code, rk, n, res.ctypes.data, oks.ctypes.data, out.ctypes.data, nb - 1) == \
            LMR_E_LENGTH
    assert capi.lmr_reply_bytes(code, 0, n) == 0
