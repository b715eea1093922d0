"""CPU ORACLE FOR TESTS ONLY: the reference's op-AM wire format, restated in Python.

An independent encoder/decoder (struct module) of what the running Rust runtime puts in
a lamellae buffer for the batched element ops, used by tests/ to check the library's
lmr_am_decode / lmr_am_encode / lmr_msg_parse / lmr_reply_encode / lmr_apply_msg.

Serialization: bincode 2 legacy config (src/lib.rs:319-321): little endian, fixed-width
integers, usize as u64, enum variants as u32, Option as a u8 tag, byte vectors
(serde_bytes) and Vec<T> as a u64 length + contents.

* message   = Option<SerializeHeader{msg: Msg{src: u16, cmd: Cmd}}>  (src/lamellae.rs:33-34,
              102-104; src/active_messaging.rs:893-908) + data
* Cmd::Am   : AmHeader{am_id: i32, team_addr: usize, req_id: ReqId{id, sub_id}}
              (registered_active_message.rs:80-85, 278-300; scheduler.rs:72-75) + AM struct
* batched   : [Cmd][AmHeader][AM] | [Cmd::Data][DataHeader{size, req_id, darc_list_size}]
              [darcs][data] | [Cmd::Unit][UnitHeader{req_id}]  (simple_batcher.rs:400-481)
* AM struct : data, op: ArrayOpCmd<T>, then MVMI idx_vals: bytes, index_size: u8 |
              SVMI val: T, indices: bytes, index_size: u8 | MVSI vals: bytes, index: usize
              (impl/src/array_ops.rs:855-861, 920-927, 991-997)
* data      : UnsafeArrayInner{data: Darc, distribution, orig_elem_per_pe,
              orig_remaining_elems, elem_size, offset, size, sub: bool} (unsafe.rs:106-116);
              NativeAtomicArray appends orig_t: NativeAtomicType (native_atomic.rs:819-822);
              GenericAtomic / LocalLock / GlobalLock prepend their lock Darc
              (generic_atomic.rs:272-275, local_lock_atomic.rs:50-53, global_lock_atomic.rs:43-46)
* Darc      : __NetworkDarc{inner_addr: usize, backend: Backend, orig_world_pe: usize,
              orig_team_pe: usize} (darc.rs:227-234, 1838-1843)
* IdxVal<I,T> is #[repr(C)] (operations.rs:213-230): value at round_up(|I|, |T|), record
  padded to a multiple of max(|I|, |T|).

Parity unpinned: no reference test or fixture holds serialized bytes; this
restates the serde derives, it is not checked against bytes the reference produced.
"""
import struct

import numpy as np

CMD_AM, CMD_RETURN_AM, CMD_DATA, CMD_UNIT, CMD_BATCHED = 0, 1, 2, 3, 4
SHAPE_MVMI, SHAPE_SVMI, SHAPE_MVSI = 0, 1, 2
KIND_UNSAFE, KIND_NATIVE, KIND_GENERIC, KIND_LOCAL_LOCK, KIND_GLOBAL_LOCK, KIND_READ_ONLY = range(6)
OP_CAS, OP_CAS_EPS = 21, 22


def _u(v, n):
    return int(v).to_bytes(n, "little", signed=False)


def net_darc(inner_addr, backend=1, world_pe=0, team_pe=0):
    return _u(inner_addr, 8) + _u(backend, 4) + _u(world_pe, 8) + _u(team_pe, 8)


def array_handle(kind, h):
    """h: dict with data (darc bytes), distribution, orig_elem_per_pe, orig_remaining_elems,
    elem_size, offset, size, sub, [lock (darc bytes)], [native_type]."""
    unsafe = (h["data"] + _u(h["distribution"], 4) + _u(h["orig_elem_per_pe"], 8) +
              _u(h["orig_remaining_elems"], 8) + _u(h["elem_size"], 8) + _u(h["offset"], 8) +
              _u(h["size"], 8) + _u(1 if h["sub"] else 0, 1))
    if kind in (KIND_GENERIC, KIND_LOCAL_LOCK, KIND_GLOBAL_LOCK):
        return h["lock"] + unsafe
    if kind == KIND_NATIVE:
        return unsafe + _u(h["native_type"], 4)
    return unsafe


def op_cmd(op, eb, cmp_bits=0, eps_bits=0):
    b = _u(op, 4)
    if op == OP_CAS:
        b += _u(cmp_bits, eb)
    elif op == OP_CAS_EPS:
        b += _u(cmp_bits, eb) + _u(eps_bits, eb)
    return b


def record_layout(iw, eb):
    vo = -(-iw // eb) * eb
    a = max(iw, eb)
    return -(-(vo + eb) // a) * a, vo


def idx_vals(iw, eb, idx, val_bits):
    """IdxVal<I,T> records (padding bytes zero) from integer indices and value bits."""
    rb, vo = record_layout(iw, eb)
    out = bytearray(rb * len(idx))
    for k, (i, v) in enumerate(zip(idx, val_bits)):
        out[k * rb:k * rb + iw] = _u(i, iw)
        out[k * rb + vo:k * rb + vo + eb] = _u(v, eb)
    return bytes(out)


def am_body(shape, kind, eb, handle, op, recs, cmp_bits=0, eps_bits=0, index_size=4, val_bits=0, index=0):
    b = array_handle(kind, handle) + op_cmd(op, eb, cmp_bits, eps_bits)
    if shape == SHAPE_SVMI:
        b += _u(val_bits, eb)
    b += _u(len(recs), 8) + bytes(recs)
    if shape == SHAPE_MVSI:
        b += _u(index, 8)
    else:
        b += _u(index_size, 1)
    return b


def am_header(am_id, team_addr, req_id, sub_id):
    return struct.pack("<i", am_id) + _u(team_addr, 8) + _u(req_id, 8) + _u(sub_id, 8)


def ser_header(src, cmd):
    return b"\x01" + _u(src, 2) + _u(cmd, 4)


def message_single(src, am_id, team_addr, req_id, sub_id, body):
    return ser_header(src, CMD_AM) + am_header(am_id, team_addr, req_id, sub_id) + body


def message_batched(src, entries):
    """entries: ("am", am_id, team_addr, req_id, sub_id, body) | ("data", req_id, sub_id, darcs,
    data) | ("unit", req_id, sub_id) | ("return_am", am_id, team_addr, req_id, sub_id, body)."""
    out = ser_header(src, CMD_BATCHED)
    for e in entries:
        if e[0] in ("am", "return_am"):
            out += _u(CMD_AM if e[0] == "am" else CMD_RETURN_AM, 4) + am_header(*e[1:5]) + e[5]
        elif e[0] == "data":
            _, req, sub, darcs, data = e
            out += _u(CMD_DATA, 4) + _u(len(data), 8) + _u(req, 8) + _u(sub, 8) + _u(len(darcs), 8) + darcs + data
        else:
            out += _u(CMD_UNIT, 4) + _u(e[1], 8) + _u(e[2], 8)
    return out


def decode_reply(eb, ret_kind, buf):
    """Vec<T> (ret_kind 1) -> value bits; Vec<Result<T,T>> (2) -> (value bits, ok flags)."""
    n = int.from_bytes(buf[:8], "little")
    if ret_kind == 1:
        vals = [int.from_bytes(buf[8 + k * eb:8 + (k + 1) * eb], "little") for k in range(n)]
        return np.array(vals, dtype=np.uint64), None
    vals, oks = [], []
    for k in range(n):
        o = 8 + k * (4 + eb)
        tag = int.from_bytes(buf[o:o + 4], "little")
        oks.append(1 if tag == 0 else 0)
        vals.append(int.from_bytes(buf[o + 4:o + 4 + eb], "little"))
    return np.array(vals, dtype=np.uint64), np.array(oks, dtype=np.uint8)
