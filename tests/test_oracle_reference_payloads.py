"""Pin the CPU oracle on the rest of the reference's test payloads (tests/payloads.py).

Restated over 1-4 simulated PEs (each PE's requests applied as that PE's batch, the PEs
in turn), Block and Cyclic, the payloads' lengths 4 / 19 / 128 and every element type
each payload instantiates (usize = u64, isize = i64; 128-bit types are out of scope):
  arithmetic_ops/{fetch_sub,fetch_mul,fetch_div,rem,fetch_rem}_test.rs,
  bitwise_ops/{fetch_and,fetch_or}_test.rs, atomic_ops/load_store_test.rs,
  atomic_ops/compare_exchange_test.rs (epsilon half :235-412 and input variant :448-470),
  and the OpInput `input` variants of add_test.rs:326-505 and fetch_add_test.rs:371-560.
"""
import numpy as np
import pytest

import payloads as P
from simworld import SimArray

PES = [1, 2, 3, 4]
LENS = [4, 19, 128]
DISTS = [0, 1]


class _SimArr:
    def __init__(self, s):
        self.s = s

    def fill(self, v):
        self.s.fill(v)

    def set(self, vals):
        for i, v in enumerate(vals):
            pe, off = self.s.orc.pe_and_offset(self.s.L, i)
            self.s.slices()[pe][off] = v

    def op(self, op, idx, vals, current=None, eps=None, pe=0):
        st, res, ok = self.s.op(op, np.asarray(idx, dtype=np.uint64), vals, current, eps)
        assert st == 0, (op, st)
        return res, ok

    def op_mvsi(self, op, index, vals, pe=0):
        return self.op(op, [index], vals, pe=pe)

    def to_numpy(self):
        return self.s.to_numpy()

    def sub_array(self, lo, hi):
        return _SimArr(self.s.sub_array(lo, hi))

    def len(self):
        return self.s.len()


class SimWorld:
    def __init__(self, orc, npes):
        self.orc, self.npes = orc, npes

    def array(self, kind, length, dist, dt):
        return _SimArr(SimArray(self.orc, self.npes, length, dist, dt, kind))


KINDS = ["AtomicArray", "LocalLockArray", "UnsafeArray"]


@pytest.mark.parametrize("dist", DISTS, ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", P.ALL_TYPES)
def test_fetch_sub_payload(orc, dt, npes, dist):
    for kind in KINDS:
        for n in LENS:
            P.fetch_sub_payload(SimWorld(orc, npes), kind, dt, n, dist, np.random.default_rng(n + npes))


@pytest.mark.parametrize("dist", DISTS, ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", P.ALL_TYPES)
def test_fetch_mul_div_payloads(orc, dt, npes, dist):
    for kind in KINDS:
        for n in LENS:
            P.fetch_mul_div_payload(SimWorld(orc, npes), kind, dt, n, dist)


@pytest.mark.parametrize("dist", DISTS, ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", P.ALL_TYPES)
def test_rem_payloads(orc, dt, npes, dist):
    for kind in KINDS:
        for n in LENS:
            P.rem_payload(SimWorld(orc, npes), kind, dt, n, dist)


@pytest.mark.parametrize("dist", DISTS, ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", P.INT_TYPES)
def test_fetch_and_or_payloads(orc, dt, npes, dist):
    for kind in KINDS:
        for n in LENS:
            P.fetch_and_or_payload(SimWorld(orc, npes), kind, dt, n, dist)


@pytest.mark.parametrize("dist", DISTS, ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", P.ALL_TYPES)
def test_load_store_payload(orc, dt, npes, dist):
    for kind in KINDS:
        for n in LENS:
            P.load_store_payload(SimWorld(orc, npes), kind, dt, n, dist)


@pytest.mark.parametrize("dist", DISTS, ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", ["f32", "f64"])
def test_compare_exchange_epsilon_payload(orc, dt, npes, dist):
    for kind in ["AtomicArray", "LocalLockArray"]:
        for n in LENS:
            P.cas_epsilon_payload(SimWorld(orc, npes), kind, dt, n, dist)


@pytest.mark.parametrize("dist", DISTS, ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
def test_compare_exchange_input_payload(orc, npes, dist):
    for kind in ["AtomicArray", "LocalLockArray"]:
        for n in (4, 100, 2000):
            P.cas_input_payload(SimWorld(orc, npes), kind, n, dist)


@pytest.mark.parametrize("dist", DISTS, ids=["Block", "Cyclic"])
@pytest.mark.parametrize("npes", PES)
def test_add_and_fetch_add_input_payloads(orc, npes, dist):
    """tests/add.rs:89-112 and fetch_add.rs:93-115 run the input variants at len 4, 100,
    2000 (the reference's `input` matrix); the local-data container is an UnsafeArray of
    len * num_pes whose local data is 0..len on every PE."""
    cont = P.index_containers(lambda n, pe: [np.arange(n, dtype=np.uint64)])
    for kind in ["AtomicArray", "LocalLockArray", "UnsafeArray"]:
        for n in (4, 100, 2000):
            P.add_input_payload(SimWorld(orc, npes), kind, n, dist, cont)
            P.fetch_add_input_payload(SimWorld(orc, npes), kind, n, dist, cont)


@pytest.mark.parametrize("npes", PES)
@pytest.mark.parametrize("dt", ["u8", "f64"])
def test_array_ops_example_payload(orc, dt, npes):
    """examples/array_examples/array_ops.rs (u8 and f64 halves, incl. shl / shr)."""
    P.array_ops_example_payload(SimWorld(orc, npes), dt)
