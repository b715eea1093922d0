"""The reference's own test programs, restated on the device path (one PE).

Each test follows one of the reference's integration-test payloads
(tests/array/**, run by tests/<op>.rs through lamellar_run.sh) through the
host-side op-builder API (array.py) -> engine -> C ABI -> gfx950 kernels, and
checks the payload's known answer. The reference issues most of these as
per-element calls (`array.add(idx, 1)` in a loop); the batched forms it also
tests (`batch_add(indices, 1)`, add_test.rs:131-160) are used here, plus the
per-element form on the shortest length. Matrix as in SURVEY.md §4: Unsafe /
Atomic / LocalLock arrays, Block / Cyclic, lengths 4, 19, 128; C1 (1,000,000
u64 elements, add_test's pattern) on top.
"""
import numpy as np
import pytest

from opgen import NP

pytestmark = pytest.mark.gpu

KINDS = ["UnsafeArray", "AtomicArray", "LocalLockArray"]
DTS = ["u8", "u16", "u32", "u64", "i8", "i16", "i32", "i64", "f32", "f64"]
LENS = [4, 19, 128]


def max_updates(dt, num_pes=1):
    """mul_test.rs:59-75: floor(log2(T::MAX / num_pes)) / num_pes (floats saturate the u128 cast)."""
    if dt.startswith("f"):
        mx = (1 << 128) - 1
    else:
        mx = int(np.iinfo(NP[dt]).max)
    return ((mx // num_pes).bit_length() - 1) // num_pes


def new(lam, world, kind, n, dist, dt):
    return getattr(lam, kind)(world.team(), n, dist, dt)


def host(arr, dt):
    return arr.to_numpy().astype(NP[dt])


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("kind", KINDS)
def test_reference_arithmetic_programs(world, lam, kind, dt):
    """add_test.rs:88-160 (each element += 1, pe_max_val times: 50, 9 for f32), sub_test.rs:96-118
    (100 - 100 x 1 = 0), mul_test.rs:99-117 (1 x 2^max_updates), div_test.rs:91-110 (back to 1)."""
    t = NP[dt]
    pe_max_val = 9 if dt == "f32" else 50
    mu = max_updates(dt)
    for dist in (lam.Distribution.Block, lam.Distribution.Cyclic):
        for n in LENS:
            a = new(lam, world, kind, n, dist, dt)
            idx = np.tile(np.arange(n, dtype=np.uint64), pe_max_val)
            np.random.default_rng(n).shuffle(idx)
            if n == 4:                                       # per-element form, as the payload issues it
                for i in range(n):
                    for _ in range(pe_max_val):
                        a.add(i, 1).spawn()
                a.wait_all()
            else:
                a.batch_add(idx, 1).block()
            assert np.all(host(a, dt) == t(pe_max_val)), (kind, dt, dist, n, "add")
            a.fill(100)
            a.wait_all()
            a.batch_sub(np.tile(np.arange(n, dtype=np.uint64), 100), np.ones(100 * n, dtype=t)).block()
            assert np.all(host(a, dt) == t(0)), (kind, dt, dist, n, "sub")
            a.fill(1)
            a.wait_all()
            a.batch_mul(np.tile(np.arange(n, dtype=np.uint64), mu), 2).block()
            exp = t(2.0 ** mu) if dt.startswith("f") else t(1 << mu)
            assert np.all(host(a, dt) == exp), (kind, dt, dist, n, "mul")
            a.batch_div(np.tile(np.arange(n, dtype=np.uint64), mu), 2).block()
            assert np.all(host(a, dt) == t(1)), (kind, dt, dist, n, "div")


@pytest.mark.parametrize("dt", [d for d in DTS if not d.startswith("f")])
@pytest.mark.parametrize("kind", KINDS)
def test_reference_bitwise_programs(world, lam, kind, dt):
    """xor_test.rs:78-98 / or_test.rs: PE p sets bit p -> !(!0 << num_pes) = 1;
    and_test.rs:80-100: init !0, PE p clears bit p -> !0 << num_pes;
    fetch_xor_test.rs:85-98: the returned old never already holds the caller's bit."""
    t = NP[dt]
    ones = t(~t(0))
    for dist in (lam.Distribution.Block, lam.Distribution.Cyclic):
        for n in LENS:
            a = new(lam, world, kind, n, dist, dt)
            idx = np.arange(n, dtype=np.uint64)
            a.batch_bit_xor(idx, 1).block()
            assert np.all(host(a, dt) == t(1)), (kind, dt, n, "xor")
            a.fill(0)
            a.wait_all()
            a.batch_bit_or(idx, 1).block()
            assert np.all(host(a, dt) == t(1)), (kind, dt, n, "or")
            a.fill(ones)
            a.wait_all()
            a.batch_bit_and(idx, t(~t(1))).block()
            assert np.all(host(a, dt) == t(ones << t(1))), (kind, dt, n, "and")
            a.fill(0)
            a.wait_all()
            olds = a.batch_fetch_bit_xor(idx, 1).block().cpu().numpy().view(t)
            assert np.all((olds & t(1)) == 0), (kind, dt, n, "fetch_xor")


@pytest.mark.parametrize("dt", ["u8", "u32", "u64", "i16", "i64", "f32", "f64"])
@pytest.mark.parametrize("kind", KINDS)
def test_reference_fetch_add_program(world, lam, kind, dt):
    """fetch_add_test.rs:134-149: 10 fetch_add(idx, 1) per element; the 10 olds one PE gets
    for one index are distinct (here exactly 0..9), and every element ends at 10."""
    t = NP[dt]
    for dist in (lam.Distribution.Block, lam.Distribution.Cyclic):
        for n in LENS:
            a = new(lam, world, kind, n, dist, dt)
            idx = np.tile(np.arange(n, dtype=np.uint64), 10)
            olds = a.batch_fetch_add(idx, 1).block().cpu().numpy().view(t)
            for i in range(n):
                got = np.sort(olds[idx == i].astype(np.float64))
                assert np.array_equal(got, np.arange(10, dtype=np.float64)), (kind, dt, n, i)
            assert np.all(host(a, dt) == t(10))


@pytest.mark.parametrize("dt", ["u8", "u16", "u32", "u64", "i32", "i64", "f32", "f64"])
@pytest.mark.parametrize("kind", KINDS)
def test_reference_swap_and_compare_exchange_programs(world, lam, kind, dt):
    """swap_test.rs:70-106: init num_pes; PE p swaps p into its indices (idx % num_pes == p) and
    gets init back; every load then reads idx % num_pes. compare_exchange_test.rs:70-116: the
    first round on owned indices succeeds returning the init value, the second round fails
    (compare_exchange_epsilon for floats, compare_exchange.rs:291-348)."""
    t = NP[dt]
    for dist in (lam.Distribution.Block, lam.Distribution.Cyclic):
        for n in LENS:
            a = new(lam, world, kind, n, dist, dt)
            idx = np.arange(n, dtype=np.uint64)
            a.fill(1)
            a.wait_all()
            olds = a.batch_swap(idx, 0).block().cpu().numpy().view(t)
            assert np.all(olds == t(1)), (kind, dt, n, "swap olds")
            loads = a.batch_load(idx).block().cpu().numpy().view(t)
            assert np.all(loads == t(0)), (kind, dt, n, "load")
            if dt.startswith("f"):
                r1 = a.batch_compare_exchange_epsilon(idx, 0, 5, 0.5).block()
                r2 = a.batch_compare_exchange_epsilon(idx, 0, 7, 0.5).block()
            else:
                r1 = a.batch_compare_exchange(idx, 0, 5).block()
                r2 = a.batch_compare_exchange(idx, 0, 7).block()
            v1, ok1 = r1.numpy()
            v2, ok2 = r2.numpy()
            assert np.all(ok1) and np.all(v1 == t(0)), (kind, dt, n, "cas round 1")
            assert not np.any(ok2) and np.all(v2 == t(5)), (kind, dt, n, "cas round 2")
            assert np.all(host(a, dt) == t(5))


def test_reference_add_program_c1(world, lam):
    """C1 (BASELINE.json configs[0]): add_test's pattern on a 1,000,000-element AtomicArray<u64>,
    1 PE: every element receives pe_max_val = 50 adds of 10^(2*0) = 1 (5 x 10^7 records in one
    shuffled batch, add_test.rs:131-160), then the per-PE sub-array form (:166-290)."""
    n = 1_000_000
    a = lam.AtomicArray(world.team(), n, lam.Distribution.Block, "u64")
    idx = np.tile(np.arange(n, dtype=np.uint64), 50)
    np.random.default_rng(1).shuffle(idx)
    a.batch_add(idx, 1).block()
    got = a.to_numpy()
    assert np.all(got == 50)
    assert a.sum().block() == 50 * n
    s = a.sub_array(n // 4, n // 4 + n // 2)
    s.batch_add(np.tile(np.arange(s.len(), dtype=np.uint64), 50), 1).block()
    got = a.to_numpy()
    assert np.all(got[n // 4:n // 4 + n // 2] == 100) and np.all(got[:n // 4] == 50) and np.all(got[n // 4 + n // 2:] == 50)


# ---------------------------------------------------------------- the remaining payloads
# tests/payloads.py restates fetch_sub / fetch_mul / fetch_div / rem / fetch_rem /
# fetch_and / fetch_or / load_store / compare_exchange_epsilon and the OpInput `input`
# variants once; the CPU oracle runs them over 1-4 simulated PEs
# (tests/test_oracle_reference_payloads.py), the device runs them here at 1 PE through
# the op-builder API.
import payloads as P  # noqa: E402
import torch  # noqa: E402

from opgen import (ADD, AND, CAS, CAS_EPS, DIV, FETCH_ADD, FETCH_AND, FETCH_DIV, FETCH_MUL,  # noqa: E402
                   FETCH_OR, FETCH_REM, FETCH_SHL, FETCH_SHR, FETCH_SUB, FETCH_XOR, LOAD, MUL, OR, REM,
                   SHL, SHR, STORE, SUB, XOR)

_METHOD = {ADD: "batch_add", FETCH_ADD: "batch_fetch_add", FETCH_SUB: "batch_fetch_sub",
           FETCH_MUL: "batch_fetch_mul", FETCH_DIV: "batch_fetch_div", REM: "batch_rem",
           FETCH_REM: "batch_fetch_rem", FETCH_AND: "batch_fetch_bit_and", FETCH_OR: "batch_fetch_bit_or",
           STORE: "batch_store", SUB: "batch_sub", MUL: "batch_mul", DIV: "batch_div", AND: "batch_bit_and",
           OR: "batch_bit_or", XOR: "batch_bit_xor", FETCH_XOR: "batch_fetch_bit_xor", SHL: "batch_shl",
           FETCH_SHL: "batch_fetch_shl", SHR: "batch_shr", FETCH_SHR: "batch_fetch_shr"}


class _DevArr:
    def __init__(self, a, dt):
        self.a, self.dt = a, dt

    def fill(self, v):
        self.a.fill(v)
        self.a.wait_all()

    def set(self, vals):
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(vals).astype(NP[self.dt])).view(np.int64)
                             if NP[self.dt](0).itemsize == 8 else np.asarray(vals).astype(NP[self.dt]))
        self.a.local_data().copy_(t.to(self.a.local_data().device).view(self.a.local_data().dtype))

    def _res(self, h):
        r = h.block()
        if r is None:
            return None, None
        if isinstance(r, torch.Tensor):
            return r.cpu().numpy().view(NP[self.dt]), None
        v, ok = r.numpy()
        return v, ok.astype(np.uint8)

    def op(self, op, idx, vals, current=None, eps=None, pe=0):
        a = self.a
        if op == LOAD:
            return self._res(a.batch_load(idx))
        if op == CAS:
            return self._res(a.batch_compare_exchange(idx, current, vals))
        if op == CAS_EPS:
            return self._res(a.batch_compare_exchange_epsilon(idx, current, vals, eps))
        return self._res(getattr(a, _METHOD[op])(idx, vals))

    def op_mvsi(self, op, index, vals, pe=0):
        return self._res(getattr(self.a, _METHOD[op])(int(index), vals))

    def to_numpy(self):
        return host(self.a, self.dt)

    def sub_array(self, lo, hi):
        return _DevArr(self.a.sub_array(lo, hi), self.dt)

    def len(self):
        return self.a.len()


class DevWorld:
    npes = 1

    def __init__(self, lam, world):
        self.lam, self.world = lam, world

    def array(self, kind, length, dist, dt):
        d = self.lam.Distribution.Block if dist == 0 else self.lam.Distribution.Cyclic
        return _DevArr(new(self.lam, self.world, kind, length, d, dt), dt)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("kind", KINDS)
def test_reference_fetch_arith_payloads(world, lam, kind, dt):
    """fetch_sub_test.rs, fetch_mul_test.rs, fetch_div_test.rs, rem_test.rs, fetch_rem_test.rs
    on the device (known answers as pinned in tests/payloads.py)."""
    W = DevWorld(lam, world)
    for dist in (0, 1):
        for n in LENS:
            P.fetch_sub_payload(W, kind, dt, n, dist, np.random.default_rng(n))
            P.fetch_mul_div_payload(W, kind, dt, n, dist)
            P.rem_payload(W, kind, dt, n, dist)


@pytest.mark.parametrize("dt", [d for d in DTS if not d.startswith("f")])
@pytest.mark.parametrize("kind", KINDS)
def test_reference_fetch_bitwise_and_load_store_payloads(world, lam, kind, dt):
    """fetch_and_test.rs, fetch_or_test.rs, load_store_test.rs on the device."""
    W = DevWorld(lam, world)
    for dist in (0, 1):
        for n in LENS:
            P.fetch_and_or_payload(W, kind, dt, n, dist)
            P.load_store_payload(W, kind, dt, n, dist)


@pytest.mark.parametrize("dt", ["f32", "f64"])
@pytest.mark.parametrize("kind", ["AtomicArray", "LocalLockArray"])
def test_reference_compare_exchange_epsilon_payload(world, lam, kind, dt):
    """compare_exchange_test.rs:235-412 (f32 / f64) and load_store on floats, on the device."""
    W = DevWorld(lam, world)
    for dist in (0, 1):
        for n in LENS:
            P.cas_epsilon_payload(W, kind, dt, n, dist)
            P.load_store_payload(W, kind, dt, n, dist)


@pytest.mark.parametrize("kind", KINDS)
def test_reference_input_payloads(world, lam, kind):
    """The `input` variants (add_test.rs:326-505, fetch_add_test.rs:371-560,
    compare_exchange_test.rs:448-470) at len 4 / 100 / 2000: every OpInput container --
    Python ints and numpy scalars per element, a numpy slice, a list, and another array's
    local data (a device tensor) -- on the device."""
    W = DevWorld(lam, world)
    for dist in (0, 1):
        d = lam.Distribution.Block if dist == 0 else lam.Distribution.Cyclic
        for n in (4, 100, 2000):
            inp = lam.UnsafeArray(world.team(), n, d, "usize")
            inp.local_data().copy_(torch.arange(n, dtype=torch.int64, device=inp.local_data().device))
            cont = P.index_containers(lambda m, pe, inp=inp: [inp.local_data()])
            P.add_input_payload(W, kind, n, dist, cont)
            P.fetch_add_input_payload(W, kind, n, dist, cont)
            if kind != "UnsafeArray":
                P.cas_input_payload(W, kind, n, dist)


@pytest.mark.parametrize("dt", ["u8", "f64"])
def test_reference_array_ops_example(world, lam, dt):
    """examples/array_examples/array_ops.rs (u8 and f64 halves, incl. shl / shr) on the device."""
    P.array_ops_example_payload(DevWorld(lam, world), dt)
