"""The reference's integration-test payloads, restated once for two backends (test-only).

Each function follows one payload of tests/array/** (run by tests/<op>.rs through
lamellar_run.sh) and checks that payload's own known answer. They run
against an adapter `W` with `W.npes` PEs:
  - SimWorld (tests/simworld.py): every PE simulated by the CPU oracle; PE p's requests
    are issued as PE p's batch and the PEs' batches are applied in turn (a valid
    serialisation of the reference's concurrent AMs) -> pins the oracle;
  - DevWorld (tests/test_gpu_reference_programs.py): one PE, the op-builder API over the
    gfx950 path -> the device twin.
An array adapter offers fill(v), set(values in global order), op(code, idx, vals,
current=None, eps=None) -> (results, ok), to_numpy() (global order), sub_array(lo, hi)
and len(). Float checks use the payloads' check_val! (|val - expect| <= 1e-4).

Two payloads cannot pass as written, and the restatement says why instead of copying
the wrong expectation (see rem_payload): rem_test.rs / fetch_rem_test.rs expect 1 after
`rem(2)` of 2^k, which is 0 for k >= 1, and neither is registered as an example in the
reference's Cargo.toml (so tests/rem.rs and tests/fetch_rem.rs cannot launch them).
"""
import numpy as np

from opgen import (ADD, AND, CAS, CAS_EPS, DIV, FETCH_ADD, FETCH_AND, FETCH_DIV, FETCH_MUL, FETCH_OR,
                   FETCH_REM, FETCH_SHL, FETCH_SHR, FETCH_SUB, FETCH_XOR, LOAD, MUL, NP, OR, REM, SHL, SHR,
                   STORE, SUB, XOR)

INT_TYPES = ["u8", "u16", "u32", "u64", "i8", "i16", "i32", "i64"]
ALL_TYPES = INT_TYPES + ["f32", "f64"]


def T(dt, v):
    return np.array([v]).astype(NP[dt])[0]


def close(vals, expect):
    """check_val!: ((val - expect) as f32).abs() <= 0.0001, T-wrapping subtraction."""
    vals = np.atleast_1d(vals)
    d = (vals - np.array([expect]).astype(vals.dtype)).astype(np.float64)
    return bool(np.all(np.abs(d) <= 1e-4))


def tmax(dt):
    if dt == "f32":
        return int(np.finfo(np.float32).max)          # f32::MAX as u128 (exact, below u128::MAX)
    if dt == "f64":
        return (1 << 128) - 1                          # f64::MAX as u128 saturates
    return int(np.iinfo(NP[dt]).max)


def max_updates_log2(dt, npes):
    """max_updates! of mul/div/rem/fetch_mul/fetch_div/fetch_rem_test.rs:
    (128 - (T::MAX as u128 / num_pes).leading_zeros() - 1) / num_pes."""
    q = tmax(dt) // npes
    return (q.bit_length() - 1) // npes


def max_updates_1000(dt, npes):
    """max_updates! of fetch_sub_test.rs:78-86: 1000 / num_pes if T::MAX > 1000 else T::MAX / num_pes."""
    return 1000 // npes if tmax(dt) > 1000 else tmax(dt) // npes


def sub_arrays(total, npes):
    """The sub-array sweep the payloads share: the half array [total/4, total/4 + total/2)
    and, per PE, [pe * pe_len + len/2, + len) with len = max(pe_len / 2, 1)."""
    half = total // 2
    out = [(half // 2, half // 2 + half)]
    pe_len = total // npes
    for pe in range(npes):
        ln = max(pe_len // 2, 1)
        st = pe * pe_len + ln // 2
        out.append((st, st + ln))
    return out


def distinct_per_pe(res, idx):
    """insert_prev!: the olds one PE receives for one index are all distinct."""
    for i in np.unique(idx):
        r = res[idx == i]
        if np.unique(r.view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[r.itemsize])).size != r.size:
            return False
    return True


# ---------------------------------------------------------------- arithmetic
def fetch_sub_payload(W, kind, dt, length, dist, rng):
    """fetch_sub_test.rs:97-280: init pe_max_val * num_pes (10 per PE); every PE issues 10
    fetch_sub(idx, 1) per index: its olds per index are distinct, every element ends at 0.
    Then init tot = num_updates * num_pes and each PE issues num_updates fetch_sub at random
    indices: the array sums to tot * (len - 1). Repeated on the half and per-PE sub-arrays."""
    npes = W.npes
    a = W.array(kind, length, dist, dt)
    for (lo, hi) in [(0, length)] + sub_arrays(length, npes):
        s = a if (lo, hi) == (0, length) else a.sub_array(lo, hi)
        n = s.len()
        a.fill(T(dt, 10 * npes))
        for pe in range(npes):
            idx = np.repeat(np.arange(n, dtype=np.uint64), 10)
            res, _ = s.op(FETCH_SUB, idx, T(dt, 1), pe=pe)
            assert distinct_per_pe(res, idx), ("fetch_sub olds", dt, npes, lo, hi)
        assert close(s.to_numpy(), T(dt, 0)), ("fetch_sub final", dt, npes, lo, hi)
        nu = max_updates_1000(dt, npes)
        tot = T(dt, nu * npes)
        a.fill(tot)
        for pe in range(npes):
            idx = rng.integers(0, n, nu).astype(np.uint64)
            s.op(FETCH_SUB, idx, T(dt, 1), pe=pe)
        total = float(np.sum(s.to_numpy().astype(np.float64)))
        assert abs(total - float(tot) * (n - 1)) <= 1e-4 * max(1, n), ("fetch_sub sum", dt, npes, lo, hi)


def fetch_mul_div_payload(W, kind, dt, length, dist):
    """fetch_mul_test.rs:104-160: init 1, every PE issues max_updates fetch_mul(idx, 2) per
    index: distinct olds per PE and index, final 2^(max_updates * num_pes).
    fetch_div_test.rs:107-165: init 2^(max_updates * num_pes), fetch_div(idx, 2): distinct
    olds, final 1. Repeated on the half and per-PE sub-arrays."""
    npes = W.npes
    mu = max_updates_log2(dt, npes)
    top = T(dt, 2.0 ** (mu * npes)) if dt.startswith("f") else T(dt, (1 << (mu * npes)) & ((1 << 64) - 1))
    a = W.array(kind, length, dist, dt)
    for (lo, hi) in [(0, length)] + sub_arrays(length, npes):
        s = a if (lo, hi) == (0, length) else a.sub_array(lo, hi)
        n = s.len()
        idx = np.repeat(np.arange(n, dtype=np.uint64), mu)
        a.fill(T(dt, 1))
        for pe in range(npes):
            res, _ = s.op(FETCH_MUL, idx, T(dt, 2), pe=pe)
            assert distinct_per_pe(res, idx), ("fetch_mul olds", dt, npes)
        assert close(s.to_numpy(), top), ("fetch_mul final", dt, npes, lo, hi)
        a.fill(top)
        for pe in range(npes):
            res, _ = s.op(FETCH_DIV, idx, T(dt, 2), pe=pe)
            assert distinct_per_pe(res, idx), ("fetch_div olds", dt, npes)
        assert close(s.to_numpy(), T(dt, 1)), ("fetch_div final", dt, npes, lo, hi)


def rem_payload(W, kind, dt, length, dist):
    """rem_test.rs:78-177 / fetch_rem_test.rs:108-...: init 2^(max_updates * num_pes), every
    PE applies rem(idx, 2) (fetch_rem) max_updates times per index. The payloads check the
    result against 1 and (fetch_rem) that a PE's olds per index are distinct; Rust's `%`
    (impl/src/array_ops.rs:359-368, native_atomic.rs:64-74; fmod for floats, :496-498)
    gives 2^k % 2 = 0 for k >= 1, so the final value is 0 and the olds of one index are
    [2^k, 0, 0, ...] -- what is pinned here. Neither payload is an [[example]] in the
    reference's Cargo.toml, so its drivers (tests/rem.rs, tests/fetch_rem.rs) cannot run it."""
    npes = W.npes
    mu = max_updates_log2(dt, npes)
    k = mu * npes
    top = T(dt, 2.0 ** k) if dt.startswith("f") else T(dt, (1 << k) & ((1 << 64) - 1))
    exp_final = T(dt, 0) if k >= 1 else T(dt, 1)
    a = W.array(kind, length, dist, dt)
    for (lo, hi) in [(0, length)] + sub_arrays(length, npes):
        s = a if (lo, hi) == (0, length) else a.sub_array(lo, hi)
        n = s.len()
        idx = np.repeat(np.arange(n, dtype=np.uint64), mu)
        a.fill(top)
        for pe in range(npes):
            s.op(REM, idx, T(dt, 2), pe=pe)
        assert close(s.to_numpy(), exp_final), ("rem final", dt, npes, lo, hi)
        a.fill(top)
        olds = []
        for pe in range(npes):
            res, _ = s.op(FETCH_REM, idx, T(dt, 2), pe=pe)
            olds.append(res)
        assert close(s.to_numpy(), exp_final), ("fetch_rem final", dt, npes, lo, hi)
        allr = np.concatenate(olds) if olds else np.zeros(0)
        alli = np.concatenate([idx] * npes)
        for i in range(n):
            r = np.sort(allr[alli == i].astype(np.float64))
            want = np.zeros(r.size)
            if r.size:
                want[-1] = float(top)
            assert np.array_equal(r, np.sort(want)), ("fetch_rem olds", dt, npes, i)


# ---------------------------------------------------------------- bitwise
def fetch_and_or_payload(W, kind, dt, length, dist):
    """fetch_and_test.rs:69-110: init !0, PE p fetch_bit_and(idx, !(1 << p)) on every index:
    the old it gets still holds bit p ((old & !my_val) == !my_val), final !0 << num_pes.
    fetch_or_test.rs:69-110: init 0, PE p fetch_bit_or(idx, 1 << p): the old never holds
    bit p, final !(!0 << num_pes). Repeated on the half and per-PE sub-arrays."""
    npes = W.npes
    t = NP[dt]
    ones = t(~t(0))
    a = W.array(kind, length, dist, dt)
    for (lo, hi) in [(0, length)] + sub_arrays(length, npes):
        s = a if (lo, hi) == (0, length) else a.sub_array(lo, hi)
        idx = np.arange(s.len(), dtype=np.uint64)
        a.fill(ones)
        for pe in range(npes):
            mine = t(~(t(1) << t(pe)))
            res, _ = s.op(FETCH_AND, idx, mine, pe=pe)
            assert np.all((res & t(~mine)) == t(~mine)), ("fetch_and olds", dt, npes, pe)
        assert np.all(s.to_numpy() == t(ones << t(npes))), ("fetch_and final", dt, npes, lo, hi)
        a.fill(t(0))
        for pe in range(npes):
            mine = t(t(1) << t(pe))
            res, _ = s.op(FETCH_OR, idx, mine, pe=pe)
            assert np.all((res & mine) == 0), ("fetch_or olds", dt, npes, pe)
        assert np.all(s.to_numpy() == t(~(ones << t(npes)))), ("fetch_or final", dt, npes, lo, hi)


# ---------------------------------------------------------------- access
def load_store_payload(W, kind, dt, length, dist):
    """load_store_test.rs:67-...: init num_pes; PE p store(idx, p) on idx % num_pes == p; then
    every load(idx) reads idx % num_pes. Repeated on the half and per-PE sub-arrays."""
    npes = W.npes
    a = W.array(kind, length, dist, dt)
    for (lo, hi) in [(0, length)] + sub_arrays(length, npes):
        s = a if (lo, hi) == (0, length) else a.sub_array(lo, hi)
        n = s.len()
        a.fill(T(dt, npes))
        for pe in range(npes):
            idx = np.arange(pe, n, npes, dtype=np.uint64)
            if idx.size:
                s.op(STORE, idx, T(dt, pe), pe=pe)
        for pe in range(npes):
            res, _ = s.op(LOAD, np.arange(n, dtype=np.uint64), T(dt, 0), pe=pe)
            want = (np.arange(n) % npes).astype(NP[dt])
            assert close(res - want, T(dt, 0)) if n else True, ("load", dt, npes, lo, hi)


def cas_epsilon_payload(W, kind, dt, length, dist):
    """compare_exchange_test.rs:235-412 (f32 / f64 on Atomic = Generic and LocalLock):
    init num_pes, eps = 0.0001; PE p compare_exchange_epsilon(idx, init, p, eps) on
    idx % num_pes == p returns Ok(~init); then the same on every index fails (Err) since
    every element now holds idx % num_pes. Repeated on the half and per-PE sub-arrays."""
    npes = W.npes
    init, eps = T(dt, npes), T(dt, 0.0001)
    a = W.array(kind, length, dist, dt)
    for (lo, hi) in [(0, length)] + sub_arrays(length, npes):
        s = a if (lo, hi) == (0, length) else a.sub_array(lo, hi)
        n = s.len()
        a.fill(init)
        for pe in range(npes):
            idx = np.arange(pe, n, npes, dtype=np.uint64)
            if idx.size == 0:
                continue
            res, ok = s.op(CAS_EPS, idx, T(dt, pe), current=init, eps=eps, pe=pe)
            assert np.all(ok == 1) and close(res, init), ("cas_eps round 1", dt, npes, lo, hi)
        for pe in range(npes):
            idx = np.arange(n, dtype=np.uint64)
            res, ok = s.op(CAS_EPS, idx, T(dt, pe), current=init, eps=eps, pe=pe)
            assert not np.any(ok), ("cas_eps round 2", dt, npes, lo, hi)


def cas_input_payload(W, kind, length, dist):
    """compare_exchange_test.rs:448-470 (input variant, usize): init num_pes; PE p
    batch_compare_exchange(p, p + num_pes, ...; current = num_pes, new = p): all Ok; then
    batch_compare_exchange(every index, current = p, new = p): Ok exactly where
    idx % num_pes == p (check_input!, :428-446)."""
    npes = W.npes
    a = W.array(kind, length, dist, "u64")
    a.fill(T("u64", npes))
    for pe in range(npes):
        idx = np.arange(pe, length, npes, dtype=np.uint64)
        if idx.size:
            res, ok = a.op(CAS, idx, T("u64", pe), current=T("u64", npes), pe=pe)
            assert np.all(ok == 1), ("cas input round 1", npes, pe)
    for pe in range(npes):
        idx = np.arange(length, dtype=np.uint64)
        res, ok = a.op(CAS, idx, T("u64", pe), current=T("u64", pe), pe=pe)
        assert np.all((ok == 1) == (idx % npes == pe)), ("cas input round 2", npes, pe)
        assert np.all(res[ok == 0] == (idx[ok == 0] % npes)), ("cas input Err values", npes, pe)


# ---------------------------------------------------------------- OpInput containers
def add_input_payload(W, kind, length, dist, containers):
    """add_test.rs:326-505 (input variant, usize): every PE batch_add(indices 0..len, 1)
    through each OpInput container -- a scalar index per call (T, &T), slices, Vecs,
    memory regions and other arrays' local data (an UnsafeArray of len * num_pes whose
    local data on every PE is 0..len) -- and every element then holds num_pes
    (check_results!, :298-324)."""
    npes = W.npes
    a = W.array(kind, length, dist, "u64")
    for name, make in containers:
        a.fill(T("u64", 0))
        for pe in range(npes):
            for idx in make(length, pe):
                a.op(ADD, idx, T("u64", 1), pe=pe)
        assert np.all(a.to_numpy() == npes), ("add input", name, npes, length)


def fetch_add_input_payload(W, kind, length, dist, containers):
    """fetch_add_test.rs:371-560 (input variant, usize): init a[i] = i; every PE
    batch_fetch_add(indices 0..len, 1) through each container. check_results!
    (:371-430): the k-th result a PE receives (in request order) lies in [0, k + num_pes),
    and finally a[i] = i + num_pes. MVSI form batch_fetch_add(my_pe, &[1; len]): results
    in [0, num_pes + len), final a[i] = i + len for i < num_pes, i otherwise."""
    npes = W.npes
    a = W.array(kind, length, dist, "u64")
    base = np.arange(length, dtype=np.uint64)
    for name, make in containers:
        a.set(base)
        for pe in range(npes):
            got = []
            for idx in make(length, pe):
                res, _ = a.op(FETCH_ADD, idx, T("u64", 1), pe=pe)
                got.append(np.asarray(res, dtype=np.uint64))
            got = np.concatenate(got)
            assert np.all(got < np.arange(got.size, dtype=np.uint64) + np.uint64(npes)), \
                ("fetch_add input olds", name, npes, pe)
        assert np.array_equal(a.to_numpy(), base + np.uint64(npes)), ("fetch_add input final", name, npes)
    a.set(base)
    for pe in range(npes):
        res, _ = a.op_mvsi(FETCH_ADD, pe, np.ones(length, dtype=np.uint64), pe=pe)
        assert np.all(np.asarray(res, dtype=np.uint64) < np.uint64(npes + length)), ("fetch_add mvsi olds", npes)
    exp = base.copy()
    exp[:min(npes, length)] += np.uint64(length)
    assert np.array_equal(a.to_numpy(), exp), ("fetch_add mvsi final", npes, length)


def index_containers(local_data_of=None):
    """The OpInput containers of the input variants, as index lists issued by one PE:
    per-element scalars (T, &T), one slice/Vec (&[T], Vec<T>, &Vec<T>, scoped forms,
    LMR / SMR: same indices), and an array's local data (0..len on every PE)."""
    out = [("T", lambda n, pe: [i for i in range(n)]),
           ("&T", lambda n, pe: [np.uint64(i) for i in range(n)]),
           ("&[T]", lambda n, pe: [np.arange(n, dtype=np.uint64)]),
           ("Vec<T>", lambda n, pe: [list(range(n))]),
           ("LMR<T>", lambda n, pe: [np.arange(n, dtype=np.uint64)])]
    if local_data_of is not None:
        out.append(("&UnsafeArray<T>", local_data_of))
    return out


# ---------------------------------------------------------------- examples/array_examples/array_ops.rs
def _step(op, dt, x, v):
    """One record on a register copy (the reference's per-op semantics, array_ops.rs:327-458)."""
    t = NP[dt]
    with np.errstate(over="ignore"):
        x, v = t(x), t(v)
        if op in (ADD, FETCH_ADD):
            return t(x + v)
        if op in (SUB, FETCH_SUB):
            return t(x - v)
        if op in (MUL, FETCH_MUL):
            return t(x * v)
        if op in (DIV, FETCH_DIV):
            return t(x / v) if dt.startswith("f") else t(x // v)
        if op in (REM, FETCH_REM):
            return t(np.fmod(x, v)) if dt.startswith("f") else t(x % v)
        if op in (AND, FETCH_AND):
            return t(x & v)
        if op in (OR, FETCH_OR):
            return t(x | v)
        if op in (XOR, FETCH_XOR):
            return t(x ^ v)
        bits = 8 * t(0).itemsize
        if op in (SHL, FETCH_SHL):
            return t((int(x) << (int(v) & (bits - 1))) & ((1 << bits) - 1))
        return t(int(x) >> (int(v) & (bits - 1)))


def _reachable(op, dt, x0, vals):
    """Every value an element can hold after some subset of `vals` in some order (the
    olds one PE's fetch may return while the other PEs' records run concurrently)."""
    states = {NP[dt](x0).tobytes(): NP[dt](x0)}
    frontier = [(NP[dt](x0), tuple(range(len(vals))))]
    while frontier:
        nxt = []
        for x, rest in frontier:
            for j in rest:
                y = _step(op, dt, x, vals[j])
                r = tuple(q for q in rest if q != j)
                if y.tobytes() not in states or r:
                    states[y.tobytes()] = y
                    nxt.append((y, r))
        frontier = nxt
    return set(states)


ARRAY_OPS_EXAMPLE = {
    # dt: [(op, fetch op, init, per-PE value (pe, npes) -> v, reset before the fetch phase,
    #       trailing single op at index 3 or 1 (index, value(npes)) or None)]
    "u8": [(ADD, FETCH_ADD, 0, lambda pe, n: 1, False, (3, lambda n: 1)),
           (SUB, FETCH_SUB, 10, lambda pe, n: 1, False, (3, lambda n: 1)),
           (MUL, FETCH_MUL, 1, lambda pe, n: 2, False, None),
           (DIV, FETCH_DIV, 255, lambda pe, n: 2, False, None),
           (REM, FETCH_REM, 255, lambda pe, n: 2, False, None),
           (AND, FETCH_AND, 255, lambda pe, n: 1 << pe, True, (3, lambda n: 1 << n)),
           (OR, FETCH_OR, 0, lambda pe, n: 1 << pe, True, (3, lambda n: 1 << n)),
           (XOR, FETCH_XOR, 0, lambda pe, n: 1 << pe, True, (3, lambda n: 1 << n)),
           (SHL, FETCH_SHL, 1, lambda pe, n: 3, False, (1, lambda n: 3)),
           (SHR, FETCH_SHR, 255, lambda pe, n: 3, False, (1, lambda n: 3))],
    "f64": [(ADD, FETCH_ADD, 0.0, lambda pe, n: 1.0, False, (3, lambda n: 1.0)),
            (SUB, FETCH_SUB, 10.0, lambda pe, n: 1.0, False, None),
            (MUL, FETCH_MUL, 1.0, lambda pe, n: 2.5, False, None),
            (DIV, FETCH_DIV, 1000.0, lambda pe, n: 2.5, False, None),
            (REM, FETCH_REM, 1000.0, lambda pe, n: 2.5, False, None)],
}


def array_ops_example_payload(W, dt):
    """examples/array_examples/array_ops.rs:474-830 on AtomicArray<u8> and AtomicArray<f64>
    (num_pes * 10 elements, Block): each test_<op> (:80-458) stores init, every PE issues
    <op>(i, val) for every index i, then fetch_<op>(i, val) for every i (test_and / test_or /
    test_xor store init again first), and main follows some tests with one more <op> at
    index 3 (or 1 for shl / shr) from every PE. The example only prints; its answers follow
    from the ops: after the first phase every element holds init with every PE's value
    applied, the fetch olds a PE gets are init' with some subset of the other PEs' values
    applied (_reachable), and the final value has every value applied again. Also
    test_store_load (:360-392): PE p stores p on i = p (mod num_pes), every load(i) reads
    i % num_pes. Shl / shr here are the batched path's (array_ops.rs:420-458); the element
    wrapper's ShlAssign / ShrAssign (native_atomic.rs:90-111) shift the wrong way on a CAS
    retry (shl) or on the first try (shr) -- not on this path, not reproduced."""
    npes = W.npes
    n = 10 * npes
    t = NP[dt]
    a = W.array("AtomicArray", n, 0, dt)
    idx = np.arange(n, dtype=np.uint64)
    for op, fop, init, val, reset, trail in ARRAY_OPS_EXAMPLE[dt]:
        vals = [t(val(pe, npes)) for pe in range(npes)]
        a.fill(t(init))
        for pe in range(npes):
            a.op(op, idx, vals[pe], pe=pe)
        x1 = t(init)
        for v in vals:
            x1 = _step(op, dt, x1, v)
        got = a.to_numpy()
        assert np.array_equal(got, np.full(n, x1, dtype=t)), ("phase 1", dt, op, npes, got[:4], x1)
        if reset:
            a.fill(t(init))
            x1 = t(init)
        for pe in range(npes):
            res, _ = a.op(fop, idx, vals[pe], pe=pe)
            others = [vals[q] for q in range(npes) if q != pe]
            ok = _reachable(op, dt, x1, others)
            assert all(t(r).tobytes() in ok for r in res), ("fetch olds", dt, fop, npes, pe)
        x2 = x1
        for v in vals:
            x2 = _step(op, dt, x2, v)
        assert np.array_equal(a.to_numpy(), np.full(n, x2, dtype=t)), ("phase 2", dt, fop, npes)
        if trail is not None:
            i, tv = trail
            for pe in range(npes):
                a.op(op, np.array([i], dtype=np.uint64), t(tv(npes)), pe=pe)
            x3 = x2
            for _ in range(npes):
                x3 = _step(op, dt, x3, t(tv(npes)))
            want = np.full(n, x2, dtype=t)
            want[i] = x3
            assert np.array_equal(a.to_numpy(), want), ("trailing", dt, op, npes)
    # test_store_load
    a.fill(t(0))
    for pe in range(npes):
        a.op(STORE, np.arange(pe, n, npes, dtype=np.uint64), t(pe), pe=pe)
    for pe in range(npes):
        res, _ = a.op(LOAD, idx, t(0), pe=pe)
        assert np.array_equal(res, (np.arange(n) % npes).astype(t)), ("load", dt, npes)
