"""CPU check of the one-AM replay checker used by test_gpu_dist_small.py: a simulated
exchange that applies every source's AM in PE order (the oracle standing in for the
device) passes, and one whose final state or returned values were produced by a
different in-AM order fails."""
import numpy as np
import pytest

from opgen import CAS, CODE, FETCH_ADD, NP, SWAP
from test_gpu_dist_small import LEN_SMALL, check_small, owner_slices


def simulate(orc, ws, dist_kind, op, dt, nrec=300, reverse_in_am=False, seed=3):
    t = NP[dt]
    rng = np.random.default_rng(seed)
    hot = rng.choice(LEN_SMALL, 24, replace=False).astype(np.uint64)
    before = (rng.integers(0, 3, LEN_SMALL) if op == CAS else rng.integers(0, 2**40, LEN_SMALL)).astype(t)
    if dt == "f64":
        before = rng.random(LEN_SMALL) * 1e3
    L0 = orc.layout_new(LEN_SMALL, ws, 0, dist_kind)
    iw = orc.index_size(L0)
    glob = owner_slices(orc, L0, LEN_SMALL, ws)
    pe = [dict() for _ in range(ws)]
    name = "case"
    cur = t(1) if op == CAS else None
    for s in range(ws):
        pe[s][name + ":idx"] = hot[rng.integers(0, hot.size, nrec)]
        v = rng.integers(0, 3, nrec) if op == CAS else rng.integers(0, 2**40, nrec)
        pe[s][name + ":vals"] = (rng.random(nrec) * 10 - 5) if dt == "f64" else v.astype(t)
        pe[s][name + ":res"] = np.zeros(nrec, t)
        if op == CAS:
            pe[s][name + ":ok"] = np.zeros(nrec, np.uint8)
            pe[s][name + ":cur"] = np.array([cur], t)
        pe[s][name + ":meta"] = np.array([op, CODE[dt], 2 if dt == "f64" else 1])
    after = before.copy()
    for o in range(ws):
        sl = after[glob[o]].copy()
        for s in range(ws):
            Ls = orc.layout_new(LEN_SMALL, ws, s, dist_kind)
            idx, vals = pe[s][name + ":idx"], pe[s][name + ":vals"]
            if reverse_in_am:
                idx, vals = idx[::-1].copy(), vals[::-1].copy()
            st, lst = orc.pack(Ls, CODE[dt], t, idx, vals, iw)
            for dst, byts, pos in lst:
                if dst != o:
                    continue
                st, res, ok = orc.apply_mvmi(sl, 2 if dt == "f64" else 1, CODE[dt], t, op, byts, iw, cur, None)
                p = pos.astype(np.int64)
                if reverse_in_am:
                    p = nrec - 1 - p
                pe[s][name + ":res"][p] = res
                if op == CAS:
                    pe[s][name + ":ok"][p] = ok
        after[glob[o]] = sl
    for s in range(ws):
        pe[s][name + ":before"], pe[s][name + ":after"] = before, after
    # the checker expects five cases; replicate this one under five names
    out = []
    for s in range(ws):
        d = {}
        for k in range(5):
            d.update({f"c{k}" + key[len(name):]: val for key, val in pe[s].items()})
        out.append(d)
    return out


@pytest.mark.parametrize("ws,dist_kind", [(2, 0), (3, 1)])
@pytest.mark.parametrize("op,dt", [(SWAP, "u64"), (CAS, "i64"), (FETCH_ADD, "f64")])
def test_replay_checker_accepts_per_source_order(orc, ws, dist_kind, op, dt):
    check_small(orc, simulate(orc, ws, dist_kind, op, dt), ws, dist_kind)


@pytest.mark.parametrize("op,dt", [(SWAP, "u64"), (FETCH_ADD, "f64")])
def test_replay_checker_rejects_other_in_am_order(orc, op, dt):
    with pytest.raises(AssertionError):
        check_small(orc, simulate(orc, 2, 0, op, dt, reverse_in_am=True), 2, 0)
