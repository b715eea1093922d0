"""One-AM batches through the device exchange (lmr_batch_exchange) at 1, 2, 3 and 4 PEs
sharing the box's GPU: the reference's outcome, bit for bit.

In the reference a batch of fewer than 1000 records is one OpInput chunk
(src/array/operations.rs:462-469); its pack appends each destination's records in input
order into one buffer, flushed as one AM per destination (unsafe/operations.rs:709-778),
and the owner's AM applies its records sequentially (impl/src/array_ops.rs:203-250; a
PE's own buffer through the local shortcut, registered_active_message.rs:150-154). AMs
of different sources run concurrently, so the outcome is fixed per source, not across
sources: `batch_swap([5, 5], [1, 2])` on a remote element always ends at 2.

Check, per op (swap, store, compare_exchange, fetch_rem, f64 fetch_add with non-exact
sums; indices repeated within and across PEs) and per owner PE: some order of the
sources' AMs, each AM applied sequentially by the oracle (oracle/lamellar_oracle.c, the
AMs built by the oracle's restatement of the reference's pack), reproduces the owner's
final slice and every returned value / Ok flag bit-exactly. The AMs are the reference's
own: `orc.pack` of each source's batch, one AM per destination below 1000 records.
"""
import itertools
import tempfile

import numpy as np
import pytest

from opgen import NP, bits_equal
from test_gpu_dist_ordered import DTN, run_pes

pytestmark = pytest.mark.gpu

LEN_SMALL = 997
NREC_SMALL = 700


def owner_slices(orc, L, n_len, ws):
    """global index -> (owner PE, local offset) for the whole array; per PE the global
    indices of its local slice in offset order."""
    own = np.zeros(n_len, np.int64)
    off = np.zeros(n_len, np.int64)
    for g in range(n_len):
        own[g], off[g] = orc.pe_and_offset(L, g)
    return [np.arange(n_len)[own == o][np.argsort(off[own == o])] for o in range(ws)]


def check_small(orc, pe, ws, dist_kind):
    names = sorted({k.split(":")[0] for k in pe[0] if k.endswith(":meta")})
    assert len(names) == 5, names
    L0 = orc.layout_new(LEN_SMALL, ws, 0, dist_kind)
    iw = orc.index_size(L0)
    glob = owner_slices(orc, L0, LEN_SMALL, ws)
    for name in names:
        op, code, kind = (int(x) for x in pe[0][name + ":meta"])
        t = NP[DTN[code]]
        before, after = pe[0][name + ":before"], pe[0][name + ":after"]
        for p in pe[1:]:
            assert np.array_equal(p[name + ":after"].view(np.uint8), after.view(np.uint8)), name
        cur = pe[0][name + ":cur"][0] if name + ":cur" in pe[0] else None
        # every source's AMs, as the reference's pack builds them
        ams = {}
        for s in range(ws):
            Ls = orc.layout_new(LEN_SMALL, ws, s, dist_kind)
            st, lst = orc.pack(Ls, code, t, pe[s][name + ":idx"], pe[s][name + ":vals"].astype(t), iw)
            assert st == 0
            for dst, byts, pos in lst:
                assert (s, dst) not in ams, "more than one AM per destination: not a one-AM batch"
                ams[(s, dst)] = (byts, pos)
        for o in range(ws):
            g = glob[o]
            srcs = [s for s in range(ws) if (s, o) in ams]
            matched = False
            for order in itertools.permutations(srcs):
                sl = before[g].copy()
                good = True
                for s in order:
                    byts, pos = ams[(s, o)]
                    st, res, ok = orc.apply_mvmi(sl, kind, code, t, op, byts, iw, cur, None)
                    assert st == 0
                    if name + ":res" in pe[s]:
                        good = good and bits_equal(pe[s][name + ":res"].astype(t)[pos.astype(np.int64)], res)
                    if name + ":ok" in pe[s]:
                        good = good and np.array_equal(pe[s][name + ":ok"][pos.astype(np.int64)], ok)
                good = good and bits_equal(sl, after[g])
                if good:
                    matched = True
                    break
            assert matched, (name, "owner", o, "no order of the sources' AMs reproduces the device")
        if name == "cas_i64":
            oks = np.concatenate([p[name + ":ok"] for p in pe])
            assert oks.any() and not oks.all(), "expected successes and failures"


@pytest.mark.parametrize("ws,dist_kind,xport", [(2, 0, "host"), (3, 1, "host"), (4, 0, "host"), (3, 0, "devptr")],
                         ids=["2pe-Block", "3pe-Cyclic", "4pe-Block", "3pe-Block-devptr"])
def test_one_am_batches_match_reference_order(orc, ws, dist_kind, xport):
    env = {"LAMELLAR_COMM_BACKEND": "gloo", "LMR_MODE": "small", "LMR_LEN": str(LEN_SMALL),
           "LMR_NREC": str(NREC_SMALL)}
    if xport == "devptr":
        env["LMR_XPORT"] = "devptr"
    with tempfile.TemporaryDirectory() as d:
        pe = run_pes(ws, dist_kind, env, d, 29500 + 10 * ws + dist_kind + (5 if xport == "devptr" else 0))
    check_small(orc, pe, ws, dist_kind)


def test_one_am_batches_rccl_one_rank(orc):
    """One source through a 1-rank RCCL communicator (LAMELLAR_FORCE_EXCHANGE=1): the
    exchange's ordered path over RCCL's grouped send / recv."""
    env = {"LAMELLAR_COMM_BACKEND": "nccl", "LAMELLAR_FORCE_EXCHANGE": "1", "LMR_MODE": "small",
           "LMR_LEN": str(LEN_SMALL), "LMR_NREC": str(NREC_SMALL)}
    with tempfile.TemporaryDirectory() as d:
        pe = run_pes(1, 0, env, d, 29590)
    check_small(orc, pe, 1, 0)
