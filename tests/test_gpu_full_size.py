"""BASELINE.json's single-GPU configurations at their full sizes, checked through properties that
do not depend on size (the oracle's serial replay covers the same paths at 2^22 records in
test_gpu_deferred_inputs.py, test_gpu_linearize.py and test_gpu_wide.py; at 2^28 it would take
minutes of CPU time). Every check runs on the device with torch as the counter:

- C2 (configs[1]): two deferred 2^28-record u64 batch_add batches from distinct buffers into a
  2^26-element shard — one shard sweep — against torch's index_add_ (wrapping int64 adds: exact in
  any order), bit for bit.
- C4's exchange path (configs[3] at one rank): the same two batches forced through
  lmr_batch_exchange over a 1-rank RCCL communicator (pack, all-to-all-v, the owner's deferred
  count-free session), the same bit-exact check.
- C3 (configs[2]): two 2^26-record f64 batch_fetch_add batches of 1.0 on Zipf(0.99) indices over
  2^24 elements (the wide one-level path), from an integer-valued start: per element, the olds of
  both batches are exactly start, start + 1, ..., start + c - 1 (every fetch saw a distinct
  prefix: linearisable), and the final value is start + c.
- C5 (configs[4], one PE's 2^27 records): u32 bit_and / bit_or / bit_xor batches, each final
  state against per-bit counts (AND: every record has the bit; OR: any; XOR: odd count), and a
  swap batch whose olds plus the final values are the multiset of the previous values plus the
  swapped-in ones, per element.
Each check runs in a process of its own: the workspace these sizes reserve (grow-only, up to
2^29 records) must not outlive them in the test session, whose other tests size their deferred
sessions by the workspace they reserve.
Reference semantics: src/array/operations/arithmetic.rs, bitwise.rs, access.rs (swap);
fetch results in input order, handle.rs:293-325."""
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

M32 = 0xFFFFFFFF


def _gen(seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return g


def c2_full_size_two_batch_session(world, lam, exchange=False):
    team = world.team()
    k = team.kernels
    n_el, n = 1 << 26, 1 << 28
    g = _gen(0xC2)
    arr = lam.AtomicArray(team, n_el, lam.Distribution.Block, "u64")
    s0 = torch.randint(-2**63, 2**63 - 1, (n_el,), dtype=torch.int64, device="cuda", generator=g)
    arr.local_data().copy_(s0)
    batches = [(torch.randint(0, n_el, (n,), dtype=torch.int64, device="cuda", generator=g),
                torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda", generator=g))
               for _ in range(2)]
    k.reserve(2 * n)
    arr.local_data()
    k.profile(True)
    k.profile_read(reset=True)
    try:
        for i, v in batches:
            arr.batch_add(i, v).spawn()
        world.wait_all()
        stages = k.profile_read(reset=True)
    finally:
        k.profile(False)
    assert k.errors() == 0
    assert stages["tile_apply"][1] == 1, stages           # both batches in one shard sweep
    if exchange:                                          # packed, sent and staged by the owner
        assert stages.get("pack", (0, 0))[1] >= 2, stages
    ref = s0.clone()
    for i, v in batches:
        ref.index_add_(0, i, v)
    assert torch.equal(arr.local_data(), ref)


def c3_full_size_fetch_add_linearisable(world, lam):
    team = world.team()
    k = team.kernels
    n_el, n = 1 << 24, 1 << 26
    g = _gen(0xC3)
    ranks = torch.arange(1, n_el + 1, dtype=torch.float64, device="cuda")
    cdf = torch.cumsum(ranks.pow(-0.99), 0)
    cdf /= cdf[-1].clone()
    perm = torch.randperm(n_el, device="cuda", generator=g)
    batches = []
    for _ in range(2):
        r = torch.searchsorted(cdf, torch.rand(n, dtype=torch.float64, device="cuda", generator=g))
        batches.append(perm[r.clamp_(max=n_el - 1)].contiguous())
    del ranks, cdf
    arr = lam.AtomicArray(team, n_el, lam.Distribution.Block, "f64")
    s0 = torch.randint(0, 1 << 20, (n_el,), device="cuda", generator=g).to(torch.float64)
    arr.local_data().copy_(s0)
    ones = torch.ones(n, dtype=torch.float64, device="cuda")
    k.reserve(2 * n)
    hs = [arr.batch_fetch_add(i, ones).spawn() for i in batches]
    olds = torch.cat([h.block() for h in hs])
    world.wait_all()
    assert k.errors() == 0
    idx = torch.cat(batches)
    cnt = torch.bincount(idx, minlength=n_el)
    assert int(cnt.max()) > 1 << 16                       # Zipf-hot: the top element's records
    assert torch.equal(arr.local_data(), s0 + cnt.to(torch.float64))
    rank = olds - s0[idx]                                 # this record's place in its element's order
    assert torch.equal(rank, rank.round()) and bool((rank >= 0).all())
    key = (idx << 27) | rank.to(torch.int64)              # rank < 2^27 records
    key, _ = torch.sort(key)
    sidx, srank = key >> 27, key & ((1 << 27) - 1)
    starts = torch.cumsum(cnt, 0) - cnt
    pos = torch.arange(idx.numel(), device="cuda")
    assert torch.equal(srank, pos - starts[sidx])         # ranks 0..c-1 per element, each once


def _bit_counts(idx, v, n_el):
    """per element and bit: how many records set it (int64 [32, n_el])"""
    out = torch.zeros(32, n_el, dtype=torch.int64, device="cuda")
    for b in range(32):
        out[b].index_add_(0, idx, (v >> b) & 1)
    return out


def c5_full_size_bitwise_and_swap(world, lam):
    team = world.team()
    k = team.kernels
    n_el, n = 1 << 26, (1 << 27) // 5
    g = _gen(0xC5)
    arr = lam.AtomicArray(team, n_el, lam.Distribution.Block, "u32")
    s0 = torch.randint(-2**31, 2**31 - 1, (n_el,), dtype=torch.int32, device="cuda", generator=g)
    arr.local_data().copy_(s0)
    k.reserve(n)
    weights = (torch.ones(32, 1, dtype=torch.int64, device="cuda") << torch.arange(32, device="cuda").view(32, 1))

    def state():
        return arr.local_data().to(torch.int64) & M32

    for op in ("and", "or", "xor"):
        i = torch.randint(0, n_el, (n,), dtype=torch.int64, device="cuda", generator=g)
        v = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=g)
        before = state()
        getattr(arr, f"batch_bit_{op}")(i, v).spawn()
        world.wait_all()
        assert k.errors() == 0
        bits = _bit_counts(i, v.to(torch.int64) & M32, n_el)
        if op == "and":
            cnt = torch.bincount(i, minlength=n_el)
            mask = ((bits == cnt.view(1, -1)).to(torch.int64) * weights).sum(0)   # every record has it
            expect = before & mask
        elif op == "or":
            expect = before | ((bits > 0).to(torch.int64) * weights).sum(0)
        else:
            expect = before ^ ((bits & 1) * weights).sum(0)
        assert torch.equal(state(), expect), op
        del bits
    i = torch.randint(0, n_el, (n,), dtype=torch.int64, device="cuda", generator=g)
    v = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=g)
    before = state()
    olds = arr.batch_swap(i, v).block().to(torch.int64) & M32
    assert k.errors() == 0
    after = state()
    hit = torch.bincount(i, minlength=n_el) > 0
    touched = torch.nonzero(hit).flatten()
    assert torch.equal(after[~hit], before[~hit])
    # per element: {olds} + {final} == {previous} + {swapped-in values}, as multisets of (element, value)
    lhs = torch.cat([(i << 32) | olds, (touched << 32) | after[touched]])
    rhs = torch.cat([(touched << 32) | before[touched], (i << 32) | (v.to(torch.int64) & M32)])
    assert torch.equal(torch.sort(lhs)[0], torch.sort(rhs)[0])


CHECKS = {"c2": c2_full_size_two_batch_session, "c3": c3_full_size_fetch_add_linearisable,
          "c4": lambda w, lam_: c2_full_size_two_batch_session(w, lam_, exchange=True),
          "c5": c5_full_size_bitwise_and_swap}


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", sorted(CHECKS))
def test_full_size(cfg):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    if cfg == "c4":      # C2's batches through lmr_batch_exchange over a 1-rank RCCL communicator
        env.update(LAMELLAR_COMM_BACKEND="nccl", LAMELLAR_FORCE_EXCHANGE="1", RANK="0", WORLD_SIZE="1",
                   LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29600 + os.getpid() % 200))
    p = subprocess.run([sys.executable, os.path.abspath(__file__), cfg], env=env, timeout=170,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert p.returncode == 0, p.stdout[-4000:]
    assert f"{cfg} ok" in p.stdout, p.stdout[-4000:]


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    from _lamellar_bootstrap import load_package
    lam_ = load_package()
    world_ = lam_.LamellarWorldBuilder().build()
    CHECKS[sys.argv[1]](world_, lam_)
    print(sys.argv[1], "ok", flush=True)
