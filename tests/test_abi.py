"""C-ABI checks that need no GPU: the library loads, exports every symbol
include/lamellar_gpu_ops.h declares, and its host-side index math / record
layout / op tables agree with the CPU oracle (no device compute is called)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "lamellar_gpu_ops.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lmr_[a-z0-9_]+)\s*\((?!\*)", src)))   # not function-pointer fields


def test_library_exports_every_declared_symbol(capi):
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(capi, s)]
    assert not missing, missing


def test_ctypes_binding_covers_header(lam):
    from lamellar_runtime_amd import _capi
    assert set(declared_symbols()) == set(_capi.SIGNATURES)


def test_integration_extern_block_covers_header():
    """INTEGRATION.md's Rust `extern "C"` block declares every function of the C ABI."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```rust\n(.*?)```", text, flags=re.S)
    declared = set()
    for b in blocks:
        for ext in re.findall(r'extern "C" \{(.*?)\n\}', b, flags=re.S):
            declared |= set(re.findall(r"\bpub fn (lmr_[a-z0-9_]+)\s*\(", ext))
    missing = sorted(set(declared_symbols()) - declared)
    assert not missing, missing
    extra = sorted(declared - set(declared_symbols()))
    assert not extra, extra


def test_abi_version_and_status_strings(capi, lam):
    from lamellar_runtime_amd import _capi
    assert capi.lmr_abi_version() == 8
    assert _capi.status_string(2) == "index out of bounds"
    assert _capi.status_string(3).startswith("integer division")


def _pair(capi, orc, size, npes, dist, sub=None):
    from lamellar_runtime_amd import _capi
    Lo = orc.layout_new(size, npes, 0, dist)
    Ld = _capi.lmr_layout_t()
    assert capi.lmr_layout_new(ctypes.byref(Ld), size, npes, 0, dist) == 0
    if sub:
        Lo = orc.layout_sub(Lo, *sub)
        L2 = _capi.lmr_layout_t()
        assert capi.lmr_layout_sub(ctypes.byref(Ld), sub[0], sub[1], ctypes.byref(L2)) == 0
        Ld = L2
    return Lo, Ld


@pytest.mark.parametrize("dist", [0, 1])
@pytest.mark.parametrize("npes", [1, 2, 3, 4, 7, 8])
def test_host_index_math_matches_oracle(capi, orc, npes, dist):
    """pe_and_offset / num_elems_pe / local slice / IndexSize on full and sub arrays."""
    rng = np.random.default_rng(npes * 10 + dist)
    for size in [1, 2, 3, 7, 19, 128, 255, 256, 1000, 65535, 65536, 70001]:
        subs = [None, (0, size)]
        if size > 4:
            a = int(rng.integers(0, size // 2))
            subs.append((a, int(rng.integers(a + 1, size + 1))))
        for sub in subs:
            Lo, Ld = _pair(capi, orc, size, npes, dist, sub)
            assert Lo.as_tuple() == Ld.as_tuple()
            assert orc.index_size(Lo) == capi.lmr_index_size(ctypes.byref(Ld))
            tot = 0
            for p in range(npes):
                n = orc.num_elems_pe(Lo, p)
                tot += n
                assert n == capi.lmr_num_elems_pe(ctypes.byref(Ld), p)
                assert orc.local_slice_start(Lo, p) == capi.lmr_local_slice_start(ctypes.byref(Ld), p)
            assert tot == Lo.size
            seen = set()
            idxs = list(range(min(Lo.size, 400))) + [Lo.size, Lo.size + 5]
            for i in idxs:
                a = orc.pe_and_offset(Lo, i)
                pe, off = ctypes.c_uint64(), ctypes.c_uint64()
                okd = capi.lmr_pe_and_offset(ctypes.byref(Ld), i, ctypes.byref(pe), ctypes.byref(off))
                assert a == ((pe.value, off.value) if okd else None), (size, npes, dist, sub, i)
                if a is not None:
                    assert a[1] < orc.num_elems_pe(Lo, a[0])        # lands inside the PE's slice
                    assert a not in seen                            # bijective
                    seen.add(a)


def test_record_layout_and_op_tables(capi, orc):
    """IdxVal<I,T> repr(C) sizes; BatchReturnType per op; op availability per (kind, T)."""
    for iw in (1, 2, 4, 8):
        for d in range(10):
            assert capi.lmr_record_bytes(iw, d) == orc.record_bytes(iw, d)
            assert capi.lmr_record_val_offset(iw, d) == orc.record_val_offset(iw, d)
    # IdxVal<u32,u64> = 16 B (4 idx + 4 pad + 8 val), IdxVal<u32,u32> = 8 B
    assert capi.lmr_record_bytes(4, 3) == 16 and capi.lmr_record_bytes(4, 2) == 8
    assert capi.lmr_record_bytes(1, 3) == 16 and capi.lmr_record_bytes(2, 0) == 4
    for op in range(27):
        assert capi.lmr_op_ret_kind(op) == orc.lib().orc_op_ret_kind(op)
        for kind in range(6):
            for d in range(10):
                assert bool(capi.lmr_op_supported(kind, d, op)) == bool(orc.lib().orc_op_supported(kind, d, op))


def test_python_op_table_matches_abi(capi, lam):
    from lamellar_runtime_amd.types import DTYPES, RET_KIND, ArrayOpCmd, op_supported
    for op in ArrayOpCmd:
        assert int(RET_KIND[op]) == capi.lmr_op_ret_kind(int(op))
        for name in ("u8", "i64", "f32", "f64"):
            for kind in range(6):
                assert op_supported(kind, DTYPES[name], op) == bool(capi.lmr_op_supported(kind, DTYPES[name].code, int(op)))


def test_device_path_fails_loudly_without_gpu(lam):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(lam.LamellarError):
        lam.LamellarWorldBuilder().build()


def test_pack_oracle_buffers_respect_am_threshold(orc):
    """The reference's op buffers hold ceil(100000 / sizeof(IdxVal)) records at most
    (unsafe/operations.rs:679-681): 6250 x 16 B for (u32, u64)."""
    L = orc.layout_new(1 << 20, 4, 0, 0)
    rng = np.random.default_rng(0)
    g = rng.integers(0, 1 << 20, 50000).astype(np.uint64)
    v = rng.integers(0, 1000, 50000).astype(np.uint64)
    st, ams = orc.pack(L, 3, np.uint64, g, v, 4, threshold=100000, threads=1)
    assert st == 0
    assert max(a[1].size for a in ams) == 6250 * 16
    assert sum(a[2].size for a in ams) == 50000
    L1 = orc.layout_new(1 << 20, 1, 0, 0)
    st, ams = orc.pack(L1, 3, np.uint64, g, None, 4, threshold=100000, threads=1)
    assert max(a[1].size for a in ams) == 25000 * 4      # SVMI: 25000 u32 indices (:488-489)


def test_host_unregister_refuses_unknown_ranges(capi):
    """lmr_host_unregister only takes the start of a range lmr_host_register registered (a
    pointer inside a registered range makes hipHostUnregister abort the process,
    tools/hostreg_probe.cpp scenario E): anything else is LMR_E_INVALID, decided by the
    library's registry before any runtime call (no GPU needed)."""
    buf = np.zeros(4096, np.uint8)
    assert capi.lmr_host_unregister(ctypes.c_void_p(buf.ctypes.data)) == 1
    assert capi.lmr_host_unregister(ctypes.c_void_p(buf.ctypes.data + 64)) == 1
    assert capi.lmr_host_unregister(None) == 1
