"""bench.py's algorithmic bytes per op of each kernel stage (DESIGN.md §4's table): the figures
the line's per-stage fractions divide by. C2 at N = 1 (u64 global indices, 2^28 records into a
2^26-element shard), C3 on the wide path, and the input-set rule."""
import importlib.util
import os
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_c2_stage_bytes():
    b = _bench()
    n, L = 1 << 28, 1 << 26
    assert b.stage_bytes_per_op("bin_scatter", 8, 8, 8, n, L, False) == 28       # 16 in, 12 out
    assert b.stage_bytes_per_op("fine_scatter", 8, 8, 8, n, L, False) == 22      # 12 in, 10 out
    assert b.stage_bytes_per_op("tile_apply", 8, 8, 8, n, L, False) == 14        # 10 in + shard r/w / 4
    assert b.stage_bytes_per_op("unpartition", 8, 8, 8, n, L, False) == 0        # nothing returned


def test_c3_wide_stage_bytes():
    b = _bench()
    n, L = 1 << 26, 1 << 24
    w = dict(wide=True)
    assert b.stage_bytes_per_op("bin_count", 8, 8, 8, n, L, True, **w) == 8
    assert b.stage_bytes_per_op("bin_scatter", 8, 8, 8, n, L, True, **w) == 28   # + u16 offset, u16 position
    assert b.stage_bytes_per_op("tile_apply", 8, 8, 8, n, L, True, **w) == 2 + 8 + 8 + 4
    assert b.stage_bytes_per_op("unpartition", 8, 8, 8, n, L, True, **w) == 18   # position + old in, old out


def test_input_sets_cap():
    b = _bench()
    a = types.SimpleNamespace(input_sets=0)
    assert b.input_sets(a, 1 << 30, 1 << 28) == 4
    assert b.input_sets(a, 1 << 30, 1 << 26) == 16
    assert b.input_sets(a, 1 << 30, 1 << 20) == 16
    assert b.input_sets(types.SimpleNamespace(input_sets=3), 1 << 30, 1 << 28) == 3
