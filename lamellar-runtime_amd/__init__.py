"""lamellar_runtime_amd — MI355X-native LamellarArray batched element-op path.

A drop-in for pnnl/lamellar-runtime's batched array-op path
(src/array/unsafe/operations.rs pack + impl/src/array_ops.rs apply): op
records are packed, exchanged (RCCL all-to-all over xGMI) and scatter-applied
by hand-written gfx950 HIP kernels in liblamellar_gpu_ops.so, behind the C ABI
of include/lamellar_gpu_ops.h. This package is the host-side mirror of the
reference's op-builder API over that ABI.

The directory is `lamellar-runtime_amd/`; import it as `lamellar_runtime_amd`
after `load_package()` (see _lamellar_bootstrap.py at the repo root) — tests, bench.py and
__graft_entry__.py do this.
"""
from .types import (ArrayKind, ArrayOpCmd, BatchReturnType, Distribution, LmrStatus, Strategy,
                    DTYPES, dtype_of)
from .kernels import LamellarError, DeviceKernels
from .world import LamellarWorld, LamellarWorldBuilder, LamellarTeam
from .array import (AtomicArray, Err, GlobalLockArray, LocalLockArray, Ok, ReadOnlyArray,
                    UnsafeArray)
from .engine import BatchResult, Owned, run_batch

__all__ = [
    "ArrayKind", "ArrayOpCmd", "BatchReturnType", "Distribution", "LmrStatus", "Strategy",
    "DTYPES", "dtype_of", "LamellarError", "DeviceKernels", "LamellarWorld",
    "LamellarWorldBuilder", "LamellarTeam", "AtomicArray", "Err", "GlobalLockArray",
    "LocalLockArray", "Ok", "ReadOnlyArray", "UnsafeArray", "BatchResult", "Owned", "run_batch",
]
