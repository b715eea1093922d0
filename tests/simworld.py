"""A CPU stand-in of N PEs built on the oracle (test-only).

`SimArray` gives the oracle the shape of the reference's tests: every PE's
shard is a numpy array, ops are issued "by PE p" and applied with the
reference's sequential semantics through orc_batch_op.
"""
import numpy as np

from opgen import CODE, NP

KINDS = {"UnsafeArray": 0, "AtomicArray": None, "LocalLockArray": 3, "GlobalLockArray": 4}


class SimArray:
    def __init__(self, orc, num_pes, length, dist, dt, array_type="AtomicArray"):
        self.orc, self.num_pes, self.dt = orc, num_pes, dt
        self.np = NP[dt]
        self.L = orc.layout_new(length, num_pes, 0, dist)
        root = self.L if not self.L.sub else orc.layout_new(max(length, num_pes), num_pes, 0, dist)
        self.shards = [np.zeros(orc.num_elems_pe(root, p), dtype=self.np) for p in range(num_pes)]
        k = KINDS[array_type]
        self.kind = (2 if dt.startswith("f") else 1) if k is None else k

    def sub_array(self, start, end):
        s = object.__new__(SimArray)
        s.__dict__.update(self.__dict__)
        s.L = self.orc.layout_sub(self.L, start, end)
        return s

    def len(self):
        return int(self.L.size)

    def slices(self):
        out = []
        for p in range(self.num_pes):
            st = self.orc.local_slice_start(self.L, p)
            n = self.orc.num_elems_pe(self.L, p)
            out.append(self.shards[p][st:st + max(n, 0)])
        return out

    def fill(self, v):
        for s in self.slices():
            s[:] = np.array([v]).astype(self.np)[0]

    def op(self, op, idx, vals, current=None, eps=None):
        idx = np.atleast_1d(np.asarray(idx, dtype=np.uint64))
        vals = np.atleast_1d(np.asarray(vals).astype(self.np))
        sl = self.slices()
        st, res, ok = self.orc.batch_op(self.L, sl, self.kind, CODE[self.dt], self.np, op, idx, vals,
                                        current, eps)
        return st, res, ok

    def to_numpy(self):
        out = np.empty(self.len(), dtype=self.np)
        sl = self.slices()
        for i in range(self.len()):
            pe, off = self.orc.pe_and_offset(self.L, i)
            out[i] = sl[pe][off]
        return out
