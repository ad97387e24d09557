"""Probe: device vs oracle (x86 gcc -O2) results for every pair of special fp values.

Prints, per (dtype, op), how many special-value pairs differ bitwise and a few
examples.  Used to pin the NaN-propagation rules the kernels must reproduce.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from sos_amd import _lib as L  # noqa: E402


def specials(ft):
    it = np.uint32 if ft == np.float32 else np.uint64
    bits = [0x7FC00000, 0xFFC00000, 0x7FC00123, 0x7F800001, 0xFF800123] if ft == np.float32 else \
        [0x7FF8000000000000, 0xFFF8000000000000, 0x7FF8000000000123, 0x7FF0000000000001,
         0xFFF0000000000123]
    nans = list(np.array(bits, dtype=it).view(ft))
    vals = [0.0, -0.0, np.inf, -np.inf, 1.0, -2.5, np.finfo(ft).tiny / 4, np.finfo(ft).max]
    return np.array(nans + [ft(v) for v in vals], dtype=ft)


def run(dt, op, a, b):
    ref = a.copy()
    O.reduce_local(op, dt, b, ref)
    da = torch.from_numpy(a.view(np.uint8).copy()).cuda()
    db = torch.from_numpy(b.view(np.uint8).copy()).cuda()
    L.combine(op, dt, da.data_ptr(), db.data_ptr(), a.size)
    torch.cuda.synchronize()
    got = da.cpu().numpy().view(a.dtype)
    return got, ref


def main():
    for ft, dt, cdt in ((np.float32, 23, 26), (np.float64, 24, 27)):
        s = specials(ft)
        A, B = np.meshgrid(s, s, indexing="ij")
        a, b = A.reshape(-1).copy(), B.reshape(-1).copy()
        ib = np.uint32 if ft == np.float32 else np.uint64
        for op in (3, 4, 5, 6):
            got, ref = run(dt, op, a, b)
            bad = np.nonzero(got.view(ib) != ref.view(ib))[0]
            print(f"real dt={dt} op={op}: {bad.size} of {a.size} differ")
            for k in bad[:6]:
                print(f"   a={a.view(ib)[k]:#x} b={b.view(ib)[k]:#x} gpu={got.view(ib)[k]:#x} x86={ref.view(ib)[k]:#x}")
        # complex: all combinations of (re, im) specials for a short list
        sc = s[[0, 1, 2, 5, 6, 7, 9, 10]]
        grid = np.array(np.meshgrid(sc, sc, sc, sc, indexing="ij")).reshape(4, -1).T.copy()
        ca = grid[:, :2].copy().reshape(-1).view(O.np_type(cdt))
        cb = grid[:, 2:].copy().reshape(-1).view(O.np_type(cdt))
        for op in (5, 6):
            got, ref = run(cdt, op, ca, cb)
            gb, rb = got.view(ib).reshape(-1, 2), ref.view(ib).reshape(-1, 2)
            bad = np.nonzero((gb != rb).any(1))[0]
            print(f"cplx dt={cdt} op={op}: {bad.size} of {ca.size} differ")
            av, bv = ca.view(ib).reshape(-1, 2), cb.view(ib).reshape(-1, 2)
            for k in bad[:6]:
                print(f"   a=({av[k,0]:#x},{av[k,1]:#x}) b=({bv[k,0]:#x},{bv[k,1]:#x}) "
                      f"gpu=({gb[k,0]:#x},{gb[k,1]:#x}) x86=({rb[k,0]:#x},{rb[k,1]:#x})")


if __name__ == "__main__":
    main()
