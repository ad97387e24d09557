"""How much the HBM rate of the streaming kernels depends on where the buffers sit.

For each of --layouts rounds, every operand buffer starts a random number of 4 KiB pages
(0..63) into its own allocation; the three kernels are then timed on that layout with HIP
events (torch's current stream, the one they are launched on):

  combine  k_combine3, inout OP= in, n elements                3 streams, 3*n*s bytes
  fold     k_fold<8>,  out = fold of 8 chunks of n/8            9 streams, 9/8*n*s bytes
  prefix   k_prefix<8>, 8 outs from 8 chunks of n/8            16 streams, 2*n*s bytes

Prints one JSON line: per kernel the median, min and max TB/s over layouts.
"""
import argparse
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128 << 20)
    ap.add_argument("--dtype", default="float")
    ap.add_argument("--layouts", type=int, default=12)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from sos_amd import _lib as L
    torch.cuda.set_device(0)
    dt = L.dtype_id(a.dtype)
    es = L.dtype_size(dt)
    P, chunk, pages = 8, a.n // 8, 64
    rng = random.Random(4321)
    res = {"combine": [], "fold": [], "prefix": []}
    algo = {"combine": 3 * a.n * es, "fold": (P + 1) * chunk * es, "prefix": 2 * P * chunk * es}

    def timed(fn):
        for _ in range(3):
            fn()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(a.reps):
            fn()
        s1.record()
        torch.cuda.synchronize()
        return s0.elapsed_time(s1) / a.reps / 1e3

    def bufs(count, elems):
        raw = [torch.empty(elems * es + pages * 4096, dtype=torch.uint8, device="cuda")
               for _ in range(count)]
        return raw, [b.data_ptr() + rng.randrange(pages) * 4096 for b in raw]

    for _ in range(a.layouts):
        raw, (io, x) = bufs(2, a.n)
        L.fill(dt, 0, 0x5EED, 0, io, a.n)
        L.fill(dt, 0, 0x5EED, 1, x, a.n)
        res["combine"].append(timed(lambda: L.combine("sum", dt, io, x, a.n)))
        del raw
        raw, ptrs = bufs(2 * P + 1, chunk)
        ins, outs, fo = ptrs[:P], ptrs[P:2 * P], ptrs[2 * P]
        for k, p in enumerate(ins):
            L.fill(dt, 0, 0x5EED, k, p, chunk)
        res["fold"].append(timed(lambda: L.fold("sum", dt, L.ORDER_LINEAR, fo, ins, chunk)))
        res["prefix"].append(timed(lambda: L.prefix("sum", dt, outs, ins, chunk, -1)))
        del raw
    out = {"n": a.n, "dtype": a.dtype, "layouts": a.layouts}
    for k, v in res.items():
        v = sorted(v)
        tb = lambda s: round(algo[k] / s / 1e12, 3)  # noqa: E731
        out[k] = {"median_TBs": tb(v[len(v) // 2]), "min_TBs": tb(v[-1]), "max_TBs": tb(v[0]),
                  "median_ms": round(v[len(v) // 2] * 1e3, 5)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
