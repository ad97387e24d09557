"""Interleaved A/B of the local-combine kernel shapes (bench-only library tools/variants/)
against the product default, on one GPU: nreduce fp32 sum, `--rounds` rounds of every
shape back to back in one process (guide rule: interleave, never compare across
processes), plus the HIP runtime's device-to-device copy of the same bytes as a
calibration line.  Shape 0 is the product default (sos::k_combine3 U=1 nontemporal).

Usage: python tools/variants_bench.py [--nreduce N] [--rounds R]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(HERE, "variants"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nreduce", type=int, default=128 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import variants as V
    from sos_amd import _lib as L
    torch.cuda.set_device(0)
    n, es = a.nreduce, 4
    x = torch.empty(n * es, dtype=torch.uint8, device="cuda")
    y = torch.empty_like(x)
    L.fill("float", L.DIST_UNIFORM, 0x5EED, 0, x.data_ptr(), n)
    L.fill("float", L.DIST_UNIFORM, 0x5EED, 1, y.data_ptr(), n)
    names = V.names("combine")
    res = {v: [] for v in range(len(names))}
    for _ in range(a.rounds):
        for v in range(len(names)):
            for _ in range(3):
                V.combine(v, x.data_ptr(), x.data_ptr(), y.data_ptr(), n)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.reps):
                V.combine(v, x.data_ptr(), x.data_ptr(), y.data_ptr(), n)
            e.record()
            torch.cuda.synchronize()
            res[v].append(s.elapsed_time(e) / a.reps)
    rows = {}
    for v, name in enumerate(names):
        ms = sorted(res[v])
        med = ms[len(ms) // 2]
        rows[name] = {"median_ms": round(med, 5), "min_ms": round(ms[0], 5),
                      "GBs": round(3 * n * es / (med / 1e3) / 1e9, 1)}
        print(f"{name:>20} {med:10.4f} ms {rows[name]['GBs']:10.1f} GB/s", file=sys.stderr)
    for _ in range(3):
        y.copy_(x)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.reps):
        y.copy_(x)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.reps
    print(json.dumps({"combine_ab": rows, "nreduce": n, "rounds": a.rounds,
                      "calib_d2d_copy_GBs": round(2 * n * es / (ms / 1e3) / 1e9, 1)}))


if __name__ == "__main__":
    main()
