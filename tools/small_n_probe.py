"""Bench-only probe: where the time of a SMALL local combine / fold
goes.  Back-to-back launches on one stream at nreduce = 128Ki and 1Mi fp32 (and 1 element
as the launch floor), operands rotated over >= 1 GiB of device-heap pairs so every
launch streams from HBM; per shape the mean HIP-event time per launch.  Run it under
`rocprofv3 --kernel-trace --stats` to split that into kernel duration and the gap to the
next dispatch (tools/kernel_gaps.py reads the trace).

Shapes: the product's sosx_combine (k_combine3, U = 1) and sosx_fold (8 inputs, k_fold
U = 1), and the bench-only combine shapes U = 2 / U = 4 (tools/variants).

Usage: python tools/small_n_probe.py [--reps 200]
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
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--sizes", default="1,131072,1048576")
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    import torch
    import variants as V
    from sos_amd import _lib as L
    from sos_amd import shmem as SH
    torch.cuda.set_device(0)
    os.environ.setdefault("SHMEMX_DEVICE_HEAP_SIZE", str(3 << 30))
    os.environ.setdefault("SHMEMX_STAGE_BYTES", str(64 << 20))
    SH.shmem_init()
    stream = torch.cuda.Stream()
    S = stream.cuda_stream
    dt, op = L.dtype_id("float"), L.op_id("sum")
    out = {}
    for n in [int(x) for x in a.sizes.split(",")]:
        nb = n * 4
        npairs = max(2, -(-(1 << 30) // (2 * nb))) if n > 1 else 2
        npairs = min(npairs, 2048)
        bufs = [(SH.shmemx_malloc_device(nb), SH.shmemx_malloc_device(nb)) for _ in range(npairs)]
        for x, y in bufs:
            L.fill(dt, 0, 5, 0, x, n, 0, S)
            L.fill(dt, 0, 5, 1, y, n, 0, S)
        fold_n = max(1, n // 8)   # one PE's chunk of an 8-PE ring: 8 inputs of n/8
        shapes = {
            "sosx_combine_u1": lambda x, y: L.combine(op, dt, x, y, n, S),
            "variant_combine_u2": lambda x, y: V.combine(2, x, x, y, n, S),
            "variant_combine_u4": lambda x, y: V.combine(1, x, x, y, n, S),
            "sosx_fold8_u1": lambda x, y: L.fold(op, dt, L.ORDER_LINEAR, x,
                                                 [y + k * fold_n * 4 for k in range(8)], fold_n, S),
        }
        row = {}
        times = {name: [] for name in shapes}
        for rnd in range(a.rounds):      # shapes interleaved, a median over rounds
            for name, fn in shapes.items():
                for i in range(5):
                    fn(*bufs[i % npairs])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(stream)
                for i in range(a.reps):
                    fn(*bufs[(i + rnd) % npairs])
                e1.record(stream)
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) * 1e3 / a.reps)
        for name in shapes:
            us = sorted(times[name])[len(times[name]) // 2]
            algo = 3 * nb if "combine" in name else 9 * fold_n * 4
            row[name] = {"us_per_launch_median": round(us, 3), "us_range": [round(min(times[name]), 3),
                                                                           round(max(times[name]), 3)],
                         "GBs": round(algo / (us * 1e-6) / 1e9, 1)}
            print(f"n={n:>9} {name:>20} {us:8.3f} us {row[name]['GBs']:9.1f} GB/s", file=sys.stderr, flush=True)
        out[str(n)] = row
        for x, y in bufs:
            SH.lib().shmemx_free_device(x)
            SH.lib().shmemx_free_device(y)
    print(json.dumps({"small_n": out, "reps": a.reps, "rounds": a.rounds,
                      "ideal_us_1Mi_combine_at_6p6TBs": round(12 * 2**20 / 6.6e12 * 1e6, 3)}))
    SH.shmem_finalize()


if __name__ == "__main__":
    main()
