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
    ap.add_argument("--rotate", action="store_true",
                    help="rotate over operand pairs totalling >= 1 GiB, so every launch streams "
                         "from HBM (small sizes otherwise stay in the 256 MiB Infinity Cache)")
    ap.add_argument("--heap", action="store_true",
                    help="operands from the device symmetric heap (shmemx_malloc_device, the "
                         "bench's placement: consecutive large buffers 4 KiB colours apart)")
    ap.add_argument("--only", default="", help="comma-separated variant indices (default: all)")
    a = ap.parse_args()
    import torch
    import variants as V
    from sos_amd import _lib as L
    torch.cuda.set_device(0)
    n, es = a.nreduce, 4
    npairs = max(1, -(-(1 << 30) // (2 * n * es))) if a.rotate else 1
    pairs = []
    if a.heap:
        from sos_amd import shmem as SH
        os.environ.setdefault("SHMEMX_DEVICE_HEAP_SIZE", str(2 * npairs * n * es + (1 << 30)))
        SH.shmem_init()

    class HeapBuf:  # the two attributes the loop uses
        def __init__(self, nbytes):
            self.p = SH.shmemx_malloc_device(nbytes)

        def data_ptr(self):
            return self.p

    for _ in range(npairs):
        x = HeapBuf(n * es) if a.heap else torch.empty(n * es, dtype=torch.uint8, device="cuda")
        y = HeapBuf(n * es) if a.heap else torch.empty_like(x)
        L.fill("float", L.DIST_UNIFORM, 0x5EED, 0, x.data_ptr(), n)
        L.fill("float", L.DIST_UNIFORM, 0x5EED, 1, y.data_ptr(), n)
        pairs.append((x, y))
    reps = max(a.reps, 2 * npairs)
    names = V.names("combine")
    sel = [int(v) for v in a.only.split(",")] if a.only else list(range(len(names)))
    res = {v: [] for v in sel}
    for _ in range(a.rounds):
        for v in sel:
            for i in range(3):
                x, y = pairs[i % npairs]
                V.combine(v, x.data_ptr(), x.data_ptr(), y.data_ptr(), n)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for i in range(reps):
                x, y = pairs[i % npairs]
                V.combine(v, x.data_ptr(), x.data_ptr(), y.data_ptr(), n)
            e.record()
            torch.cuda.synchronize()
            res[v].append(s.elapsed_time(e) / reps)
    rows = {}
    for v in sel:
        name = names[v]
        ms = sorted(res[v])
        med = ms[len(ms) // 2]
        rows[name] = {"median_ms": round(med, 5), "min_ms": round(ms[0], 5),
                      "GBs": round(3 * n * es / (med / 1e3) / 1e9, 1)}
        print(f"{name:>20} {med:10.4f} ms {rows[name]['GBs']:10.1f} GB/s", file=sys.stderr)
    calib = None
    if not a.heap:
        x, y = pairs[0]
        for _ in range(3):
            y.copy_(x)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            y.copy_(x)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.reps
        calib = round(2 * n * es / (ms / 1e3) / 1e9, 1)
    print(json.dumps({"combine_ab": rows, "nreduce": n, "rounds": a.rounds, "operand_pairs": npairs,
                      "operands": "device heap" if a.heap else "torch", "calib_d2d_copy_GBs": calib}))


if __name__ == "__main__":
    main()
