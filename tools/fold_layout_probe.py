"""Does the spacing of the fold's scratch slots change its HBM rate?  (Bench only.)

Inside the 8-PE ring the fold k_fold<8> reads the PE's own source chunk (the caller's
buffer), 7 peer chunks that the exchange put into the library's scratch slots (plan.cpp:
slot k at k * stride, stride = chunk bytes + 16 rounded up to 256 B), and writes the
caller's target chunk.  rocprof shows its per-launch time spread 93-110 us across the 8
PEs of one run (profiles/r3final_loopback8_ring_kernel_stats.csv): some layouts stream
at the combine's rate, some do not.  This probe times the fold with the 7 scratch inputs
at stride = chunk + pad for a set of pads (own source and output in allocations of
their own, shifted by a few pages), median over rounds, and prints one JSON line.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PADS = [16, 256, 1024, 4096, 4096 + 256, 16384, 65536, 65536 + 4096, 1 << 20, (2 << 20) + 4096]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128 << 20, help="elements of the whole vector")
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from sos_amd import _lib as L
    torch.cuda.set_device(0)
    dt, es, P = L.dtype_id("float"), 4, a.P
    chunk = a.n // P
    cb = chunk * es
    algo = (P + 1) * cb
    maxpad = max(PADS)
    scratch = torch.empty((P - 1) * (cb + maxpad) + 4096, dtype=torch.uint8, device="cuda")
    own_raw = torch.empty(cb + 64 * 4096, dtype=torch.uint8, device="cuda")
    out_raw = torch.empty(cb + 64 * 4096, dtype=torch.uint8, device="cuda")
    L.fill(dt, 0, 0x5EED, 0, scratch.data_ptr(), scratch.numel() // es)
    L.fill(dt, 0, 0x5EED, 1, own_raw.data_ptr(), own_raw.numel() // es)
    torch.cuda.synchronize()

    def timed(ins, out):
        for _ in range(3):
            L.fold("sum", dt, L.ORDER_LINEAR, out, ins, chunk)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(a.reps):
            L.fold("sum", dt, L.ORDER_LINEAR, out, ins, chunk)
        s1.record()
        torch.cuda.synchronize()
        return s0.elapsed_time(s1) / a.reps / 1e3

    res = {}
    for r in range(a.rounds):
        own = own_raw.data_ptr() + (r * 7 % 64) * 4096
        out = out_raw.data_ptr() + (r * 13 % 64) * 4096
        for pad in PADS:
            base = scratch.data_ptr()
            ins = [own] + [base + k * (cb + pad) for k in range(P - 1)]
            t = timed(ins, out)
            res.setdefault(pad, []).append(algo / t / 1e12)
    rows = {str(p): {"median_TBs": round(statistics.median(v), 3), "min": round(min(v), 3),
                     "max": round(max(v), 3)} for p, v in res.items()}
    print(json.dumps({"kernel": f"k_fold<{P}> float sum", "chunk_elems": chunk,
                      "algorithmic_bytes": algo, "by_scratch_pad_bytes": rows}), flush=True)


if __name__ == "__main__":
    main()
