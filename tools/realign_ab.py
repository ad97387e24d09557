"""A/B of the realigning 8-input fold shapes (tools/variants: sosxv_fold_realign), VERDICT r5
item 6: 16Mi fp32 per input, every input at its own 16-B offset ("mixed": input k at
4(k+1) mod 16 bytes, 6 of 8 incongruent) and every input at +4; the product's sosx_fold
beside them.  Rounds interleave the shapes; each shape's output is compared bit for bit
with the product's.  Prints one line per shape and round, then a JSON summary.

  python tools/realign_ab.py [--rounds 3] [--reps 20] [--only 0,3]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = {0: "two nt loads (round 5)", 1: "nt + plain second load", 2: "two plain loads",
         3: "nt + DPP wave_shl:1", 4: "nt + __shfl_down", 5: "plain incongruent, 2 loads",
         6: "plain + DPP", 7: "plain incongruent + DPP", 8: "DPP + LDS across waves"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated shapes (default: all)")
    ap.add_argument("--layouts", default="mixed,all+4")
    args = ap.parse_args()
    import torch
    from sos_amd import _lib as L
    V = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", "libsos_variants.so"))
    V.sosxv_fold_realign.restype = ctypes.c_int
    V.sosxv_fold_realign.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                     ctypes.c_size_t, ctypes.c_void_p]
    torch.cuda.set_device(0)
    S = torch.cuda.current_stream()
    st = S.cuda_stream
    P, n, es = 8, 16 << 20, 4
    nb = n * es
    bufs = [torch.empty(nb + (1 << 20), dtype=torch.uint8, device="cuda") for _ in range(P + 2)]
    base = [((b.data_ptr() + 4095) & ~4095) + 4096 * (k % 8) for k, b in enumerate(bufs)]
    out, ref = base[P], base[P + 1]
    modes = [int(m) for m in args.only.split(",")] if args.only else sorted(NAMES)
    layouts = {"mixed": [(4 * (k + 1)) % 16 for k in range(P)], "all+4": [4] * P,
               "input0+4": [4] + [0] * (P - 1), "two+4": [4, 0, 0, 0, 4, 0, 0, 0]}
    for m in range(1, P + 1):  # m<k>: inputs 0..k-1 at 4, 8, 12, 4, ... bytes, the rest congruent
        layouts[f"m{m}"] = [4 * (j % 3 + 1) if j < m else 0 for j in range(P)]
    res = {}
    for lay in args.layouts.split(","):
        offs = layouts[lay]
        ins = [base[k] + offs[k] for k in range(P)]
        for k in range(P):
            L.fill(23, 0, 0x5EED, k, ins[k], n, 0, st)
        arr = (ctypes.c_void_p * P)(*ins)
        L.fold(5, 23, 0, ref, ins, n, st)
        torch.cuda.synchronize()
        launches = {"product": lambda: L.fold(5, 23, 0, out, ins, n, st)}
        for m in modes:
            launches[m] = (lambda m=m: L.check(V.sosxv_fold_realign(m, out, arr, n, st), "sosxv_fold_realign"))
        times = {k: [] for k in launches}
        for r in range(args.rounds):
            for k, launch in launches.items():
                for _ in range(3):
                    launch()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(S)
                for _ in range(args.reps):
                    launch()
                e1.record(S)
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / 1e3 / args.reps
                times[k].append(round((P + 1) * nb / t / 1e9, 1))
                mm = ctypes.c_ulonglong()
                L.check(L.lib().sosx_count_mismatch(out, ref, n, 4, ctypes.byref(mm), st), "mismatch")
                tag = NAMES.get(k, k) if k != "product" else "product sosx_fold"
                print(f"{lay:>6} round {r} {tag:>24}: {times[k][-1]:8.1f} GB/s  mismatches {mm.value}",
                      file=sys.stderr, flush=True)
                if mm.value:
                    raise SystemExit(f"{lay} shape {k}: {mm.value} elements differ from the product")
        res[lay] = {str(k): times[k] for k in times}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
