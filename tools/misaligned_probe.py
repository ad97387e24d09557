"""Bench-only probe: the local combine (sosx_combine, inout = inout OP in) when the two
operands are NOT 16-B congruent (in starts `off` bytes past a 16-B boundary, inout on
one), against the same call on congruent operands.  SOS's reduce_local takes any element
alignment (src/shmem_internal_op.h:305-339); a caller reducing into a sub-array hits this.

Usage: python tools/misaligned_probe.py [--bytes 536870912] [--reps 20]
Prints one JSON line: {type/offset: {"ms", "GBs", "frac"}}.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=512 << 20)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from sos_amd import _lib as L
    torch.cuda.set_device(0)
    S = torch.cuda.current_stream()
    st = S.cuda_stream
    nb = a.bytes
    x = torch.empty(nb + 4096, dtype=torch.uint8, device="cuda")
    y = torch.empty(nb + 4096 + (1 << 20), dtype=torch.uint8, device="cuda")
    xa = (x.data_ptr() + 4095) & ~4095
    ya = ((y.data_ptr() + (1 << 20) - 1) & ~((1 << 20) - 1)) + 4096  # 4 KiB colour apart
    out = {}
    for tname, offs in (("float", (0, 4, 8)), ("double", (0, 8)), ("uchar", (0, 1, 3)),
                        ("short", (0, 2)), ("complexd", (0,))):
        dt = L.dtype_id(tname)
        es = L.dtype_size(dt)
        n = (nb - 64) // es
        op = L.op_id("sum")
        for off in offs:
            b = ya + off
            L.fill(dt, 0, 0x5EED, 0, xa, n, 0, st)
            L.fill(dt, 0, 0x5EED, 1, b, n, 0, st)
            for _ in range(3):
                L.combine(op, dt, xa, b, n, st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(S)
            for _ in range(a.reps):
                L.combine(op, dt, xa, b, n, st)
            e1.record(S)
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 1e3 / a.reps
            gbs = 3 * n * es / t / 1e9
            out[f"{tname}/+{off}"] = {"ms": round(t * 1e3, 4), "GBs": round(gbs, 1), "frac": round(gbs / 8000, 4)}
            print(f"{tname:>9} +{off}: {t * 1e3:.4f} ms {gbs:8.1f} GB/s", file=sys.stderr, flush=True)
    print(json.dumps(out))


def fold(args):
    """The 8-input LINEAR fold (sosx_fold, the ring's local step) over 16Mi fp32 per input:
    all inputs congruent with the output, input 0 (the PE's own source chunk) at +4 bytes,
    and every input at +4 / +8 / +12 (peers' sources read in place, target elsewhere:
    k_fold_outshift, or k_fold_realign under SOSX_FOLD_OUTSHIFT=0)."""
    import torch
    from sos_amd import _lib as L
    torch.cuda.set_device(0)
    S = torch.cuda.current_stream()
    st = S.cuda_stream
    P, n, es = args.np, 16 << 20, 4
    nb = n * es
    bufs = [torch.empty(nb + (1 << 20), dtype=torch.uint8, device="cuda") for _ in range(P + 1)]
    # page-aligned, 4 KiB colours apart (as the device heap places them); 1 MiB of slack
    base = [((b.data_ptr() + 4095) & ~4095) + 4096 * (k % 8) for k, b in enumerate(bufs)]
    out = {}
    for name, offs in (("congruent", [0] * P), ("input0+4", [4] + [0] * (P - 1)), ("all+4", [4] * P), ("all+8", [8] * P), ("all+12", [12] * P),
                        ("mixed", [(4 * (k + 1)) % 16 for k in range(P)])):
        if args.only and name not in args.only.split(","):
            continue
        ins = [base[k] + offs[k] for k in range(P)]
        for k in range(P):
            L.fill(23, 0, 0x5EED, k, ins[k], n, 0, st)
        launch = lambda: L.fold(5, 23, 0, base[P], ins, n, st)  # noqa: E731
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
        gbs = (P + 1) * nb / t / 1e9
        out[name] = {"ms": round(t * 1e3, 4), "GBs": round(gbs, 1), "frac": round(gbs / 8000, 4)}
        print(f"fold {name:>10}: {t * 1e3:.4f} ms {gbs:8.1f} GB/s", file=sys.stderr, flush=True)
    print(json.dumps(out))


def prefix(args):
    """The 8-input SUM prefix (sosx_prefix, the team scan's local step) over 16Mi fp32 per
    input, outputs congruent with one another: inputs congruent, input 0 at +4 bytes, every
    input at +4, each input at its own offset (k_prefix_realign_np, or the runtime-P
    k_prefix_realign under SOSX_PREFIX_REALIGN=0).  GB/s = 2 x 8 x 64 MiB / time."""
    import torch
    from sos_amd import _lib as L
    torch.cuda.set_device(0)
    S = torch.cuda.current_stream()
    st = S.cuda_stream
    P, n, es = args.np, 16 << 20, 4
    nb = n * es
    bufs = [torch.empty(nb + (1 << 20), dtype=torch.uint8, device="cuda") for _ in range(2 * P)]
    base = [((b.data_ptr() + 4095) & ~4095) + 4096 * (k % 8) for k, b in enumerate(bufs)]
    outs = base[P:]
    out = {}
    for name, offs in (("congruent", [0] * P), ("input0+4", [4] + [0] * (P - 1)), ("all+4", [4] * P),
                       ("all+8", [8] * P), ("mixed", [(4 * (k + 1)) % 16 for k in range(P)])):
        if args.only and name not in args.only.split(","):
            continue
        ins = [base[k] + offs[k] for k in range(P)]
        for k in range(P):
            L.fill(23, 0, 0x5EED, k, ins[k], n, 0, st)
        launch = lambda: L.prefix(5, 23, outs, ins, n, stream=st)  # noqa: E731
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
        gbs = 2 * P * nb / t / 1e9
        out[name] = {"ms": round(t * 1e3, 4), "GBs": round(gbs, 1), "frac": round(gbs / 8000, 4)}
        print(f"prefix {name:>10}: {t * 1e3:.4f} ms {gbs:8.1f} GB/s", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__" and "--prefix" in sys.argv:
    sys.argv.remove("--prefix")
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated layouts (default: all)")
    ap.add_argument("--np", type=int, default=8, help="inputs (1..8)")
    prefix(ap.parse_args())
    sys.exit(0)


if __name__ == "__main__" and "--fold" in sys.argv:
    sys.argv.remove("--fold")
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated layouts (default: all)")
    ap.add_argument("--np", type=int, default=8, help="inputs (2..8)")
    fold(ap.parse_args())
    sys.exit(0)


if __name__ == "__main__":
    main()
