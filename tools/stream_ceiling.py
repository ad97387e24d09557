"""Bench-only probe: the HBM stream ceilings of this kernel shape on MI355X.

Read-only, write-only, copy and two-reads-one-write (the combine's shape) streams over
512 MiB per stream, the tile shape of k_combine3 (tools/variants k_stream), operands in
4 KiB-staggered allocations as the device heap places them; the product combine
(sosx_combine) on the same buffers beside them.  GB/s = bytes moved / median time of
`--reps` launches (HIP events), `--rounds` interleaved rounds.  Prints one JSON line:
what fraction of the nominal 8 TB/s each shape reaches, i.e. the practical ceiling the
headline's 0.83 is measured against.
Usage: python tools/stream_ceiling.py [--mib 512] [--reps 20] [--rounds 5] [--multi]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--multi", action="store_true", help="also the fold's and prefix's multi-stream shapes")
    a = ap.parse_args()
    import torch
    from sos_amd import _lib as L
    torch.cuda.set_device(0)
    v = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", "libsos_variants.so"))
    v.sosxv_stream.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                               ctypes.c_void_p]
    nb = a.mib << 20
    big = torch.empty(3 * nb + (64 << 20), dtype=torch.uint8, device="cuda")
    base = (big.data_ptr() + (2 << 20) - 1) & ~((2 << 20) - 1)
    # three streams 4 KiB-coloured apart in HBM's 32 KiB channel interleave
    ptr = [base + k * (nb + (1 << 20)) + 4096 * k for k in range(3)]
    big.fill_(1)
    S = torch.cuda.current_stream()
    st = S.cuda_stream
    nvec = nb // 16
    shapes = {"read-only": (0, nb), "write-only": (1, nb), "copy": (2, 2 * nb), "2 reads + 1 write": (3, 3 * nb)}
    res = {k: [] for k in list(shapes) + ["sosx_combine (fp32 sum)"]}
    for _ in range(a.rounds):
        for name, (kind, moved) in list(shapes.items()) + [("sosx_combine (fp32 sum)", (None, 3 * nb))]:
            if kind is None:
                launch = lambda: L.combine(5, 23, ptr[0], ptr[1], nb // 4, st)  # noqa: E731
            else:
                launch = lambda: v.sosxv_stream(kind, ptr[0], ptr[1], ptr[2], nvec, st)  # noqa: E731
            for _ in range(3):
                launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(S)
            for _ in range(a.reps):
                launch()
            e1.record(S)
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 1e3 / a.reps
            res[name].append(moved / t / 1e9)
    if a.multi:
        # the fold's 9 and the prefix's 16 streams: bare streams (with and without the
        # product's occupancy cap) beside the product kernels, 16Mi fp32 per stream in 17
        # allocations 64 MiB + 4 KiB colour apart (the device heap's placement)
        v.sosxv_fold_fast8.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint,
                                       ctypes.c_void_p]
        v.sosxv_mstream.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint,
                                    ctypes.c_void_p]
        chunk = 16 << 20
        cb = chunk * 4
        mb = torch.empty(17 * (cb + (1 << 20)) + (4 << 20), dtype=torch.uint8, device="cuda")
        mbase = (mb.data_ptr() + (2 << 20) - 1) & ~((2 << 20) - 1)
        mp = [mbase + k * cb + 4096 * (k % 8) for k in range(17)]
        mb.fill_(1)
        ins = (ctypes.c_void_p * 8)(*mp[:8])
        outs = (ctypes.c_void_p * 8)(*mp[8:16])
        one = (ctypes.c_void_p * 8)(*([mp[16]] * 8))
        legs = {"bare 8 reads + 1 write": lambda: v.sosxv_mstream(0, one, ins, cb // 16, 0, st),
                "bare 8 reads + 1 write, 3 per CU": lambda: v.sosxv_mstream(0, one, ins, cb // 16, 48 << 10, st),
                "sosx_fold 8 inputs": lambda: L.fold(5, 23, 0, mp[16], mp[:8], chunk, st),
                "fast-path fold 8 inputs, 3 per CU": lambda: v.sosxv_fold_fast8(mp[16], ins, chunk, 48 << 10, st),
                "bare 8 reads + 8 writes": lambda: v.sosxv_mstream(1, outs, ins, cb // 16, 0, st),
                "bare 8 reads + 8 writes, 2 per CU": lambda: v.sosxv_mstream(1, outs, ins, cb // 16, 64 << 10, st),
                "sosx_prefix 8 inputs": lambda: L.prefix(5, 23, mp[8:16], mp[:8], chunk, -1, st)}
        moved = {k: (9 if "1 write" in k or "fold" in k else 16) * cb for k in legs}
        for k in legs:
            res[k] = []
        for _ in range(a.rounds):
            for name, launch in legs.items():
                for _ in range(3):
                    launch()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(S)
                for _ in range(a.reps):
                    launch()
                e1.record(S)
                torch.cuda.synchronize()
                res[name].append(moved[name] / (e0.elapsed_time(e1) / 1e3 / a.reps) / 1e9)
    out = {k: {"median_GBs": round(statistics.median(x), 1), "frac_of_8TBs": round(statistics.median(x) / 8000, 4),
               "rounds_GBs": [round(y, 1) for y in x]} for k, x in res.items()}
    print(json.dumps({"what": f"HBM stream ceilings, {a.mib} MiB per stream, k_combine3's tile shape", "legs": out}))


if __name__ == "__main__":
    main()
