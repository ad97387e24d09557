"""Stress of the tests' CHECK path, not the library ("Open (round 4)").

team_check_pe.py builds each expected vector on the CPU, copies it to the GPU with
torch (`torch.from_numpy(...).cuda()`, a pageable H2D into a block the caching allocator
hands out again and again) and compares it with the library's target in a kernel
(`sosx_count_mismatch`).  This tool repeats exactly that pattern with no library
collective in the loop: per iteration a fresh CPU vector (oracle_fill), its torch H2D
copy, and the same vector generated on the GPU (sosx_fill, bit-identical by
construction); every count must be 0.  Run as P concurrent processes on one GPU (under
tools/oshrun, which only sets the environment here) to load the device as the 12-PE
team_check does.  A non-zero count, and whether a recount and a CPU-side comparison
agree with it, says whether the check path itself can read stale bytes.

Usage: tools/oshrun -np 12 python tools/check_path_stress.py [--iters 300] [--n 1048579]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from sos_amd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--n", type=int, default=(1 << 20) + 3)
    a = ap.parse_args()
    me = int(os.environ.get("SHMEM_PE", "0"))
    torch.cuda.set_device(0)
    dt = L.dtype_id("float")
    n = a.n
    dev = torch.empty(n * 4, dtype=torch.uint8, device="cuda")
    bad = []
    for it in range(a.iters):
        seed = 0xC0DE00 + 1000 * me + it
        # the expected vector exactly as team_check_pe.expected() makes it
        host = O.fill(dt, 0, seed, me, n)
        exp = torch.from_numpy(np.frombuffer(host.tobytes(), np.uint8).copy()).cuda()
        L.fill(dt, 0, seed, me, dev.data_ptr(), n)
        mm = L.count_mismatch(exp.data_ptr(), dev.data_ptr(), n, 4)
        if mm:
            torch.cuda.synchronize()
            again = L.count_mismatch(exp.data_ptr(), dev.data_ptr(), n, 4)
            cpu = int(np.count_nonzero(exp.cpu().numpy() != dev.cpu().numpy()))
            bad.append({"iter": it, "count": int(mm), "recount": int(again), "cpu_bytes_differ": cpu})
        del exp
    if bad:
        print(f"proc {me}: {len(bad)} of {a.iters} counts non-zero: {bad[:4]}", flush=True)
        return 1
    print(f"proc {me}: {a.iters} counts 0", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
