"""Stress of freshly allocated device memory under allocation churn from several processes
("Open (round 4)": the one wrong 12-PE result came from the first
call after the PE's exchange scratch had grown, i.e. from a fresh hipMalloc).

Per iteration, in each of P concurrent processes: return torch's cached blocks to the
driver (torch.cuda.empty_cache), allocate a fresh buffer of 16-64 MiB, write a seeded
pattern into it with one kernel (sosx_fill), and compare it with a second kernel against
the same pattern in a long-lived buffer (sosx_count_mismatch); every count must be 0.  A
non-zero count means a fresh allocation lost or reverted part of a completed kernel's
writes (an asynchronous clear of recycled memory racing with the first user writes),
which no library ordering can prevent.

Usage: tools/oshrun -np 12 python tools/fresh_alloc_stress.py [--iters 200]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from sos_amd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    me = int(os.environ.get("SHMEM_PE", "0"))
    torch.cuda.set_device(0)
    dt = L.dtype_id("float")
    nmax = 16 << 20                                  # ref holds the largest n
    ref = torch.empty(nmax * 4, dtype=torch.uint8, device="cuda")
    bad = []
    for it in range(a.iters):
        n = (4 << 20) * (1 + (it + me) % 4) - 5        # 16-64 MiB (<= nmax), varying per process
        assert n <= nmax
        seed = 0xF2E500 + 1000 * me + it
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        buf = torch.empty(n * 4, dtype=torch.uint8, device="cuda")
        L.fill(dt, 0, seed, me, buf.data_ptr(), n)
        L.fill(dt, 0, seed, me, ref.data_ptr(), n)
        mm = L.count_mismatch(ref.data_ptr(), buf.data_ptr(), n, 4)
        if mm:
            torch.cuda.synchronize()
            again = L.count_mismatch(ref.data_ptr(), buf.data_ptr(), n, 4)
            bad.append({"iter": it, "n": n, "count": int(mm), "recount": int(again)})
        del buf
    if bad:
        print(f"proc {me}: {len(bad)} of {a.iters} fresh buffers wrong: {bad[:4]}", flush=True)
        return 1
    print(f"proc {me}: {a.iters} fresh buffers OK", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
