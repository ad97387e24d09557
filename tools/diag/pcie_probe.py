"""Diagnostic: PCIe copy rates from pinned host memory, alone and overlapped.

Per process: H2D alone, D2H alone, H2D || D2H on two streams, for 64 MiB.  Run plain
(one process) or under tools/oshrun -np N to see N processes sharing the card's link.
"""
import os
import sys
import time

import torch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
torch.cuda.set_device(0)
h_in = torch.empty(N, dtype=torch.uint8, pin_memory=True)
h_out = torch.empty(N, dtype=torch.uint8, pin_memory=True)
d_a = torch.empty(N, dtype=torch.uint8, device="cuda")
d_b = torch.empty(N, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def h2d():
    with torch.cuda.stream(s1):
        d_a.copy_(h_in, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h_out.copy_(d_b, non_blocking=True)


def both():
    h2d()
    d2h()


pe = os.environ.get("SHMEM_PE", "0")
for name, fn in (("h2d", h2d), ("d2h", d2h), ("both", both)):
    t = timed(fn)
    print(f"PE {pe} {name}: {t * 1e3:.3f} ms = {N / t / 1e9:.1f} GB/s per direction", flush=True)
