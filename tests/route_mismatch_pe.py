"""Run under tools/oshrun with 2 PEs (tests/test_gpu_multipe.py::test_route_mismatch_*).

The PEs pass operands of different residency to one shmem_float_sum_reduce: PE 0 host
symmetric heap (the small shared-memory path), PE 1 device heap above SHMEMX_SMALL_DEVICE
(the executor).  SOS's schedule choice depends only on the size, so its PEs always agree
(src/shmem_collectives.h:179-200); this build's choice also depends on residency, and a
disagreement must end the job at once with both PEs' operands named, not after
SHMEMX_P2P_TIMEOUT.  Argument `setter`: instead, the PEs pass different limits to the
collective sosx_set_small_device_bytes, which must refuse them."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402,F401

from sos_amd import shmem as S  # noqa: E402


def main():
    S.shmem_init()
    me = S.shmem_my_pe()
    mode = sys.argv[1] if len(sys.argv) > 1 else "residency"
    if mode == "setter":
        S.lib().sosx_set_small_device_bytes(4096 * (me + 1))
        print(f"PE {me}: setter returned", flush=True)
        S.shmem_finalize()
        return 0
    n = 4096  # 16 KiB: host operands take the small path, 2 x 16 KiB device ones do not
    # every PE allocates both kinds (the allocations are collective), then uses its own
    hsrc, hdst = S.lib().shmem_malloc(n * 4), S.lib().shmem_malloc(n * 4)
    dsrc, ddst = S.shmemx_malloc_device(n * 4), S.shmemx_malloc_device(n * 4)
    src, dst = (hsrc, hdst) if me == 0 else (dsrc, ddst)
    S.shmem_barrier_all()
    print(f"PE {me}: call starts at {time.time():.3f}", flush=True)
    S.shmem_float_sum_reduce(S.team_world(), dst, src, n)
    print(f"PE {me}: reduction returned", flush=True)
    S.shmem_finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
