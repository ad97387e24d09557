"""Run under tools/oshrun with 4 PEs (p2p transport, stream-ordered signalling): one
4-round call (rechalving: 2 reduce-scatter + 2 allgather rounds, so three DEVICE
signalling steps after the host entry boundary) in which PE 1 stops right after the
entry boundary (SOSX_P2P_TEST_STALL_PE=1).  The other PEs' device waits time out after
SHMEMX_P2P_TIMEOUT; the later steps of the same call must not wait again, so the job
ends about one timeout after the call starts (tests/test_gpu_multipe.py)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402,F401

from sos_amd import _lib as L  # noqa: E402
from sos_amd import shmem as S  # noqa: E402


def main():
    S.shmem_init()
    me = S.shmem_my_pe()
    n = 1 << 16
    src = S.shmemx_malloc_device(n * 4)
    dst = S.shmemx_malloc_device(n * 4)
    S.shmemx_set_reduce_algorithm(L.ALGS["rechalving"])
    S.shmem_barrier_all()
    print(f"PE {me}: call starts at {time.time():.3f}", flush=True)
    S.shmem_float_sum_reduce(S.team_world(), dst, src, n)
    print(f"PE {me}: reduction returned", flush=True)
    S.shmem_finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
