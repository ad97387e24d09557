"""Small-message team-reduction latency per schedule (run under tools/oshrun).

Every PE times `reps` back-to-back shmem_float_sum_reduce(SHMEM_TEAM_WORLD) calls on
device-heap buffers for each schedule and size; PE 0 prints microseconds per call
(the calls are collective, so PE 0's time is the team's).  Used to compare recdbl_sw's
log2(P)-round butterfly with its one-round gather form (SOSX_ALG_RECDBL_GATHER), and the
p2p transport's signalling modes (SHMEMX_P2P_SIGNAL=stream|host) from 4 B to 4 MiB.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402,F401

from sos_amd import _lib as L  # noqa: E402
from sos_amd import shmem as S  # noqa: E402


def main():
    S.shmem_init()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    sizes = [1, 64, 1024, 4095]
    ring_sizes = [16384, 262144, 1 << 20]
    nmax = max(ring_sizes)
    src = S.shmemx_malloc_device(nmax * 4)
    dst = S.shmemx_malloc_device(nmax * 4)
    L.fill(23, 0, 7, me, src, nmax)
    team = S.team_world()
    reps = int(os.environ.get("LAT_REPS", "200"))
    for alg, ns in (("recdbl", sizes), ("recdbl_gather", sizes), ("ring", ring_sizes)):
        S.shmemx_set_reduce_algorithm(L.ALGS[alg])
        for n in ns:
            for _ in range(10):
                S.shmem_float_sum_reduce(team, dst, src, n)
            S.shmem_barrier_all()
            t0 = time.perf_counter()
            for _ in range(reps):
                S.shmem_float_sum_reduce(team, dst, src, n)
            t = (time.perf_counter() - t0) / reps
            if me == 0:
                print(f"P={P} {alg:14s} n={n:7d}: {t * 1e6:8.1f} us/call", flush=True)
    S.shmem_barrier_all()
    S.shmemx_free_device(dst)
    S.shmemx_free_device(src)
    S.shmem_finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
