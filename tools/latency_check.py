"""Small-message team-reduction latency (run under tools/oshrun -np P).

Every PE times `reps` back-to-back shmem_float_sum_reduce(SHMEM_TEAM_WORLD) calls per
schedule and size; PE 0 prints microseconds per call, the max over PEs (the calls are
collective).  Legs:
  dev   : operands in the device symmetric heap (shmemx_malloc_device)
  host  : operands in the host symmetric heap (shmem_malloc: pinned host memory, SOS's
          own case -- the reductions below COLL_SIZE_CROSSOVER that SOS runs on the CPU)
  cpu   : SOS's own CPU recdbl_sw (oracle/sos_oracle.c oracle_pe_recdbl,
          src/collectives.c:850-984), one pinned core per PE, memcpy puts and flag stores
          over a /dev/shm segment (the XPMEM model), on the same P processes, one
          barrier per call (the team API's pSync reuse rule) -- the reference baseline
Schedules: recdbl (recdbl_sw butterfly), recdbl_gather (one all-gather round + every
PE's own tree: AUTO below the crossover), ring (AUTO above it).

--crossover-dev: device-heap operands through the library under AUTO at 4 B .. 1 MiB (run
once with SHMEMX_SMALL_DEVICE=0, the executors, and once with it large, the shared-memory
small path wherever a slot fits): where the small path's limit for device operands lies.

--crossover: host-heap operands through the library under AUTO, and SOS's CPU under its
own AUTO rule (recdbl_sw below SHMEM_COLL_SIZE_CROSSOVER = 16 KiB, ring above,
src/shmem_collectives.h:180-199), from 16 KiB to 16 MiB: where the GPU path starts to
win for SOS's own (host-resident) operands.
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from sos_amd import _lib as L  # noqa: E402
from sos_amd import shmem as S  # noqa: E402

SMALL = [1, 64, 1024, 4095]      # fp32: up to 16380 B, below the 16 KiB crossover
CROSS = [4095, 16384, 65536, 262144, 1 << 20, 1 << 22]   # fp32: 16 KiB .. 16 MiB
CROSS_DEV = [1, 1024, 4095, 16384, 65536, 262144]       # fp32: 4 B .. 1 MiB


def max_over_pes(v, scratch):
    """Max of a float over all PEs, through the library's own double max reduce."""
    a = np.ctypeslib.as_array((ctypes.c_double * 2).from_address(scratch))
    a[0] = v
    S.shmem_double_max_reduce(S.team_world(), scratch + 8, scratch, 1)
    return float(a[1])


def time_calls(fn, reps):
    for _ in range(10):
        fn()
    S.shmem_barrier_all()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def cpu_leg(me, P, reps, scratch, sizes=None):
    """SOS's recdbl_sw on the CPU, one pinned physical core per PE (with `sizes`: SOS's
    AUTO choice per size, recdbl_sw below 16 KiB and ring above, `reps` scaled down for
    large sizes)."""
    from oracle import oracle as O
    allowed = sorted(os.sched_getaffinity(0))
    prim = []
    for c in allowed:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                first = int(f.read().replace("-", ",").split(",")[0])
        except (OSError, ValueError):
            first = c
        if first == c or first not in allowed:
            prim.append(c)
    path = f"/dev/shm/sosx_lat_{os.getppid()}_{P}"
    auto = sizes is not None
    sizes = sizes or SMALL
    nmax = max(sizes)
    if me == 0:
        if os.path.exists(path):
            os.unlink(path)
        ring = O.PeRing(path, P, 0, nmax, 23, create=True, alg="recdbl")
    S.shmem_barrier_all()
    if me != 0:
        ring = O.PeRing(path, P, me, nmax, 23, create=False, alg="recdbl")
    S.shmem_barrier_all()
    if me == 0:
        os.unlink(path)
    src = O.fill(23, 0, 7, me, nmax)
    out = {}
    os.sched_setaffinity(0, {prim[me % len(prim)]})
    try:
        for n in sizes:
            ring.count = n
            if auto:
                ring.alg = PeAlg.RECDBL if n * 4 < 16384 else PeAlg.RING
            r = max(10, min(reps, int(reps * 4096 / max(n, 4096))))
            ring.time(5, src, max(5, r // 10))     # warm-up
            t = ring.time(5, src, r) / r
            out[n] = t
    finally:
        os.sched_setaffinity(0, set(allowed))
    S.shmem_barrier_all()
    ring.close()
    return {n: max_over_pes(t, scratch) for n, t in out.items()}, prim[0]


class PeAlg:
    RING, RECDBL = 0, 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", default="dev,host,cpu")
    ap.add_argument("--reps", type=int, default=int(os.environ.get("LAT_REPS", "200")))
    ap.add_argument("--ring", action="store_true", help="also the ring above the crossover (dev)")
    ap.add_argument("--bcast", action="store_true",
                    help="host-heap shmem_broadcastmem from PE 0 at the small sizes (replaces the legs)")
    ap.add_argument("--crossover-dev", action="store_true",
                    help="device-heap AUTO from 4 B to 1 MiB (replaces the legs)")
    ap.add_argument("--crossover", action="store_true",
                    help="host-heap AUTO vs SOS CPU AUTO from 16 KiB to 16 MiB (replaces the legs)")
    a = ap.parse_args()
    S.shmem_init()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    legs = a.legs.split(",")
    team = S.team_world()
    ring_sizes = [16384, 262144, 1 << 20]
    nmax = max(ring_sizes)
    scratch = S.lib().shmem_malloc(64)
    rows = []
    if a.bcast:
        legs = []
        hs = S.lib().shmem_malloc(max(SMALL) * 4)
        hd = S.lib().shmem_malloc(max(SMALL) * 4)
        np.ctypeslib.as_array((ctypes.c_float * max(SMALL)).from_address(hs))[:] = 0.5 + me
        for n in SMALL:
            t = time_calls(lambda: S.shmem_broadcastmem(team, hd, hs, n * 4, 0), a.reps)
            rows.append(("host", "bcast", n, max_over_pes(t, scratch)))
        S.lib().shmem_free(hd)
        S.lib().shmem_free(hs)
    if a.crossover_dev:
        legs = []
        nmx = max(CROSS_DEV)
        src = S.shmemx_malloc_device(nmx * 4)
        dst = S.shmemx_malloc_device(nmx * 4)
        L.fill(23, 0, 7, me, src, nmx)
        S.shmemx_set_reduce_algorithm(L.ALGS["auto"])
        before = L.lib().sosx_small_path_device_calls()
        for n in CROSS_DEV:
            r = max(10, min(a.reps, int(a.reps * 4096 / max(n, 4096))))
            t = time_calls(lambda: S.shmem_float_sum_reduce(team, dst, src, n), r)
            rows.append(("dev", "auto", n, max_over_pes(t, scratch)))
        small_dev = L.lib().sosx_small_path_device_calls() - before
        S.shmemx_free_device(dst)
        S.shmemx_free_device(src)
        if me == 0:
            print(f"# SHMEMX_SMALL_DEVICE={os.environ.get('SHMEMX_SMALL_DEVICE', 'default')}: "
                  f"{small_dev} device calls on PE 0 took the small path", flush=True)
    if a.crossover:
        legs = []
        nmx = max(CROSS)
        hs = S.lib().shmem_malloc(nmx * 4)
        hd = S.lib().shmem_malloc(nmx * 4)
        np.ctypeslib.as_array((ctypes.c_float * nmx).from_address(hs))[:] = 0.5 + me
        S.shmemx_set_reduce_algorithm(L.ALGS["auto"])
        for n in CROSS:
            r = max(10, min(a.reps, int(a.reps * 4096 / max(n, 4096))))
            t = time_calls(lambda: S.shmem_float_sum_reduce(team, hd, hs, n), r)
            rows.append(("host", "auto", n, max_over_pes(t, scratch)))
        S.lib().shmem_free(hd)
        S.lib().shmem_free(hs)
        cpu, core0 = cpu_leg(me, P, max(a.reps * 10, 2000), scratch, sizes=CROSS)
        for n, t in cpu.items():
            rows.append(("cpu", "auto(sos)", n, t))
    if "dev" in legs:
        src = S.shmemx_malloc_device(nmax * 4)
        dst = S.shmemx_malloc_device(nmax * 4)
        L.fill(23, 0, 7, me, src, nmax)
        plan = [("recdbl", SMALL), ("recdbl_gather", SMALL)] + ([("ring", ring_sizes)] if a.ring else [])
        for alg, ns in plan:
            S.shmemx_set_reduce_algorithm(L.ALGS[alg])
            for n in ns:
                t = time_calls(lambda: S.shmem_float_sum_reduce(team, dst, src, n), a.reps)
                rows.append(("dev", alg, n, max_over_pes(t, scratch)))
        S.shmemx_free_device(dst)
        S.shmemx_free_device(src)
    if "host" in legs:
        hs = S.lib().shmem_malloc(max(SMALL) * 4)
        hd = S.lib().shmem_malloc(max(SMALL) * 4)
        np.ctypeslib.as_array((ctypes.c_float * max(SMALL)).from_address(hs))[:] = 0.5 + me
        for alg in ("recdbl", "recdbl_gather"):
            S.shmemx_set_reduce_algorithm(L.ALGS[alg])
            for n in SMALL:
                t = time_calls(lambda: S.shmem_float_sum_reduce(team, hd, hs, n), a.reps)
                rows.append(("host", alg, n, max_over_pes(t, scratch)))
        S.lib().shmem_free(hd)
        S.lib().shmem_free(hs)
    S.shmemx_set_reduce_algorithm(L.ALGS["auto"])
    if "cpu" in legs:
        cpu, core0 = cpu_leg(me, P, max(a.reps * 10, 2000), scratch)
        for n, t in cpu.items():
            rows.append(("cpu", "recdbl_sw", n, t))
    if me == 0:
        for leg, alg, n, t in rows:
            print(f"P={P} {leg:4s} {alg:14s} n={n:7d}: {t * 1e6:8.2f} us/call", flush=True)
        if a.crossover:
            print(f"# cpu: SOS AUTO on the CPU (oracle_pe_recdbl below 16 KiB, oracle_pe_ring above), "
                  f"{P} processes pinned to consecutive physical cores from {core0}, barrier per call",
                  flush=True)
        if "cpu" in legs:
            print(f"# cpu: oracle_pe_recdbl, {P} processes pinned to consecutive physical cores "
                  f"from {core0}, barrier per call included", flush=True)
    S.shmem_barrier_all()
    S.lib().shmem_free(scratch)
    S.shmem_finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
