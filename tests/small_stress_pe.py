"""Slot-protocol stress of the small shared-memory path (run under tools/oshrun, P >= 2).

Every PE walks the same seeded sequence of small reductions over interleaved teams --
the world, the even PEs and the odd PEs (split_strided, P >= 4) -- with host-heap and
device-heap operands and sizes on both sides of the crossover, so the per-pair post
counters of different pairs drift apart and each PE's two slots are reused across teams
in every order (smallpath.cpp: posted / consumed / ring of slot ids; device operands are
staged and posted by the copy kernel).  A PE takes part only in the calls of teams it
belongs to.  Every result is checked bit for bit against the CPU oracle (recdbl_sw below
16 KiB, the ring above, as SOS AUTO resolves) over the members' regenerated inputs.
Prints one line per PE, exit 0 = OK.  Test infrastructure: the oracle is the checker.
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from sos_amd import _lib as L  # noqa: E402
from sos_amd import shmem as S  # noqa: E402

CALLS = int(os.environ.get("SMALL_STRESS_CALLS", "400"))
CASES = [("float", "sum"), ("double", "max"), ("int", "xor"), ("long", "prod")]
SIZES = [1, 3, 64, 1000, 4101]


def main():
    S.shmem_init()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    torch.cuda.set_device(S.lib().shmemx_get_device())
    world = S.team_world()
    teams = [(world, list(range(P)))]
    if P >= 4:
        for start in (0, 1):
            h = ctypes.c_void_p(0)
            size = (P - start + 1) // 2
            S.lib().shmem_team_split_strided(world, start, 2, size, None, 0, ctypes.byref(h))
            teams.append((h.value, list(range(start, P, 2))))
    nmax, es_max = max(SIZES), 8
    hsrc, hdst = S.lib().shmem_malloc(nmax * es_max), S.lib().shmem_malloc(nmax * es_max)
    dsrc, ddst = S.shmemx_malloc_device(nmax * es_max), S.shmemx_malloc_device(nmax * es_max)
    rng = np.random.default_rng(2024)      # the same sequence on every PE
    small_before = L.lib().sosx_small_path_calls()
    dev_before = L.lib().sosx_small_path_device_calls()
    bad, checks = [], 0
    for call in range(CALLS):
        ti = int(rng.integers(len(teams)))
        tname, oname = CASES[int(rng.integers(len(CASES)))]
        n = SIZES[int(rng.integers(len(SIZES)))]
        dev = bool(rng.integers(2))
        handle, members = teams[ti]
        if me not in members:
            continue
        dt, opid = L.dtype_id(tname), L.op_id(oname)
        es = L.dtype_size(dt)
        dist = L.DIST_PROD if oname == "prod" else L.DIST_UNIFORM
        ins = [O.fill(dt, dist, call, pe, n) for pe in members]
        idx = members.index(me)
        resolved = S.lib().sosx_resolve_alg(L.ALGS["auto"], n * es, 16384)
        exp = (O.ring if resolved == L.ALGS["ring"] else O.recdbl)(opid, dt, ins)[idx]
        mine = np.frombuffer(ins[idx].tobytes(), np.uint8).copy()
        fn = getattr(S, f"shmem_{tname}_{oname}_reduce")
        if dev:
            L.check(L.lib().sosx_memcpy(dsrc, mine.ctypes.data, n * es, None), "sosx_memcpy")
            fn(handle, ddst, dsrc, n)
            got = np.empty(n * es, np.uint8)
            L.check(L.lib().sosx_memcpy(got.ctypes.data, ddst, n * es, None), "sosx_memcpy")
        else:
            ctypes.memmove(hsrc, mine.ctypes.data, n * es)
            fn(handle, hdst, hsrc, n)
            got = np.ctypeslib.as_array((ctypes.c_uint8 * (n * es)).from_address(hdst)).copy()
        checks += 1
        if not np.array_equal(got, np.frombuffer(exp.tobytes(), np.uint8)):
            bad.append((call, ti, tname, oname, n, "dev" if dev else "host"))
    small = L.lib().sosx_small_path_calls() - small_before
    small_dev = L.lib().sosx_small_path_device_calls() - dev_before
    S.shmem_barrier_all()
    for h, _ in teams[1:]:
        if h:
            S.lib().shmem_team_destroy(ctypes.c_void_p(h))
    S.shmemx_free_device(ddst)
    S.shmemx_free_device(dsrc)
    S.lib().shmem_free(hdst)
    S.lib().shmem_free(hsrc)
    S.shmem_finalize()
    if bad:
        print(f"PE {me}/{P}: {len(bad)} of {checks} checks FAILED: {bad[:6]}", flush=True)
        return 1
    print(f"PE {me}/{P}: {checks} checks OK (small-path calls {small}, device {small_dev})", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
