"""Run under tools/oshrun (tests/test_gpu_multipe.py::test_calls_end_with_system_release).

Round 5's fix for the 12-PE wrong results: a call's device results
are in HBM -- not only complete -- when it returns, and a p2p post is made only after
the posted bytes are: both go through an event with a system-scope release
(sync_system / release_system, runtime.h), counted by sosx_sys_releases().  This checks,
deterministically, that every executor call of the public API -- team reductions under
each schedule in both p2p signalling modes, a scan, a broadcast, reduce_local on device
operands and a barrier -- issued at least one such marker, and that the results are the
oracle's (read back through tests/readback.py).  Prints one line per PE.

Test infrastructure: the oracle is the checker only.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402,F401

from oracle import oracle as O  # noqa: E402
from sos_amd import _lib as L  # noqa: E402
from sos_amd import shmem as S  # noqa: E402
from tests import readback as R  # noqa: E402


def main():
    S.shmem_init()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    torch.cuda.set_device(S.lib().shmemx_get_device())
    world = S.team_world()
    n = (1 << 20) + 3               # executor sizes (past the small paths)
    dt, op = L.dtype_id("float"), L.op_id("sum")
    hsrc = S.shmemx_malloc_device(n * 4)
    hdst = S.shmemx_malloc_device(n * 4)
    ins = [O.fill(dt, 0, 77, q, n) for q in range(P)]
    L.check(L.lib().sosx_memcpy(hsrc, ins[me].ctypes.data, n * 4, None), "sosx_memcpy")
    bad, calls = [], 0

    def call(what, fn, exp=None):
        nonlocal calls
        r0 = L.lib().sosx_sys_releases()
        fn()
        r1 = L.lib().sosx_sys_releases()
        calls += 1
        if r1 <= r0:
            bad.append((what, "no system-scope release"))
        if exp is not None:
            mm = R.mismatches(exp, R.device_bytes(hdst, n * 4), 4)
            if mm:
                bad.append((what, f"{mm} wrong"))

    modes = [m for m in (1, 0) if L.lib().sosx_set_p2p_signal_mode(m) >= 0] or [None]
    for mode in modes:
        for alg in ("auto", "recdbl_gather", "recdbl", "rechalving"):
            S.shmemx_set_reduce_algorithm(L.ALGS[alg])
            res = S.lib().sosx_resolve_alg(L.ALGS[alg], n * 4, 16384)
            exp = (O.ring(op, dt, ins) if res == L.ALGS["ring"] else O.recdbl(op, dt, ins))[me]
            call(f"reduce {alg} signal {mode}",
                 lambda: S.shmem_float_sum_reduce(world, hdst, hsrc, n), exp)
    S.shmemx_set_reduce_algorithm(L.ALGS["auto"])
    call("inscan", lambda: S.shmemx_float_sum_inscan(world, hdst, hsrc, n),
         O.scan(op, dt, ins, False)[me])
    call("broadcast", lambda: S.shmem_float_broadcast(world, hdst, hsrc, n, 0), ins[0])
    L.check(L.lib().sosx_memcpy(hdst, ins[me].ctypes.data, n * 4, None), "sosx_memcpy")
    local = ins[me].copy()
    O.reduce_local(op, dt, ins[me], local)
    call("reduce_local", lambda: S.lib().shmemx_reduce_local(op, dt, n, hsrc, hdst), local)
    call("barrier", S.shmem_barrier_all)
    S.shmemx_free_device(hdst)
    S.shmemx_free_device(hsrc)
    S.shmem_finalize()
    if bad:
        print(f"PE {me}/{P}: {len(bad)} of {calls} calls FAILED: {bad[:6]}", flush=True)
        return 1
    print(f"PE {me}/{P}: {calls} calls, each ended with a system-scope release", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
