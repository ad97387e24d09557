"""Run under tools/oshrun (tests/test_gpu_multipe.py::test_peer_reads_follow_system_acquire).

The consumer half of the memory-visibility rule (DESIGN.md section
7.3): a launch that reads bytes a peer published -- the p2p executor's gathers and its
folds of peer memory in place, the small path's reads of the peers' slots -- follows, in
stream order, a system-scope acquire issued after the wait that saw the peer's post.  The
library classifies its waits and launches itself and counts (sosx_acquire_stats):
acquires issued, peer reads, and peer reads with a wait since the last acquire.  This
checks, deterministically and per call, that every team call read peers' bytes, issued
acquires, and left the unacquired count at 0 -- reductions under four schedules in both
p2p signalling modes at 1Mi + 3 elements and under two at 16Ki + 3 (gathers small enough
to carry their signalling step), a scan, a broadcast, and the small path with host and
device operands -- and that every result is the oracle's, read back by a plain D2H copy
(tests/readback.py).  Small consuming grids carry the acquire in their own workgroups
(carry.h): the 16Ki + 3 calls must run no acquire kernel at all, and an 8Mi + 3 call,
whose folds stream, must run them.  Prints one line per PE with the XCD mask of the
acquire kernels.

Test infrastructure: the oracle is the checker only.
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from oracle import oracle as O  # noqa: E402
from sos_amd import _lib as L  # noqa: E402
from sos_amd import shmem as S  # noqa: E402
from tests import readback as R  # noqa: E402


def stats(mask=False):
    a, r, u = ctypes.c_long(), ctypes.c_long(), ctypes.c_long()
    m = ctypes.c_uint()
    L.lib().sosx_acquire_stats(ctypes.byref(a), ctypes.byref(r), ctypes.byref(u),
                               ctypes.byref(m) if mask else None)
    return a.value, r.value, u.value, m.value


def main():
    S.shmem_init()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    torch.cuda.set_device(S.lib().shmemx_get_device())
    world = S.team_world()
    dt, op = L.dtype_id("float"), L.op_id("sum")
    bad, calls = [], 0

    def call(what, fn, exp=None, got=None, reads=True, kernels=None):
        nonlocal calls
        a0, r0, u0, _ = stats()
        k0 = L.lib().sosx_acquire_kernels()
        fn()
        a1, r1, u1, _ = stats()
        k1 = L.lib().sosx_acquire_kernels()
        calls += 1
        if kernels is not None and (k1 > k0) != kernels:
            bad.append((what, f"{k1 - k0} acquire kernels, expected {'some' if kernels else 'none'}"))
        if reads and r1 <= r0:
            bad.append((what, "no launch read a peer's bytes"))
        if reads and a1 <= a0:
            bad.append((what, "no system-scope acquire"))
        if u1 != u0:
            bad.append((what, f"{u1 - u0} peer reads without an acquire"))
        if exp is not None:
            mm = R.mismatches(exp, got(), 4)
            if mm:
                bad.append((what, f"{mm} wrong"))

    # the executors: device-heap operands past the small paths
    n = (1 << 20) + 3
    big = (8 << 20) + 3
    dsrc = S.shmemx_malloc_device(big * 4)
    ddst = S.shmemx_malloc_device(big * 4)
    ins = [O.fill(dt, 0, 91, q, n) for q in range(P)]
    L.check(L.lib().sosx_memcpy(dsrc, ins[me].ctypes.data, n * 4, None), "sosx_memcpy")
    dget = lambda: R.device_bytes(ddst, n * 4)  # noqa: E731
    modes = [m for m in (1, 0) if L.lib().sosx_set_p2p_signal_mode(m) >= 0] or [None]
    for mode in modes:
        for alg in ("auto", "recdbl_gather", "recdbl", "rechalving"):
            S.shmemx_set_reduce_algorithm(L.ALGS[alg])
            res = S.lib().sosx_resolve_alg(L.ALGS[alg], n * 4, 16384)
            exp = (O.ring(op, dt, ins) if res == L.ALGS["ring"] else O.recdbl(op, dt, ins))[me]
            call(f"reduce {alg} signal {mode}",
                 lambda: S.shmem_float_sum_reduce(world, ddst, dsrc, n), exp, dget)
        S.shmemx_set_reduce_algorithm(L.ALGS["auto"])
        # PE 0's inclusive prefix and the root's broadcast need nothing from a peer
        call(f"inscan signal {mode}", lambda: S.shmemx_float_sum_inscan(world, ddst, dsrc, n),
             O.scan(op, dt, ins, False)[me], dget, reads=me != 0)
        call(f"broadcast signal {mode}", lambda: S.shmem_float_broadcast(world, ddst, dsrc, n, 0),
             ins[0], dget, reads=me != 0)
    # streaming folds (8Mi + 3 elements): the acquire kernel before them
    bins = [O.fill(dt, 0, 94, q, big) for q in range(P)]
    L.check(L.lib().sosx_memcpy(dsrc, bins[me].ctypes.data, big * 4, None), "sosx_memcpy")
    bexp = O.ring(op, dt, bins)[me]
    for mode in modes:
        call(f"big ring signal {mode}", lambda: S.shmem_float_sum_reduce(world, ddst, dsrc, big), bexp,
             lambda: R.device_bytes(ddst, big * 4), kernels=True)
    # mid-size device operands (past SHMEMX_SMALL_DEVICE, gathers of <= 256 KiB): in stream
    # mode the signalling step rides in the gather launch, which acquires per workgroup;
    # every consuming launch is small enough to carry the acquire (no acquire kernel)
    mid = 16384 + 3
    mins = [O.fill(dt, 0, 93, q, mid) for q in range(P)]
    L.check(L.lib().sosx_memcpy(dsrc, mins[me].ctypes.data, mid * 4, None), "sosx_memcpy")
    for mode in modes:
        for alg in ("auto", "recdbl_gather"):
            S.shmemx_set_reduce_algorithm(L.ALGS[alg])
            res = S.lib().sosx_resolve_alg(L.ALGS[alg], mid * 4, 16384)
            exp = (O.ring(op, dt, mins) if res == L.ALGS["ring"] else O.recdbl(op, dt, mins))[me]
            call(f"mid {alg} signal {mode}", lambda: S.shmem_float_sum_reduce(world, ddst, dsrc, mid), exp,
                 lambda: R.device_bytes(ddst, mid * 4), kernels=False)
    S.shmemx_set_reduce_algorithm(L.ALGS["auto"])
    # the small path: host-heap operands, then small device-heap operands
    m = 64
    sins = [O.fill(dt, 0, 92, q, m) for q in range(P)]
    sexp = O.recdbl(op, dt, sins)[me]
    hsrc = S.lib().shmem_malloc(m * 4)
    hdst = S.lib().shmem_malloc(m * 4)
    ctypes.memmove(hsrc, sins[me].ctypes.data, m * 4)
    small0 = L.lib().sosx_small_path_calls()
    call("small host", lambda: S.shmem_float_sum_reduce(world, hdst, hsrc, m), sexp,
         lambda: np.frombuffer(ctypes.string_at(hdst, m * 4), np.uint8))
    L.check(L.lib().sosx_memcpy(dsrc, sins[me].ctypes.data, m * 4, None), "sosx_memcpy")
    call("small device", lambda: S.shmem_float_sum_reduce(world, ddst, dsrc, m), sexp,
         lambda: R.device_bytes(ddst, m * 4))
    if L.lib().sosx_small_path_calls() - small0 != 2:
        bad.append(("small", "the small calls did not take the small path"))
    acq, reads, unacq, mask = stats(mask=True)
    S.lib().shmem_free(hdst)
    S.lib().shmem_free(hsrc)
    S.shmemx_free_device(ddst)
    S.shmemx_free_device(dsrc)
    S.shmem_finalize()
    if bad:
        print(f"PE {me}/{P}: {len(bad)} of {calls} calls FAILED: {bad[:6]}", flush=True)
        return 1
    print(f"PE {me}/{P}: {calls} calls, {reads} peer reads, {acq} acquires, {unacq} unacquired, "
          f"{L.lib().sosx_acquire_kernels()} acquire kernels, xcc mask 0x{mask:02x}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
