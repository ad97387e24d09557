"""Stress of the p2p executor's in-place peer reads (run under tools/oshrun, P PEs on one
GPU; DESIGN.md section 5 "Open (round 4)").

Repeats the sequence team_check_pe.py ran when PE 8 of 12 once saw a wrong
recdbl_gather result: per iteration, with a fresh seed, shmem_float_sum_reduce on
device-heap operands (out of place, then in place), then a staged call on torch buffers
(the stage region), each checked bit for bit against the CPU oracle's recdbl_sw value
(oracle/sos_oracle.c, src/collectives.c:850-984).  On a mismatch it prints the differing
element runs, a recount after a device synchronisation, and which single peer input,
replaced by that peer's previous heap contents (the last in-place result), would explain
the wrong elements -- i.e. whether a stale peer operand was read.

Bench/diagnostic code: the oracle is the checker only.
Usage: tools/oshrun -np 12 python tools/p2p_stress.py [--iters 60] [--n 1048579] [--alg recdbl_gather]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from sos_amd import _lib as L  # noqa: E402
from sos_amd import shmem as S  # noqa: E402


def download(ptr, nbytes):
    t = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    L.check(L.lib().sosx_memcpy(t.data_ptr(), ptr, nbytes, None), "sosx_memcpy")
    torch.cuda.synchronize()
    return t.cpu().numpy()


def runs_of(idx, k=4):
    if idx.size == 0:
        return []
    cuts = np.nonzero(np.diff(idx) != 1)[0]
    starts = np.concatenate(([idx[0]], idx[cuts + 1]))
    ends = np.concatenate((idx[cuts], [idx[-1]])) + 1
    return [(int(a), int(b)) for a, b in zip(starts[:k], ends[:k])] + [f"{starts.size} runs"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--n", type=int, default=(1 << 20) + 3)
    ap.add_argument("--n2", type=int, default=65536)
    ap.add_argument("--alg", default="recdbl_gather")
    ap.add_argument("--release", action="store_true",
                    help="every iteration starts from released workspaces and runs a small call "
                         "first, so each big call is the first after its scratch grew (hipFree + "
                         "hipMalloc), the condition of the round-4 failure, every iteration")
    a = ap.parse_args()
    S.shmem_init()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    torch.cuda.set_device(S.lib().shmemx_get_device())
    world = S.team_world()
    dt, op = L.dtype_id("float"), L.op_id("sum")
    S.shmemx_set_reduce_algorithm(L.ALGS[a.alg])
    n, n2 = a.n, a.n2
    hsrc = S.shmemx_malloc_device(n * 4)
    hdst = S.shmemx_malloc_device(n * 4)
    fn = S.shmem_float_sum_reduce
    prev = None      # every PE's hsrc contents before this iteration's fill
    bad, checks = [], 0
    grows = 0
    for it in range(a.iters):
        seed = 0x51A000 + it
        if a.release:
            L.lib().sosx_release_workspaces()
            # a small heap call: the scratch is allocated at its (small) size first
            t1 = O.fill(dt, 0, seed + 3, me, n2)
            L.check(L.lib().sosx_memcpy(hsrc, t1.ctypes.data, n2 * 4, None), "sosx_memcpy")
            fn(world, hdst, hsrc, n2)
            e1 = O.recdbl(op, dt, [O.fill(dt, 0, seed + 3, q, n2) for q in range(P)])[me]
            checks += 1
            m1 = int(np.count_nonzero(download(hdst, n2 * 4).view(np.uint32) != e1.view(np.uint32)))
            if m1:
                bad.append({"iter": it, "mode": "small_first", "mismatches": m1})
            grows += 1
        if me == 0 and it % 10 == 0:
            print(f"[p2p_stress] iteration {it}/{a.iters}", file=sys.stderr, flush=True)
        ins = [O.fill(dt, 0, seed, q, n) for q in range(P)]
        exp = O.recdbl(op, dt, ins)[me]
        for mode in ("heap", "heap_inplace"):
            L.fill(dt, 0, seed, me, hsrc, n)
            torch.cuda.synchronize()
            out = hdst if mode == "heap" else hsrc
            fn(world, out, hsrc, n)
            got = download(out, n * 4).view(np.float32)
            checks += 1
            diff = np.nonzero(got.view(np.uint32) != exp.view(np.uint32))[0]
            if diff.size:
                torch.cuda.synchronize()
                again = np.count_nonzero(download(out, n * 4).view(np.uint32) != exp.view(np.uint32))
                culprits = []
                if prev is not None:
                    for q in range(P):
                        if q == me:
                            continue
                        alt = [x[diff].copy() for x in ins]
                        alt[q] = prev[diff].copy()
                        if np.array_equal(O.recdbl(op, dt, alt)[me].view(np.uint32),
                                          got[diff].view(np.uint32)):
                            culprits.append(q)
                bad.append({"iter": it, "mode": mode, "mismatches": int(diff.size),
                            "runs": runs_of(diff), "recount": int(again),
                            "stale_peer_explains": culprits,
                            "sample": [(int(i), float(got[i]), float(exp[i])) for i in diff[:3]]})
        prev = exp  # hsrc now holds the in-place result on every PE (same value everywhere)
        # a staged call through the stage region, as team_check's "device" mode
        t_in = torch.empty(n2 * 4, dtype=torch.uint8, device="cuda")
        t_out = torch.empty_like(t_in)
        L.fill(dt, 0, seed + 7, me, t_in.data_ptr(), n2)
        torch.cuda.synchronize()
        fn(world, t_out.data_ptr(), t_in.data_ptr(), n2)
        e2 = O.recdbl(op, dt, [O.fill(dt, 0, seed + 7, q, n2) for q in range(P)])[me]
        got2 = t_out.cpu().numpy().view(np.uint32)
        checks += 1
        m2 = int(np.count_nonzero(got2 != e2.view(np.uint32)))
        if m2:
            bad.append({"iter": it, "mode": "device_staged", "mismatches": m2})
    S.shmem_barrier_all()
    S.shmemx_free_device(hdst)
    S.shmemx_free_device(hsrc)
    S.shmem_finalize()
    if bad:
        print(f"PE {me}/{P}: {len(bad)} of {checks} FAILED: {bad[:4]}", flush=True)
        return 1
    print(f"PE {me}/{P}: {checks} checks OK ({a.alg}, n={n}, {a.iters} iterations, "
          f"{grows} calls right after a scratch grow)", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
