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
import time

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


_PINNED = {}


def direct_pinned(ptr, nbytes):
    """Host copy of device memory by ONE D2H copy into pinned host memory (a DMA read of
    HBM, no runtime staging buffer)."""
    t = _PINNED.get(nbytes)
    if t is None:
        t = _PINNED[nbytes] = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    L.check(L.lib().sosx_memcpy(t.data_ptr(), ptr, nbytes, None), "sosx_memcpy")
    return t.numpy()


def direct(ptr, nbytes):
    """Host copy of device memory by ONE D2H copy (no intermediate device buffer)."""
    h = np.empty(nbytes, np.uint8)
    L.check(L.lib().sosx_memcpy(h.ctypes.data, ptr, nbytes, None), "sosx_memcpy")
    return h


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
    ap.add_argument("--reader", default="three", choices=("three", "download"),
                    help="three: pinned D2H, pageable D2H and a compare kernel; download: round "
                         "4's path only (D2D into a torch buffer, then torch's D2H)")
    a = ap.parse_args()
    S.shmem_init()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    torch.cuda.set_device(S.lib().shmemx_get_device())
    world = S.team_world()
    dt, op = L.dtype_id("float"), L.op_id("sum")
    S.shmemx_set_reduce_algorithm(L.ALGS[a.alg])

    def oracle_of(ins):  # the schedule the call resolves to at this size (AUTO: ring or recdbl_sw)
        res = S.lib().sosx_resolve_alg(L.ALGS[a.alg], ins[0].size * 4, 16384)
        return (O.ring if res == L.ALGS["ring"] else O.recdbl)(op, dt, ins)
    n, n2 = a.n, a.n2
    hsrc = S.shmemx_malloc_device(n * 4)
    hdst = S.shmemx_malloc_device(n * 4)
    hexp = S.shmemx_malloc_device(n * 4)
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
            e1 = oracle_of([O.fill(dt, 0, seed + 3, q, n2) for q in range(P)])[me]
            checks += 1
            m1 = int(np.count_nonzero(direct(hdst, n2 * 4).view(np.uint32) != e1.view(np.uint32)))
            if m1:
                bad.append({"iter": it, "mode": "small_first", "mismatches": m1})
            grows += 1
        if me == 0 and it % 10 == 0:
            print(f"[p2p_stress] iteration {it}/{a.iters}", file=sys.stderr, flush=True)
        ins = [O.fill(dt, 0, seed, q, n) for q in range(P)]
        exp = oracle_of(ins)[me]
        # the expected bytes in device memory for the kernel reader, checked after upload
        L.check(L.lib().sosx_memcpy(hexp, exp.ctypes.data, n * 4, None), "sosx_memcpy")
        assert np.array_equal(direct_pinned(hexp, n * 4), exp.view(np.uint8)), "expected-bytes upload"
        for mode in ("heap", "heap_inplace"):
            L.fill(dt, 0, seed, me, hsrc, n)
            torch.cuda.synchronize()
            out = hdst if mode == "heap" else hsrc
            # what `out` held before this call: heap -> the small call's result in front of
            # the previous iteration's result; in place -> this PE's own input
            if mode == "heap":
                before = prev.copy() if prev is not None else np.zeros(n, np.float32)
                if a.release:
                    before[:n2] = e1
            else:
                before = ins[me]
            fn(world, out, hsrc, n)
            # three readers of `out`, in this order: a D2H copy into pinned host memory (one
            # DMA read of HBM), a D2H copy into pageable memory (staged by the runtime), and
            # a kernel comparing `out` with the expected bytes uploaded (and read back) before
            # the call (L2-coherent device reads)
            if a.reader == "download":
                seen = {"download": download(out, n * 4).view(np.float32)}
                kern = 0
            else:
                seen = {"pinned": direct_pinned(out, n * 4).view(np.float32).copy(),
                        "pageable": direct(out, n * 4).view(np.float32)}
                kern = L.count_mismatch(hexp, out, n, 4)
            checks += 1
            dd = {how: np.nonzero(seen[how].view(np.uint32) != exp.view(np.uint32))[0] for how in seen}
            if kern or any(v.size for v in dd.values()):
                time.sleep(0.05)
                later = direct_pinned(out, n * 4).view(np.uint32)
                again = int(np.count_nonzero(later != exp.view(np.uint32)))
                rec = {"iter": it, "mode": mode, "kernel_count": int(kern), "pinned_after_50ms": again}
                for how in seen:
                    diff = dd[how]
                    if not diff.size:
                        rec[how] = 0
                        continue
                    got = seen[how]
                    stale = int(np.count_nonzero(got[diff].view(np.uint32) == before[diff].view(np.uint32)))
                    rec[how] = {"mismatches": int(diff.size), "runs": runs_of(diff),
                                "equal_to_previous_contents": stale}
                bad.append(rec)
        prev = exp  # hsrc now holds the in-place result on every PE (same value everywhere)
        # a staged call through the stage region, as team_check's "device" mode
        t_in = torch.empty(n2 * 4, dtype=torch.uint8, device="cuda")
        t_out = torch.empty_like(t_in)
        L.fill(dt, 0, seed + 7, me, t_in.data_ptr(), n2)
        torch.cuda.synchronize()
        fn(world, t_out.data_ptr(), t_in.data_ptr(), n2)
        e2 = oracle_of([O.fill(dt, 0, seed + 7, q, n2) for q in range(P)])[me]
        got2 = t_out.cpu().numpy().view(np.uint32)
        checks += 1
        m2 = int(np.count_nonzero(got2 != e2.view(np.uint32)))
        if m2:
            bad.append({"iter": it, "mode": "device_staged", "mismatches": m2})
    S.shmem_barrier_all()
    S.shmemx_free_device(hexp)
    S.shmemx_free_device(hdst)
    S.shmemx_free_device(hsrc)
    S.shmem_finalize()
    if bad:
        print(f"PE {me}/{P}: {len(bad)} of {checks} FAILED: {bad[:6]}", flush=True)
        return 1
    print(f"PE {me}/{P}: {checks} checks OK ({a.alg}, n={n}, {a.iters} iterations, "
          f"{grows} calls right after a scratch grow)", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
