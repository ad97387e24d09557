"""Latency of shmemx_reduce_local (the local combine, SOS's shmem_internal_reduce_local)
on small operands by residency, one PE: host symmetric heap (pinned), pageable host
memory, device heap; beside the oracle's CPU reduce_local on the same inputs (SOS's own
loop, the baseline).  Prints one JSON line of microseconds per call.  (Bench only.)"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SIZES = [1, 64, 1024, 16384]


def main():
    import numpy as np
    import torch  # noqa: F401
    from oracle import oracle as O
    from sos_amd import _lib as L
    from sos_amd import shmem as S
    S.shmem_init()
    dt, op, es = L.dtype_id("float"), L.op_id("sum"), 4
    nmax = max(SIZES)
    ha, hb = S.lib().shmem_malloc(nmax * es), S.lib().shmem_malloc(nmax * es)
    da, db = S.shmemx_malloc_device(nmax * es), S.shmemx_malloc_device(nmax * es)
    pa, pb = np.ones(nmax, np.float32), np.full(nmax, 0.5, np.float32)
    np.ctypeslib.as_array((ctypes.c_float * nmax).from_address(ha))[:] = 1.0
    np.ctypeslib.as_array((ctypes.c_float * nmax).from_address(hb))[:] = 0.5

    def timed(fn, reps=300):
        for _ in range(20):
            fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return (time.perf_counter() - t0) / reps * 1e6

    rows = []
    for n in SIZES:
        rows.append({
            "nreduce": n,
            "host_heap_us": round(timed(lambda: S.lib().shmemx_reduce_local(op, dt, n, hb, ha)), 2),
            "pageable_us": round(timed(lambda: S.lib().shmemx_reduce_local(
                op, dt, n, pb.ctypes.data, pa.ctypes.data)), 2),
            "device_heap_us": round(timed(lambda: S.lib().shmemx_reduce_local(op, dt, n, db, da)), 2),
            "sos_cpu_us": round(O.time_reduce_local(op, dt, pb[:n], pa[:n], 20000) / 20000 * 1e6, 4),
        })
    S.lib().shmem_free(hb)
    S.lib().shmem_free(ha)
    S.shmemx_free_device(db)
    S.shmemx_free_device(da)
    S.shmem_finalize()
    print(json.dumps({"op": "float sum", "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
