"""Run under tools/oshrun (tests/test_gpu_multipe.py::test_coll_size_crossover_env).

SOS's AUTO picks recdbl_sw below SHMEM_COLL_SIZE_CROSSOVER bytes and the ring at or above
it (src/shmem_collectives.h:179-200, src/collectives.c:647-984).  Every PE reduces 8192
floats (32 KiB) under AUTO on device-heap and host-heap operands and compares its target
bit for bit with the CPU oracle's ring and recdbl_sw; argv[1] names the schedule the
job's environment should select.  The two schedules' fp sums differ on this data (checked
here, so the test cannot pass vacuously).  Prints one line per PE, exit 0 = OK.
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


def main():
    want = sys.argv[1]
    S.shmem_init()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    torch.cuda.set_device(S.lib().shmemx_get_device())
    dt, op = L.dtype_id("float"), L.op_id("sum")
    n, seed = 8192, 0xC505
    ins = [O.fill(dt, 0, seed, q, n) for q in range(P)]
    ring = O.ring(op, dt, ins)[me].view(np.uint32)
    rec = O.recdbl(op, dt, ins)[me].view(np.uint32)
    assert np.count_nonzero(ring != rec) > 0, "ring and recdbl_sw agree on this data"
    exp = {"ring": ring, "recdbl": rec}[want]
    other = rec if want == "ring" else ring
    src = S.shmemx_malloc_device(n * 4)
    dst = S.shmemx_malloc_device(n * 4)
    L.fill(dt, 0, seed, me, src, n)
    torch.cuda.synchronize()
    S.shmem_float_sum_reduce(S.team_world(), dst, src, n)
    got = np.empty(n, np.uint32)
    L.check(L.lib().sosx_memcpy(got.ctypes.data, dst, n * 4, None), "sosx_memcpy")
    hin, hout = S.lib().shmem_malloc(n * 4), S.lib().shmem_malloc(n * 4)
    ctypes.memmove(hin, ins[me].ctypes.data, n * 4)
    S.shmem_float_sum_reduce(S.team_world(), hout, hin, n)
    hgot = np.ctypeslib.as_array((ctypes.c_uint32 * n).from_address(hout)).copy()
    S.shmem_barrier_all()
    S.lib().shmem_free(hout)
    S.lib().shmem_free(hin)
    S.shmemx_free_device(dst)
    S.shmemx_free_device(src)
    S.shmem_finalize()
    bad = {"device": int(np.count_nonzero(got != exp)), "host": int(np.count_nonzero(hgot != exp))}
    if any(bad.values()):
        print(f"PE {me}/{P}: differs from the oracle's {want}: {bad} (vs the other schedule: "
              f"{int(np.count_nonzero(got != other))})", flush=True)
        return 1
    print(f"PE {me}/{P}: {want} bits on device and host heap", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
