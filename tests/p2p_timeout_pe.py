"""Run under tools/oshrun with 2 PEs (p2p transport): PE 1 reaches the reduction 60 s
late; PE 0, with SHMEMX_P2P_TIMEOUT=3, must end the job with the p2p timeout error
instead of hanging (tests/test_gpu_multipe.py::test_p2p_wait_is_bounded).  With `host`
as argument the operands are 64 floats in the host symmetric heap, with `devsmall` 64
floats in the device heap: either call takes the small shared-memory path and its own
bounded waits (test_small_path_wait_is_bounded)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402,F401

from sos_amd import shmem as S  # noqa: E402


def main():
    S.shmem_init()
    me = S.shmem_my_pe()
    mode = sys.argv[1] if len(sys.argv) > 1 else "device"
    host = mode == "host"
    n = 1 << 16 if mode == "device" else 64
    alloc = S.lib().shmem_malloc if host else S.shmemx_malloc_device
    src = alloc(n * 4)
    dst = alloc(n * 4)
    S.shmem_barrier_all()
    if me == 1:
        time.sleep(60)
    S.shmem_float_sum_reduce(S.team_world(), dst, src, n)
    print(f"PE {me}: reduction returned", flush=True)
    S.shmem_finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
