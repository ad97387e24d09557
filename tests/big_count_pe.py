"""A team reduction of 2^31 + 4101 elements per PE (run under tools/oshrun, p2p
transport): shmem_uint8_sum_reduce over SHMEM_TEAM_WORLD, which SOS's `int nreduce`
cannot express, through AUTO (the ring at this size) -- 64-bit chunk math in the plan,
the exchange and the fold.  Each PE checks its target bit for bit against the CPU
oracle's ring over every PE's regenerated input.  Prints one line per PE, exit 0 = OK.
Test infrastructure: the oracle is the checker only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from sos_amd import _lib as L  # noqa: E402
from sos_amd import shmem as S  # noqa: E402


def main():
    S.shmem_init()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    torch.cuda.set_device(S.lib().shmemx_get_device())
    n, dt, op, seed = (1 << 31) + 4101, L.dtype_id("uint8"), L.op_id("sum"), 77
    src, dst = S.shmemx_malloc_device(n), S.shmemx_malloc_device(n)
    assert src and dst
    L.fill(dt, 0, seed, me, src, n)
    torch.cuda.synchronize()
    S.shmem_uint8_sum_reduce(S.team_world(), dst, src, n)
    got = torch.empty(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    L.check(S.lib().sosx_memcpy(got.data_ptr(), dst, n, None), "sosx_memcpy")
    got = got.cpu().numpy()
    S.shmemx_free_device(dst)
    S.shmemx_free_device(src)
    resolved = S.lib().sosx_resolve_alg(L.ALGS["auto"], n, 16384)
    exp = O.ring(op, dt, [O.fill(dt, 0, seed, pe, n) for pe in range(P)])[me]
    mism = int(np.count_nonzero(got != exp))
    S.shmem_finalize()
    if resolved != L.ALGS["ring"] or mism:
        print(f"PE {me}/{P}: FAILED (alg {resolved}, {mism} mismatching bytes of {n})", flush=True)
        return 1
    print(f"PE {me}/{P}: {n} elements OK", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
