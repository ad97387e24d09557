"""Run under tools/oshrun (tests/test_gpu_multipe.py::test_device_heap_colours).

Large device-heap allocations (>= 1 MiB) start at (k mod 8) * 4 KiB mod 32 KiB from the
heap base, k counting them (runtime.cpp Heap::alloc): consecutive large buffers sit an
odd multiple of 4 KiB apart in HBM's 32 KiB channel interleave.  Small allocations and
explicit alignments above 4 KiB are not coloured.  Offsets are symmetric across PEs.
Prints one line per PE with its offsets."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402,F401

from sos_amd import shmem as S  # noqa: E402


def main():
    S.shmem_init()
    me = S.shmem_my_pe()
    L = S.lib()
    big = [S.shmemx_malloc_device((64 << 20) + 4 * k) for k in range(10)]
    small = S.shmemx_malloc_device(4096)
    after = S.shmemx_malloc_device(3 << 20)
    base = min(big + [small, after])
    offs = [p - base for p in big]
    for k, o in enumerate(offs):
        assert o % 256 == 0
    cols = [(o % 32768) // 4096 for o in offs]
    rel = [(big[k + 1] - big[k]) % 32768 for k in range(len(big) - 1)]
    assert all(r % 8192 == 4096 for r in rel), rel
    assert (after - big[-1]) % 8192 == 4096, (after - big[-1]) % 32768
    for p in big + [after, small]:
        L.shmemx_free_device(p)
    # a heap filled to capacity: the whole region (SHMEMX_DEVICE_HEAP_SIZE minus the stage
    # region) in one allocation fits only without the colour padding, which it then goes
    # without instead of failing
    region = int(os.environ["HEAP_REGION_BYTES"])
    full = S.shmemx_malloc_device(region)
    assert full == big[0], (full, big[0])
    L.shmemx_free_device(full)
    again = S.shmemx_malloc_device(64 << 20)   # the colours go on after the fallback
    assert again and (again - big[0]) % 32768 == 4096 * 4, (again - big[0]) % 32768
    L.shmemx_free_device(again)
    print(f"PE {me}: colours {cols} offsets {offs}", flush=True)
    S.shmem_finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
