"""One PE of test_ipc_heap_sizes_with_bit31: time shmem_init (device heap + IPC mapping)
for SHMEMX_DEVICE_HEAP_SIZE (also a diagnostic: run under tools/oshrun -np 2)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from sos_amd import shmem as S  # noqa: E402

t0 = time.time()
print(f"PE {os.environ.get('SHMEM_PE')}: init start heap={os.environ.get('SHMEMX_DEVICE_HEAP_SIZE')}",
      flush=True)
S.shmem_init()
print(f"PE {S.shmem_my_pe()}: init {time.time() - t0:.2f} s", flush=True)
S.shmem_barrier_all()
S.lib().shmem_finalize()
print(f"PE done {time.time() - t0:.2f} s", flush=True)
