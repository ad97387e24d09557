"""Diagnostic: sosx_combine_host (the 3-stream H2D || combine || D2H chunk pipeline, raw HIP
streams and events) on 128Mi pinned fp32 at several chunk sizes, against the serial
H2D + combine + D2H.  Shows how the HIP runtime treats many small pipelined copies."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from sos_amd import _lib as L  # noqa: E402

n = 128 << 20
torch.cuda.set_device(0)
lib = L.lib()
ha = torch.zeros(n * 4, dtype=torch.uint8, pin_memory=True)
hb = torch.zeros(n * 4, dtype=torch.uint8, pin_memory=True)
for chunk_mib in (1, 2, 4, 8, 16, 32, 64):
    cb = chunk_mib << 20
    L.check(lib.sosx_combine_host(5, 23, ha.data_ptr(), hb.data_ptr(), n, cb), "warm")
    t0 = time.perf_counter()
    for _ in range(5):
        L.check(lib.sosx_combine_host(5, 23, ha.data_ptr(), hb.data_ptr(), n, cb), "run")
    t = (time.perf_counter() - t0) / 5
    print(f"chunk {chunk_mib:3d} MiB ({n * 4 // cb:4d} chunks): {t * 1e3:8.3f} ms "
          f"= {n * 4 / t / 2**30:.2f} GiB/s payload", flush=True)
