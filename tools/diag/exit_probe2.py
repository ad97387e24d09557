"""Diagnostic: the body of test_fold_runtime_p as a plain script (exit-time crash hunt)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
from sos_amd import _lib

use_oracle = sys.argv[1] == "oracle"
Ps = [int(x) for x in sys.argv[2].split(",")]
if use_oracle:
    from oracle import oracle as O
    import plansim
for P in Ps:
    for order in (0, 1):
        n = 1001
        if use_oracle:
            ins = [O.fill(23, 0, 3, k, n) for k in range(P)]
            ref = plansim.fold_values(5, 23, ins, order)
        else:
            ins = [np.random.default_rng(k).standard_normal(n).astype(np.float32) for k in range(P)]
        di = []
        for a in ins:
            raw = np.frombuffer(a.tobytes(), np.uint8)
            t = torch.zeros(raw.size + 16, dtype=torch.uint8, device="cuda")
            t[:raw.size].copy_(torch.from_numpy(raw.copy()))
            di.append(t)
        out = torch.zeros_like(di[0])
        _lib.fold(5, 23, order, out.data_ptr(), [t.data_ptr() for t in di], n)
        torch.cuda.synchronize()
        got = np.frombuffer(out[:n * 4].cpu().numpy().tobytes(), np.float32)
        if use_oracle:
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
print("ok", sys.argv[1:], flush=True)
