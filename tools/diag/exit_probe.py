"""Diagnostic: run one kind of library call in a fresh process and exit (exit-time crash hunt)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from sos_amd import _lib, shmem as S

mode = sys.argv[1]
n = 4099
t = [torch.ones(n * 8, dtype=torch.uint8, device="cuda") for _ in range(80)]
p = [x.data_ptr() for x in t]
if mode == "combine":
    _lib.combine(5, 23, p[0], p[1], n)
elif mode == "fold8":
    _lib.fold(5, 23, 0, p[0], p[1:9], n)
elif mode == "fold12":
    _lib.fold(5, 23, 1, p[0], p[1:13], n)
elif mode == "fold16":
    _lib.fold(5, 23, 1, p[0], p[1:17], n)
elif mode == "fold64":
    _lib.fold(5, 23, 1, p[0], p[1:65], n)
elif mode == "fold64l":
    _lib.fold(5, 23, 0, p[0], p[1:65], n)
elif mode == "prefix3":
    _lib.prefix(5, 23, p[0:3], p[3:6], n)
elif mode == "prefix12":
    _lib.prefix(5, 23, [x for x in p[0:12]], [x for x in p[4:16]], 100)
elif mode == "lb_ring4":
    S.loopback_allreduce("ring", 5, 23, p[0:4], p[4:8], n)
elif mode == "lb_scan4":
    S.loopback_allreduce(16, 5, 23, p[0:4], p[4:8], n)
elif mode == "lb_bcast4":
    S.loopback_allreduce(_lib.plan_bcast(1, True), 5, 13, p[0:4], p[4:8], n)
elif mode == "lb_ring12":
    S.loopback_allreduce("ring", 5, 23, p[0:12], p[0:12], 100)
torch.cuda.synchronize()
print("ok", mode, flush=True)
