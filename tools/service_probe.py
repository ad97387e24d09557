"""Bench-only probe: the host<->GPU round trip through a resident kernel (k_ping_service,
tools/variants) against a launch + completion-word poll and a launch + stream sync.

The resident kernel polls a request word in pinned host memory and answers in another;
the host writes the request and spins on the answer.  This is the floor a resident
small-collective service would have per call, against the ~10-13 us per launch of
profiles/r5_sync_cost.json.  Prints one JSON line.
Usage: python tools/service_probe.py [--iters 20000] [--rounds 5]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HIP = ctypes.CDLL("libamdhip64.so.7")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20000)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    torch.cuda.init()
    v = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", "libsos_variants.so"))
    v.sosxv_ping_launch.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p]
    s = torch.cuda.Stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    ctl = ctypes.c_void_p()
    assert HIP.hipHostMalloc(ctypes.byref(ctl), ctypes.c_size_t(4096), ctypes.c_uint(0x2)) == 0  # coherent
    w = (ctypes.c_uint64 * 4).from_address(ctl.value)
    res = {}
    for nap in (0, 1):
        name = f"resident kernel, s_sleep {nap}"
        res[name] = []
        for _ in range(a.rounds):
            for i in range(4):
                w[i] = 0
            assert v.sosxv_ping_launch(ctl, ctypes.c_longlong(200_000_000), nap, sp) == 0  # 2 s idle
            # first answer: the kernel is resident
            w[0] = 1
            t0 = time.perf_counter()
            while w[1] != 1:
                if time.perf_counter() - t0 > 5:
                    raise SystemExit("resident kernel did not answer")
            t0 = time.perf_counter()
            for k in range(2, a.iters + 2):
                w[0] = k
                while w[1] != k:
                    pass
            res[name].append((time.perf_counter() - t0) / a.iters * 1e6)
            w[2] = 1  # stop
            HIP.hipStreamSynchronize(sp)
            assert w[3] == 1
    # request word in fine-grained device memory (the host writes it over the link, the
    # kernel polls it locally), answer in pinned host memory (the host polls it locally)
    v.sosxv_ping_split_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]
    dreq = ctypes.c_void_p()
    rc = HIP.hipExtMallocWithFlags(ctypes.byref(dreq), ctypes.c_size_t(4096), ctypes.c_uint(0x1))  # fine-grained
    name = "split: request in fine-grained device memory, answer in host memory"
    if rc == 0:
        req = (ctypes.c_uint64 * 1).from_address(dreq.value)
        res[name] = []
        try:
            for _ in range(a.rounds):
                req[0] = 0
                w[0] = w[1] = w[2] = w[3] = 0
                assert v.sosxv_ping_split_launch(dreq, ctl, ctypes.c_longlong(200_000_000), sp) == 0
                req[0] = 1
                t0 = time.perf_counter()
                while w[0] != 1:
                    if time.perf_counter() - t0 > 5:
                        raise SystemExit("split resident kernel did not answer")
                t0 = time.perf_counter()
                for k in range(2, a.iters + 2):
                    req[0] = k
                    while w[0] != k:
                        pass
                res[name].append((time.perf_counter() - t0) / a.iters * 1e6)
                req[0] = 0xFFFFFFFFFFFFFFFF
                HIP.hipStreamSynchronize(sp)
        except Exception as e:  # host access to the allocation refused
            res[name] = [float("nan")]
            print(f"split leg failed: {e}", file=sys.stderr)
    out = {k: {"median_us": round(statistics.median(x), 3), "rounds_us": [round(t, 3) for t in x]}
           for k, x in res.items()}
    print(json.dumps({"what": "host us per request/answer round trip through a resident kernel "
                      "(pinned coherent words, one polling lane)", "iters": a.iters, "legs": out}))


if __name__ == "__main__":
    main()
