"""Host-side cost of the completion primitives the p2p executor uses (one process, one GPU).

Times, per iteration (median of `--rounds` interleaved rounds of `--iters` each):
  launch+stream_sync   one 1-element sosx_combine, hipStreamSynchronize
  launch+sync_plain    the same, an event with default flags recorded + hipEventSynchronize
  launch+sync_system   the same with a hipEventReleaseToSystem event (runtime.cpp sync_system)
  launch x2+sys+sync   two combines with a system-release event between them (a queued
                       release ahead of a post), then hipStreamSynchronize
  release_only+sync    a system-release event on an idle stream + hipEventSynchronize
  other waits          a system-release event then hipStreamSynchronize / a hipEventQuery
                       spin; a hipStreamQuery spin; a flag kernel (k_p2p_signal storing a
                       sequence number to pinned host memory, system scope) after the
                       release event, polled by the host
  dirty L2 variants    the same after a 64 MiB combine left its output in L2 (not timed)
Usage: python tools/sync_cost.py [--iters 2000] [--rounds 5]
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

from sos_amd import _lib as L  # noqa: E402

HIP = ctypes.CDLL("libamdhip64.so.7")
EV_DEFAULT, EV_DISABLE_TIMING, EV_RELEASE_SYSTEM = 0x0, 0x2, 0x80000000


def ev(flags):
    e = ctypes.c_void_p()
    assert HIP.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(flags)) == 0
    return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    lib = L.lib()
    s = torch.cuda.Stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    x = torch.ones(1 << 24, device="cuda")
    y = torch.ones(1 << 24, device="cuda")
    big_a = torch.ones(1 << 24, device="cuda")
    big_b = torch.ones(1 << 24, device="cuda")
    torch.cuda.synchronize()
    e_plain, e_sys = ev(EV_DISABLE_TIMING), ev(EV_DISABLE_TIMING | EV_RELEASE_SYSTEM)
    op, dt = L.OPS["sum"], L.DTYPES["float"]

    def k():
        assert lib.sosx_combine(op, dt, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                ctypes.c_size_t(1), sp) == 0

    def dirty():
        assert lib.sosx_combine(op, dt, ctypes.c_void_p(big_a.data_ptr()), ctypes.c_void_p(big_b.data_ptr()),
                                ctypes.c_size_t(1 << 24), sp) == 0
        HIP.hipStreamSynchronize(sp)

    def stream_sync():
        k()
        HIP.hipStreamSynchronize(sp)

    def sync_plain():
        k()
        HIP.hipEventRecord(e_plain, sp)
        HIP.hipEventSynchronize(e_plain)

    def sync_system():
        k()
        HIP.hipEventRecord(e_sys, sp)
        HIP.hipEventSynchronize(e_sys)

    def two_with_release():
        k()
        HIP.hipEventRecord(e_sys, sp)
        k()
        HIP.hipStreamSynchronize(sp)

    def two_plain():
        k()
        k()
        HIP.hipStreamSynchronize(sp)

    def sys_then_stream_sync():
        k()
        HIP.hipEventRecord(e_sys, sp)
        HIP.hipStreamSynchronize(sp)

    def sys_then_query_spin():
        k()
        HIP.hipEventRecord(e_sys, sp)
        while HIP.hipEventQuery(e_sys) != 0:
            pass

    def stream_query_spin():
        k()
        while HIP.hipStreamQuery(sp) != 0:
            pass

    # a host-pinned word the GPU stores with a system-scope release (k_p2p_signal), polled
    # by the host: completion without the runtime's wait
    flag = ctypes.c_void_p()
    assert HIP.hipHostMalloc(ctypes.byref(flag), ctypes.c_size_t(64), ctypes.c_uint(0)) == 0
    word = (ctypes.c_uint64 * 1).from_address(flag.value)
    word[0] = 0
    sig = lib.sosx_p2p_signal
    sig.restype = ctypes.c_int
    sig.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]
    waddr = (ctypes.c_void_p * 1)(flag.value)
    wval = (ctypes.c_uint64 * 1)(0)
    seq = [0]

    def post_flag():
        seq[0] += 1
        wval[0] = seq[0]
        assert sig(1, waddr, wval, 0, None, None, None, 0, sp) == 0

    def wait_flag():
        while word[0] < seq[0]:
            pass

    def flag_after_release():
        k()
        HIP.hipEventRecord(e_sys, sp)
        post_flag()
        wait_flag()

    def flag_only():
        k()
        post_flag()
        wait_flag()

    def release_only():
        HIP.hipEventRecord(e_sys, sp)
        HIP.hipEventSynchronize(e_sys)

    legs = {"launch+stream_sync": (stream_sync, None), "launch+sync_plain": (sync_plain, None),
            "launch+sync_system": (sync_system, None), "launch x2+stream_sync": (two_plain, None),
            "launch x2, system release between": (two_with_release, None),
            "release_only+sync": (release_only, None),
            "launch+system event+hipStreamSynchronize": (sys_then_stream_sync, None),
            "launch+system event+hipEventQuery spin": (sys_then_query_spin, None),
            "launch+hipStreamQuery spin": (stream_query_spin, None),
            "launch+system event+flag kernel, host polls the flag": (flag_after_release, None),
            "launch+flag kernel, host polls the flag": (flag_only, None),
            "dirty L2 (64 MiB combine before), launch+stream_sync": (stream_sync, dirty),
            "dirty L2 (64 MiB combine before), launch+sync_system": (sync_system, dirty)}
    res = {n: [] for n in legs}
    for _ in range(a.rounds):
        for name, (fn, pre) in legs.items():
            for _ in range(50):
                fn()
            if pre is None:
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    fn()
                res[name].append((time.perf_counter() - t0) / a.iters * 1e6)
            else:
                tot = 0.0
                n = max(20, a.iters // 20)
                for _ in range(n):
                    pre()
                    t0 = time.perf_counter()
                    fn()
                    tot += time.perf_counter() - t0
                res[name].append(tot / n * 1e6)
    out = {name: {"median_us": round(statistics.median(v), 2), "rounds_us": [round(t, 2) for t in v]}
           for name, v in res.items()}
    print(json.dumps({"what": "host us per iteration, one process on one GPU, 1-element sosx_combine launches",
                      "iters": a.iters, "rounds": a.rounds, "legs": out}, indent=1))


if __name__ == "__main__":
    main()
