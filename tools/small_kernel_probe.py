"""Device-side duration of the small host-resident path's kernel (bench only; run under
rocprofv3 --kernel-trace --stats): sosx_small_fold over P operands of n floats in pinned
host memory, result to pinned memory, `calls` launches each followed by a device
synchronisation.  The rocprof average is the kernel's own time (its PCIe reads and
write-back); the host-side call time minus it is launch + completion overhead
(DESIGN.md section 7).  --stage times the device-operand copy kernel (sosx_small_stage)
the same way."""
import argparse
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=2)
    ap.add_argument("--n", type=int, default=1)
    ap.add_argument("--calls", type=int, default=500)
    ap.add_argument("--stage", action="store_true",
                    help="time sosx_small_stage instead: n floats from HBM into a pinned slot + P-1 posts")
    a = ap.parse_args()
    import torch
    from sos_amd import _lib as L
    torch.cuda.set_device(0)
    lib = L.lib()
    if a.stage:
        src = torch.full((max(a.n, 4),), 2.5, dtype=torch.float32, device="cuda")
        slot = torch.zeros(max(a.n, 4), dtype=torch.float32, pin_memory=True)
        words = torch.zeros(8 * 64, dtype=torch.int64, pin_memory=True)
        wp = (ctypes.c_void_p * (a.P - 1))(*[words.data_ptr() + 64 * k for k in range(a.P - 1)])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.calls):
            vals = (ctypes.c_uint64 * (a.P - 1))(*([k + 1] * (a.P - 1)))
            rc = lib.sosx_small_stage(ctypes.c_void_p(slot.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                      ctypes.c_size_t(4 * a.n), wp, vals, a.P - 1, None)
            assert rc == 0
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.calls
        assert float(slot[0]) == 2.5 and int(words[0]) == a.calls
        print(f"stage P={a.P} n={a.n}: {dt * 1e6:.2f} us per launch + synchronize (host clock)", flush=True)
        return
    ins = [torch.full((max(a.n, 4),), 1.0 + p, dtype=torch.float32, pin_memory=True) for p in range(a.P)]
    out = torch.zeros(max(a.n, 4), dtype=torch.float32, pin_memory=True)
    flags = torch.zeros(4096 + 8, dtype=torch.int32, pin_memory=True)
    p2 = 1 << (a.P.bit_length() - 1)
    leaves = (ctypes.c_void_p * p2)(*[ins[y].data_ptr() for y in range(p2)])
    extras = (ctypes.c_void_p * p2)(*[ins[y + p2].data_ptr() if y + p2 < a.P else None for y in range(p2)])
    nb = ctypes.c_int(0)
    t0 = time.perf_counter()
    for k in range(a.calls):
        rc = lib.sosx_small_fold(5, 23, ctypes.c_void_p(out.data_ptr()), leaves, extras, p2,
                                 ctypes.c_size_t(a.n), ctypes.c_void_p(flags.data_ptr()),
                                 ctypes.c_uint32(k + 1), ctypes.byref(nb), None)
        assert rc == 0
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.calls
    assert float(out[0]) == float(sum(1.0 + p for p in range(a.P)))
    print(f"P={a.P} n={a.n}: {dt * 1e6:.2f} us per launch + synchronize (host clock)", flush=True)


if __name__ == "__main__":
    main()
