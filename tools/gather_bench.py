"""The p2p transport's multi-segment gather kernel (sosx_gather, copy.hip k_gather) on ONE
GPU: the allgather round of an 8-PE ring at the headline size -- 7 segments of
nreduce/8 fp32 elements (64 MiB each at 128Mi) copied in one launch -- against the HIP
runtime's own device-to-device copies of the same segments (hipMemcpyAsync, one per
segment).  On the 8-GPU node the segments come from 7 peers' HBM over xGMI; here they are
local HBM, so this measures the kernel's own copy rate (2 x bytes / time vs 8 TB/s).
Also checks the copies byte for byte.  Run under `rocprofv3 --kernel-trace --stats` for
the per-kernel summary."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128 << 20, help="nreduce (fp32 elements per PE)")
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--src-offset", type=int, default=0,
                    help="bytes past a 16-B boundary for every source (incongruent with the "
                         "destinations when not a multiple of 16)")
    a = ap.parse_args()
    import torch
    from sos_amd import _lib as L
    torch.cuda.set_device(0)
    seg = a.n // a.P * 4
    nseg = a.P - 1
    off = a.src_offset
    srcbuf = [torch.empty(seg + 64, dtype=torch.uint8, device="cuda") for _ in range(nseg)]
    src = [b[off:off + seg] for b in srcbuf]
    dst = [torch.empty(seg, dtype=torch.uint8, device="cuda") for _ in range(nseg)]
    for k, b in enumerate(src):
        L.fill(L.dtype_id("float"), L.DIST_UNIFORM, 0x5EED, k, b.data_ptr(), seg // 4)
    torch.cuda.synchronize()
    S = (ctypes.c_void_p * nseg)(*[b.data_ptr() for b in src])
    D = (ctypes.c_void_p * nseg)(*[b.data_ptr() for b in dst])
    B = (ctypes.c_size_t * nseg)(*([seg] * nseg))
    stream = torch.cuda.current_stream().cuda_stream

    def gather():
        L.check(L.lib().sosx_gather(nseg, S, D, B, stream), "sosx_gather")

    def runtime_copy():
        for s_, d_ in zip(src, dst):
            d_.copy_(s_, non_blocking=True)

    out = {"P": a.P, "segments": nseg, "segment_bytes": seg, "src_offset": off,
           "bytes_moved_per_launch": 2 * nseg * seg}
    for name, fn in (("k_gather", gather), ("runtime_d2d_copies", runtime_copy)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        out[name] = {"ms": round(ms, 5), "GBs": round(2 * nseg * seg / (ms / 1e3) / 1e9, 1),
                     "frac_of_hbm_peak": round(2 * nseg * seg / (ms / 1e3) / 1e9 / 8000.0, 4)}
    for d_ in dst:
        d_.zero_()
    gather()
    torch.cuda.synchronize()
    out["bitwise_equal"] = all(torch.equal(s_, d_) for s_, d_ in zip(src, dst))
    print(json.dumps(out))
    return 0 if out["bitwise_equal"] else 1


if __name__ == "__main__":
    sys.exit(main())
