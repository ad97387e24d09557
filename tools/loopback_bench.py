"""Team-reduction kernels at the headline size on ONE GPU (loopback transport).

P simulated PEs, nreduce elements each, all resident in one MI355X's HBM; runs the
exact per-PE plans of the RCCL executor with device-to-device copies standing in for
xGMI.  Reports the fused fold kernel's HBM rate (HIP events via sosx_prof_*) and the
bit-exactness of the result against an on-GPU schedule-order re-evaluation.
Run under `rocprofv3 --kernel-trace --stats` for the per-kernel summary.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--n", type=int, default=128 << 20)
    ap.add_argument("--alg", default="ring")
    ap.add_argument("--dtype", default="float")
    ap.add_argument("--op", default="sum")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--fold-ab", action="store_true",
                    help="interleaved A/B of the 8-input fold shapes (tools/variants) on P "
                         "resident chunks of n/P elements")
    ap.add_argument("--prefix-ab", action="store_true",
                    help="interleaved A/B of the scan prefix shapes (tools/variants) "
                         "on P resident chunks of n/P elements")
    a = ap.parse_args()
    if a.fold_ab:
        return fold_ab(a)
    if a.prefix_ab:
        return prefix_ab(a)
    import torch
    from sos_amd import _lib as L
    from sos_amd import shmem as S
    torch.cuda.set_device(0)
    dt, op = L.dtype_id(a.dtype), L.op_id(a.op)
    es = L.dtype_size(dt)
    dist = L.DIST_PROD if a.op == "prod" else L.DIST_UNIFORM
    srcs = [torch.empty(a.n * es, dtype=torch.uint8, device="cuda") for _ in range(a.P)]
    dsts = [torch.empty(a.n * es, dtype=torch.uint8, device="cuda") for _ in range(a.P)]
    for p, b in enumerate(srcs):
        L.fill(dt, dist, 0x5EED, p, b.data_ptr(), a.n)
    torch.cuda.synchronize()
    sp, dp = [b.data_ptr() for b in srcs], [b.data_ptr() for b in dsts]
    S.loopback_allreduce(a.alg, op, dt, sp, dp, a.n)  # warm-up
    S.prof_enable(True)
    t0 = time.perf_counter()
    for _ in range(a.iters):
        S.loopback_allreduce(a.alg, op, dt, sp, dp, a.n)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    prof = S.prof_get()
    S.prof_enable(False)
    # check PE 0 against a direct schedule-order fold
    exp = torch.empty_like(dsts[0])
    if a.alg == "ring":
        q, r = divmod(a.n, a.P)
        for c in range(a.P):
            cnt = q + (c < r)
            first = c * cnt if c < r else c * cnt + r
            L.fold(op, dt, L.ORDER_LINEAR, exp.data_ptr() + first * es,
                   [sp[(c + k) % a.P] + first * es for k in range(a.P)], cnt)
    else:
        L.fold(op, dt, L.ORDER_TREE, exp.data_ptr(), sp, a.n)
    torch.cuda.synchronize()
    bad = L.count_mismatch(exp.data_ptr(), dp[0], a.n, es)
    nf = max(prof["nfold"], 1)
    fold_ms = prof["fold_ms"] / nf
    chunk = a.n // a.P
    fold_bytes = (a.P + 1) * chunk * es if a.alg in ("ring", "recdbl_direct") else 3 * (a.n // 2) * es
    out = {"P": a.P, "n": a.n, "alg": a.alg, "fold_launches": prof["nfold"],
           "fold_mean_ms": round(fold_ms, 5),
           "fold_GBs": round(fold_bytes / (fold_ms / 1e3) / 1e9, 1),
           "fold_frac_of_8TBs": round(fold_bytes / (fold_ms / 1e3) / 1e9 / 8000.0, 4),
           "wall_ms_per_allreduce_all_PEs": round((t1 - t0) / a.iters * 1e3, 3),
           "mismatches_pe0": bad}
    print(json.dumps(out))


def fold_ab(a, rounds=9, reps=20):
    """Interleaved A/B of the fold variants.  As in prefix_ab, every round draws a fresh
    buffer layout (each buffer a random number of 4 KiB pages into its allocation) and
    the variants are timed on it; reports the median and range over layouts."""
    import random
    import torch
    from sos_amd import _lib as L
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "variants"))
    import variants as V
    torch.cuda.set_device(0)
    a.P, a.dtype, a.op = 8, "float", "sum"      # the variant library's fold: 8 inputs, fp32 sum
    dt = L.dtype_id(a.dtype)
    es = L.dtype_size(dt)
    chunk = a.n // a.P
    names = V.names("fold")
    rng = random.Random(99)
    res = {v: [] for v in range(len(names))}
    same = True
    pages = 64
    for _ in range(rounds):
        bufs = [torch.empty(chunk * es + pages * 4096, dtype=torch.uint8, device="cuda")
                for _ in range(a.P + 1)]
        ptrs = [b.data_ptr() + rng.randrange(pages) * 4096 for b in bufs]
        ins, out = ptrs[:a.P], ptrs[a.P]
        for k, x in enumerate(ins):
            L.fill(dt, 0, 0x5EED, k, x, chunk)
        ref = None
        for v in range(len(names)):
            for _ in range(3):
                V.fold(v, out, ins, chunk)
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(reps):
                V.fold(v, out, ins, chunk)
            s1.record()
            torch.cuda.synchronize()
            res[v].append(s0.elapsed_time(s1) / reps)
            last = bufs[-1].clone()
            if ref is None:
                ref = last
            else:
                same &= torch.equal(ref, last)
        del bufs, ref, last
    algo = (a.P + 1) * chunk * es
    rows = {}
    for v, name in enumerate(names):
        ms = sorted(res[v])
        rows[name] = {"median_ms": round(ms[len(ms) // 2], 5),
                      "GBs": round(algo / (ms[len(ms) // 2] / 1e3) / 1e9, 1),
                      "GBs_range": [round(algo / (ms[-1] / 1e3) / 1e9, 1),
                                    round(algo / (ms[0] / 1e3) / 1e9, 1)]}
    print(json.dumps({"fold_ab": rows, "P": a.P, "chunk": chunk, "bytes": algo,
                      "layouts": rounds, "variants_bit_identical": same}))


def prefix_ab(a, rounds=9, reps=20):
    """Every round draws a fresh buffer layout (each of the 2P buffers starts a random
    number of 4 KiB pages into its allocation), since the relative placement of 16
    concurrent streams moves the rate by several percent; the variants are then timed
    interleaved on that layout.  Reports the median and range over layouts."""
    import random
    import torch
    from sos_amd import _lib as L
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "variants"))
    import variants as V
    torch.cuda.set_device(0)
    a.dtype, a.op = "float", "sum"              # the variant library's prefix: fp32 sum
    dt = L.dtype_id(a.dtype)
    es = L.dtype_size(dt)
    chunk = a.n // a.P
    names = V.names("prefix")
    rng = random.Random(1234)
    res = {v: [] for v in range(len(names))}
    same = True
    pages = 64
    for _ in range(rounds):
        bufs = [torch.empty(chunk * es + pages * 4096, dtype=torch.uint8, device="cuda")
                for _ in range(2 * a.P)]
        ptrs = [b.data_ptr() + rng.randrange(pages) * 4096 for b in bufs]
        ip, op_ = ptrs[:a.P], ptrs[a.P:]
        for k, x in enumerate(ip):
            L.fill(dt, 0, 0x5EED, k, x, chunk)
        ref = None
        for v in range(len(names)):
            for _ in range(3):
                V.prefix(v, op_, ip, chunk)
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(reps):
                V.prefix(v, op_, ip, chunk)
            s1.record()
            torch.cuda.synchronize()
            res[v].append(s0.elapsed_time(s1) / reps)
            last = bufs[-1].clone()  # the final output (holds every input's contribution)
            if ref is None:
                ref = last
            else:
                same &= torch.equal(ref, last)
        del bufs, ref, last
    algo = 2 * a.P * chunk * es
    rows = {}
    for v, name in enumerate(names):
        ms = sorted(res[v])
        rows[name] = {"median_ms": round(ms[len(ms) // 2], 5),
                      "GBs": round(algo / (ms[len(ms) // 2] / 1e3) / 1e9, 1),
                      "GBs_range": [round(algo / (ms[-1] / 1e3) / 1e9, 1),
                                    round(algo / (ms[0] / 1e3) / 1e9, 1)]}
    print(json.dumps({"prefix_ab": rows, "P": a.P, "chunk": chunk, "bytes": algo,
                      "layouts": rounds, "variants_bit_identical": same}))

if __name__ == "__main__":
    main()
