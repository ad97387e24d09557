#!/usr/bin/env python3
"""bench.py -- SOS team-reduction path (shmem_<T>_<op>_reduce) on MI355X.

Metric (BASELINE.json): GiB/s of the device-resident sum_reduce combine,
nreduce = 128Mi fp32, at 1/2/4/8 GPUs (one PE per GPU).

  N = 1 : one step = one local combine inout = inout + in over 128Mi fp32 resident in
          HBM (sosx_combine, the device shmem_internal_reduce_local,
          src/shmem_internal_op.h:305-339).  At PE_size 1 the reference API itself
          only copies (src/collectives.c:664-668), so the combine kernel is the
          single-GPU workload.
  N > 1 : one step = one shmem_float_sum_reduce(SHMEM_TEAM_WORLD, dest, src, 128Mi)
          over N PEs (weak scaling: every PE reduces its own 128Mi vector).
  value = sum over PEs of nreduce*sizeof(T) bytes reduced per step / step time, GiB/s.

One JSON line on rank 0's stdout.  `roofline` is the dominant kernel's algorithmic
HBM bytes per launch / its HIP-event-timed mean duration; `cpu_baseline` is the CPU
restatement of reduce_local (oracle/sos_oracle.c, gcc -O2, one core) on a bounded
sample of the same workload.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu] [--sweep]
       torchrun --nproc-per-node N bench.py --gpus N   (N > 1)
       python bench.py --gpus N   (N > 1, no launcher: bench.py starts the N rank
                                   processes itself and prints rank 0's line)
--gpus N must equal the launcher's WORLD_SIZE when there is one (exit 2 otherwise).
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

GiB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level table)
SEED = 0x5EED


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--nreduce", type=int, default=128 << 20, help="nreduce (elements per PE)")
    p.add_argument("--dtype", default="float")
    p.add_argument("--op", default="sum")
    p.add_argument("--alg", default=os.environ.get("SHMEM_REDUCE_ALGORITHM", "auto"))
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-pmc", action="store_true")
    p.add_argument("--no-host", action="store_true", help="skip the host-resident leg")
    p.add_argument("--no-small", action="store_true",
                   help="N > 1: skip the small-message leg (library vs SOS's CPU path)")
    p.add_argument("--no-adjacent", action="store_true",
                   help="skip the scan/broadcast legs (prefix kernel at N=1, team calls at N>1)")
    p.add_argument("--team", action="store_true",
                   help="run the team (shmem_*_reduce) leg even at WORLD_SIZE 1")
    p.add_argument("--sweep", action="store_true",
                   help="SURVEY 8(d) config #5 roofline scan of the combine kernel instead of "
                        "the headline line (N=1)")
    p.add_argument("--sweep-pairs", default="configs",
                   help="'configs' (SURVEY 8(d) #2/#3/#5) or 'all' (every datatype class)")
    p.add_argument("--sweep-min", type=int, default=1 << 10)
    p.add_argument("--sweep-max", type=int, default=256 << 20,
                   help="largest nreduce of the N=1 sweep and of the N>1 size curve")
    p.add_argument("--no-team-sweep", action="store_true",
                   help="N>1: skip the nreduce 1Mi..256Mi size curve")
    p.add_argument("--no-curve", action="store_true",
                   help="N=1: skip the nreduce 1Mi..256Mi combine curve (with its CPU column)")
    p.add_argument("--pmc-save", default=None,
                   help="N=1: also copy the raw PMC CSVs into this directory")
    p.add_argument("--fold-p", type=int, default=8,
                   help="inputs of the fold / prefix kernel legs (one PE's chunk of a P-PE call)")
    p.add_argument("--child-pmc", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--launch-check", action="store_true",
                   help="N > 1 plumbing only: gloo group + rank 0 prints the ranks (no GPU)")
    a = p.parse_args()
    a.n = a.nreduce
    return a


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------------
# N = 1: the local combine
# ----------------------------------------------------------------------------------
class DevBuf:
    """A device buffer: from the library's device symmetric heap (shmemx_malloc_device,
    where an SOS program keeps device-resident symmetric data) or from torch's caching
    allocator.  .ptr is the device address."""

    def __init__(self, torch, nbytes, heap):
        self.heap = heap
        if heap:
            from sos_amd import shmem as SH
            self.ptr = SH.shmemx_malloc_device(nbytes)
            self.t = None
        else:
            self.t = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
            self.ptr = self.t.data_ptr()

    def free(self):
        if self.heap and self.ptr:
            from sos_amd import shmem as SH
            SH.lib().shmemx_free_device(self.ptr)
        self.ptr, self.t = 0, None


_SHMEM_UP = False


def shmem_up(args):
    """shmem_init() for the N = 1 legs (one PE): the device symmetric heap holds their
    operands.  The heap is sized for the largest leg (the combine's two operands, or the
    prefix's 2P chunks) plus its stage region."""
    global _SHMEM_UP
    if _SHMEM_UP:
        return
    from sos_amd import _lib as L
    from sos_amd import shmem as SH
    es = L.dtype_size(L.dtype_id(args.dtype))
    os.environ.setdefault("SHMEMX_STAGE_BYTES", str(64 << 20))
    big = max(2 * args.n * es, 2 * max(CURVE_SIZES) * es, ROTATE_BYTES)
    os.environ.setdefault("SHMEMX_DEVICE_HEAP_SIZE", str(big + (512 << 20)))
    SH.shmem_init()
    _SHMEM_UP = True


def combine_setup(args, torch, S, heap=True):
    from sos_amd import _lib as L
    dt = L.dtype_id(args.dtype)
    es = L.dtype_size(dt)
    nbytes = args.n * es
    if heap:
        shmem_up(args)
    a, b = DevBuf(torch, nbytes, heap), DevBuf(torch, nbytes, heap)
    dist = L.DIST_PROD if args.op == "prod" else L.DIST_UNIFORM
    L.fill(dt, dist, SEED, 0, a.ptr, args.n, 0, S)
    L.fill(dt, dist, SEED, 1, b.ptr, args.n, 0, S)
    torch.cuda.synchronize()
    return L, dt, es, a, b


def time_combine(args, torch, heap):
    """The combine on a fresh operand pair, timed like the headline: (mean HIP-event ms
    over K back-to-back launches, the pair's start-to-start distance in bytes)."""
    stream = torch.cuda.current_stream()
    S = stream.cuda_stream
    L, dt, es, a, b = combine_setup(args, torch, S, heap)
    op = L.op_id(args.op)
    for _ in range(args.warmup):
        L.combine(op, dt, a.ptr, b.ptr, args.n, S)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(args.steps):
        L.combine(op, dt, a.ptr, b.ptr, args.n, S)
    e1.record(stream)
    torch.cuda.synchronize()
    dist_b = b.ptr - a.ptr
    a.free()
    b.free()
    return e0.elapsed_time(e1) / args.steps, dist_b


def run_combine(args, torch):
    stream = torch.cuda.current_stream()
    S = stream.cuda_stream
    L, dt, es, a, b = combine_setup(args, torch, S)
    op = L.op_id(args.op)
    launch = lambda: L.combine(op, dt, a.ptr, b.ptr, args.n, S)  # noqa: E731

    if args.child_pmc:  # profiled child: a few launches of each measured kernel only
        for _ in range(args.warmup + args.steps):
            launch()
        torch.cuda.synchronize()
        a.free()
        b.free()
        for kind in ("fold", "prefix"):
            ms_launch, _, _, keep = multi_stream_setup(args, torch, kind)
            for _ in range(args.warmup + args.steps):
                ms_launch()
            torch.cuda.synchronize()
            for x in keep:
                x.free()
        return None

    for _ in range(args.warmup):
        launch()
    torch.cuda.synchronize()
    # Timed region: the K launches back to back on the library's stream, bracketed by two
    # HIP events (and the host clock).  Per-launch event pairs would add two queue
    # packets to every step; the span / K is the per-launch duration INCLUDING the
    # dependent-launch boundary, so `achieved` is conservative against rocprof's
    # kernel-only average.
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    mean_kern_s = e0.elapsed_time(e1) / args.steps / 1e3
    step_s = (t1 - t0) / args.steps
    # per-launch event pairs, after the timed region: the kernel-only median
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(min(args.steps, 20))]
    for s_, e_ in ev:
        s_.record(stream)
        launch()
        e_.record(stream)
    torch.cuda.synchronize()
    kern_ms = sorted(s_.elapsed_time(e_) for s_, e_ in ev)
    dist_ab = b.ptr - a.ptr
    a.free()
    b.free()
    # the same kernel on a pair from torch's caching allocator (2 MiB-aligned blocks), for
    # comparison: the placement of a caller's own buffers is the caller's
    torch_ms, torch_dist = time_combine(args, torch, heap=False)
    payload = args.n * es
    algo_bytes = 3 * payload  # read in, read inout, write inout
    achieved = algo_bytes / mean_kern_s / 1e9
    res = {
        "metric": "GiB/s device-resident sum_reduce combine, nreduce=128Mi fp32; 1/2/4/8 GPU",
        "value": round(payload / step_s / GiB, 3),
        "unit": "GiB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {"float": "f32", "double": "f64"}.get(args.dtype, args.dtype),
        "data": "synthetic (splitmix64 counter hash, SURVEY.md 8(d)), resident in HBM",
        "config": {"workload": f"shmem_{args.dtype}_{args.op}_reduce local combine "
                               f"(reduce_local inout OP= in), nreduce={args.n}, 1 PE",
                   "nreduce": args.n, "op": args.op, "type": args.dtype},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None,
                     "kernel": "sos::k_combine3", "algorithmic_bytes_per_launch": algo_bytes,
                     "mean_kernel_ms": round(mean_kern_s * 1e3, 5),
                     "mean_kernel_ms_how": "HIP-event span of the timed region / steps",
                     "median_kernel_ms": round(kern_ms[len(kern_ms) // 2], 5),
                     "median_kernel_ms_how": "per-launch HIP event pairs, after the timed region"},
        "operands": {"where": "device symmetric heap (shmemx_malloc_device), one PE",
                     "in_minus_inout_bytes": dist_ab,
                     "in_minus_inout_mod_32KiB": dist_ab % 32768,
                     "note": "the heap starts large allocations an odd multiple of 4 KiB apart "
                             "in HBM's 32 KiB channel interleave (DESIGN.md section 3, "
                             "profiles/r4_offset_probe.txt)"},
        "torch_allocator_buffers": {
            "mean_kernel_ms": round(torch_ms, 5),
            "achieved_GBs": round(algo_bytes / (torch_ms / 1e3) / 1e9, 1),
            "frac": round(algo_bytes / (torch_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "in_minus_inout_bytes": torch_dist,
            "in_minus_inout_mod_32KiB": torch_dist % 32768,
            "note": "the same kernel and timing on two torch.empty buffers (the caller's "
                    "placement, not the heap's): reported, never `value`"},
    }
    return res


def host_resident(args, torch):
    """The same combine when inout/in start and end in HOST memory (the SOS symmetric
    heap is host memory): H2D of both operands, the device combine, D2H of inout.
    Reported beside `value` (never as it): the PCIe-inclusive end-to-end rate."""
    from sos_amd import _lib as L
    dt = L.dtype_id(args.dtype)
    es = L.dtype_size(dt)
    n = args.n
    stream = torch.cuda.current_stream()
    S = stream.cuda_stream
    out = {}
    da = torch.empty(n * es, dtype=torch.uint8, device="cuda")
    db = torch.empty_like(da)
    lib = L.lib()
    for kind in ("pinned", "pageable"):
        ha = torch.empty(n * es, dtype=torch.uint8, pin_memory=(kind == "pinned"))
        hb = torch.empty(n * es, dtype=torch.uint8, pin_memory=(kind == "pinned"))
        ha.fill_(0)
        hb.fill_(0)
        reps = 5
        # serial: copy both in, combine, copy out
        for r in range(reps + 1):
            if r == 1:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            da.copy_(ha, non_blocking=True)
            db.copy_(hb, non_blocking=True)
            L.combine(args.op, dt, da.data_ptr(), db.data_ptr(), n, S)
            ha.copy_(da, non_blocking=True)
            torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        out[f"{kind}_serial_GiBs"] = round(n * es / t / GiB, 3)
        # pipelined: sosx_combine_host (what shmemx_reduce_local does for host operands)
        for r in range(reps + 1):
            if r == 1:
                t0 = time.perf_counter()
            L.check(lib.sosx_combine_host(L.op_id(args.op), dt, ha.data_ptr(), hb.data_ptr(), n, 0),
                    "sosx_combine_host")
        t = (time.perf_counter() - t0) / reps
        out[f"{kind}_pipelined_GiBs"] = round(n * es / t / GiB, 3)
        out[f"{kind}_pipelined_ms"] = round(t * 1e3, 3)
        del ha, hb
    out["static_data"] = static_data_row(args)
    out["bytes_moved_per_call"] = {"H2D": 2 * n * es, "D2H": n * es}
    out["note"] = ("payload GiB/s of reduce_local on host-resident operands through the GPU: "
                   "H2D(inout, in) + combine + D2H(inout); serial vs 3-stream chunk pipeline "
                   "(sosx_combine_host); static_data: the same pipeline on two static arrays of "
                   "an SOS-style C program (examples/static_reduce.c), whose data segment "
                   "shmem_init registers with HIP as SOS registers it (src/init.c:341-346); "
                   "PCIe Gen5 x16 = 63 GB/s per direction (spec)")
    return out


def static_data_row(args):
    """shmemx_reduce_local on STATIC symmetric arrays: examples/static_reduce (a C program,
    fp32 sum only, at most 128Mi elements) run as a child process on the same GPU."""
    exe = os.path.join(HERE, "examples", "static_reduce")
    if args.dtype != "float" or args.op != "sum" or args.n > (128 << 20):
        return {"skipped": "examples/static_reduce covers fp32 sum up to 128Mi elements"}
    if not os.path.exists(exe):
        return {"skipped": "examples/static_reduce not built (make -C examples)"}
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
              "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    try:
        r = subprocess.run([exe, "local", str(args.n), "5"], capture_output=True, text=True,
                           timeout=300, env=env)
        row = json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001  (reported in the line, never fatal for the bench)
        return {"error": f"{type(e).__name__}: {e}"}
    if r.returncode != 0 or row.get("wrong"):
        row["error"] = f"exit {r.returncode}: {r.stderr[-300:]}"
    return row


def multi_stream_setup(args, torch, kind):
    """P resident input chunks of nreduce/P elements (one PE's share of a P-PE team call)
    and the launch of the team path's local step on them:
      fold   : sosx_fold LINEAR (the ring's fused P-way combine), 1 output,
               algorithmic HBM bytes (P + 1) * chunk * sizeof(T);
      prefix : sosx_prefix (the scans' local step), P outputs, 2 * P * chunk * sizeof(T)."""
    from sos_amd import _lib as L
    P = args.fold_p     # default 8: one PE's chunk of an 8-PE call, the 8-GPU node's shape
    dt = L.dtype_id(args.dtype)
    es = L.dtype_size(dt)
    chunk = args.n // P
    S = torch.cuda.current_stream().cuda_stream
    dist = L.DIST_PROD if args.op == "prod" else L.DIST_UNIFORM
    shmem_up(args)
    # heap buffers: consecutive large allocations are 4 KiB apart in the channel
    # interleave, as the library's own scratch slots are (plan.cpp slot_stride)
    ins = [DevBuf(torch, chunk * es, True) for _ in range(P)]
    outs = [DevBuf(torch, chunk * es, True) for _ in range(P if kind == "prefix" else 1)]
    for k, x in enumerate(ins):
        L.fill(dt, dist, SEED, k, x.ptr, chunk, 0, S)
    ip, op_ = [x.ptr for x in ins], [x.ptr for x in outs]
    if kind == "prefix":
        launch = lambda: L.prefix("sum", dt, op_, ip, chunk, -1, S)  # noqa: E731
        algo = 2 * P * chunk * es
    else:
        launch = lambda: L.fold(args.op, dt, L.ORDER_LINEAR, op_[0], ip, chunk, S)  # noqa: E731
        algo = (P + 1) * chunk * es
    return launch, algo, chunk, ins + outs


def multi_stream_kernel(args, torch, kind):
    """One of the team path's multi-stream kernels at the headline size (see
    multi_stream_setup), timed like `roofline`: two HIP events around a batch of
    back-to-back launches on the stream they run on.  Reported beside `value`; `traffic`
    is filled from the PMC passes."""
    launch, algo, chunk, keep = multi_stream_setup(args, torch, kind)
    stream = torch.cuda.current_stream()
    for _ in range(3):
        launch()
    reps = max(args.steps // 2, 10)
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s0.record(stream)
    for _ in range(reps):
        launch()
    s1.record(stream)
    torch.cuda.synchronize()
    mean_s = s0.elapsed_time(s1) / reps / 1e3
    for x in keep:
        x.free()
    P = args.fold_p
    name = {"prefix": f"sos::k_prefix<NP={P}>", "fold": f"sos::k_fold<NP={P}, LINEAR>"}[kind]
    return {"kernel": name, "inputs": P, "elements_per_input": chunk,
            "algorithmic_bytes_per_launch": algo, "mean_kernel_ms": round(mean_s * 1e3, 5),
            "mean_kernel_ms_how": f"HIP-event span of {reps} back-to-back launches / {reps}",
            "achieved_GBs": round(algo / mean_s / 1e9, 1),
            "frac_of_hbm_peak": round(algo / mean_s / 1e9 / HBM_PEAK_GBS, 4), "traffic": None}


# config #5 (and #2, #3): (type, op) pairs of the roofline scan
SWEEP_ALL = [("char", "sum"), ("schar", "max"), ("short", "prod"), ("uchar", "xor"),
             ("ushort", "min"), ("uint", "sum"), ("long", "and"), ("ulong", "max"),
             ("ptrdiff", "sum"), ("size", "prod"), ("float", "max"), ("float", "prod"),
             ("complexf", "sum"), ("complexf", "prod"), ("longdouble", "sum"),
             ("longdouble", "max")]
SWEEP_PAIRS = [("int", "min"), ("int", "max"), ("int", "prod"),
               ("double", "min"), ("double", "max"), ("double", "prod"), ("double", "sum"),
               ("complexd", "prod"), ("complexd", "sum"),
               ("int64", "and"), ("int64", "or"), ("int64", "xor"),
               ("float", "sum")]


def sweep(args, torch):
    """Roofline scan of the local combine (sosx_combine) over nreduce = 1Ki * 4^k up to
    --sweep-max for every (type, op) of SURVEY 8(d) configs #2, #3 and #5.  Per point:
    the mean HIP-event kernel time over a batch of launches, algorithmic HBM GB/s
    (3 * n * sizeof(T) per launch) and its fraction of the 8 TB/s peak, and the host
    wall time per call (launch-bound at small n).  Parity at these sizes is
    tests/test_gpu_configs.py (bit-exact vs the oracle); here each point is checked
    against the fused fold kernel run on the same two inputs (an independent code path,
    sosx_fold with 2 inputs)."""
    from sos_amd import _lib as L
    stream = torch.cuda.current_stream()
    S = stream.cuda_stream
    sizes = []
    n = args.sweep_min
    while n <= args.sweep_max:
        sizes.append(n)
        n *= 4
    rows = []
    for tname, oname in (SWEEP_PAIRS if args.sweep_pairs == "configs" else SWEEP_ALL):
        dt, op = L.dtype_id(tname), L.op_id(oname)
        es = L.dtype_size(dt)
        dist = L.DIST_PROD if oname == "prod" else L.DIST_UNIFORM
        nmax = sizes[-1]
        a = torch.empty(nmax * es, dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        c = torch.empty_like(a)
        ld_src = None
        if tname == "longdouble":  # no device generator for x87 values: host-made, uploaded
            import numpy as np
            rng = np.random.default_rng(SEED)
            v = (rng.uniform(0.5, 2.0, (2, nmax)) if oname == "prod"
                 else rng.standard_normal((2, nmax))).astype(np.longdouble)
            ld_src = [torch.from_numpy(v[k].view(np.uint8).copy()).cuda() for k in range(2)]
        for n in sizes:
            if ld_src is not None:
                a[:n * es].copy_(ld_src[0][:n * es])
                b[:n * es].copy_(ld_src[1][:n * es])
            else:
                L.fill(dt, dist, SEED, 0, a.data_ptr(), n, 0, S)
                L.fill(dt, dist, SEED, 1, b.data_ptr(), n, 0, S)
            # check first: fold(a, b) -> c, then combine a OP= b, compare
            L.fold(op, dt, L.ORDER_LINEAR, c.data_ptr(), [a.data_ptr(), b.data_ptr()], n, S)
            L.combine(op, dt, a.data_ptr(), b.data_ptr(), n, S)
            bad = L.count_mismatch(a.data_ptr(), c.data_ptr(), n, es, S)
            reps = max(5, min(200, int(2e9 // (3 * n * es))))
            launch = lambda: L.combine(op, dt, a.data_ptr(), b.data_ptr(), n, S)  # noqa: E731
            for _ in range(3):
                launch()
            torch.cuda.synchronize()
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            s0.record(stream)
            for _ in range(reps):
                launch()
            s1.record(stream)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / reps
            kern = s0.elapsed_time(s1) / 1e3 / reps
            algo = 3 * n * es
            rows.append({"type": tname, "op": oname, "nreduce": n, "bytes_per_launch": algo,
                         "kernel_us": round(kern * 1e6, 3), "call_us": round(wall * 1e6, 3),
                         "GBs": round(algo / kern / 1e9, 1),
                         "frac_hbm": round(algo / kern / 1e9 / HBM_PEAK_GBS, 4),
                         "payload_GiBs": round(n * es / kern / GiB, 2),
                         "check_mismatches": int(bad)})
            log(f"{tname:>8} {oname:>4} n={n:>10} {kern * 1e6:10.2f} us "
                f"{algo / kern / 1e9:8.1f} GB/s  frac {algo / kern / 1e9 / HBM_PEAK_GBS:.3f}"
                f"  check {bad}")
        del a, b, c
    return {"sweep": "combine roofline scan, SURVEY 8(d) configs #2/#3/#5, 1 GPU",
            "peak_GBs": HBM_PEAK_GBS, "kernel": "sos::k_combine3 (sosx_combine)",
            "timing": "HIP events around a batch of back-to-back launches on one stream",
            "rows": rows}


# ----------------------------------------------------------------------------------
# PMC traffic: rocprofv3 --pmc pass(es) over a child run of this script
# ----------------------------------------------------------------------------------
PMC_KERNELS = {"combine": "sos::k_combine3<", "fold": "sos::k_fold<", "prefix": "sos::k_prefix<"}


def pmc_kernel_of(name):
    """Which measured kernel (PMC_KERNELS key) a rocprof Kernel_Name belongs to, or None."""
    for k, tag in PMC_KERNELS.items():
        if tag in name:
            return k
    return None


def pmc_traffic(args, save_dir=None):
    """HBM bytes per launch of each measured kernel (combine, fold, prefix) from TCC
    FETCH_SIZE / WRITE_SIZE (KiB units), one rocprofv3 --pmc pass per counter over a
    child run of this script (--child-pmc: a few launches of each kernel at the bench
    shapes).  gfx950: FETCH_SIZE counts half the bytes of a 16-B/lane streaming read
    (MI355X_MICROARCH.md, HBM), so reads = 2*FETCH_SIZE.  Separate passes, since
    FETCH_SIZE and WRITE_SIZE do not fit one TCC pass.  Returns ({kernel: bytes}, info)."""
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="sos_pmc_")
        cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--child-pmc", "--steps", "3",
               "--warmup", "1", "--nreduce", str(args.n), "--dtype", args.dtype, "--op", args.op,
               "--fold-p", str(args.fold_p)]
        try:
            env = {k: v for k, v in os.environ.items()
                   if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                                "GROUP_RANK", "ROLE_RANK")}   # the child is one process
            subprocess.run(cmd, check=True, timeout=240, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL, env=dict(env, TMPDIR="/tmp"))
        except Exception as exc:  # noqa: BLE001 - a profiler failure must not kill the bench
            shutil.rmtree(d, ignore_errors=True)
            return None, f"rocprofv3 {ctr} pass failed: {exc}"
        rows = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            if save_dir:
                os.makedirs(save_dir, exist_ok=True)
                shutil.copy(f, os.path.join(save_dir, f"pmc_{ctr}.csv"))
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = pmc_kernel_of(row.get("Kernel_Name", ""))
                    if k and row.get("Counter_Name") == ctr:
                        rows.setdefault(k, []).append(float(row["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if not rows:
            return None, f"no {ctr} rows"
        for k, v in rows.items():
            vals.setdefault(k, {})[ctr] = sum(v) / len(v)
    traffic = {k: (2.0 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024.0
               for k, v in vals.items() if len(v) == 2}
    return traffic, vals


# ----------------------------------------------------------------------------------
# CPU baseline: the restated reduce_local on one host core
# ----------------------------------------------------------------------------------
def cpu_baseline(args):
    import numpy as np
    from oracle import oracle as O
    from sos_amd import _lib as L
    dt = L.dtype_id(args.dtype)
    dist = L.DIST_PROD if args.op == "prod" else L.DIST_UNIFORM
    inout = O.fill(dt, dist, SEED, 0, args.n)
    inp = O.fill(dt, dist, SEED, 1, args.n)
    op = L.op_id(args.op)
    t = O.time_reduce_local(op, dt, inp, inout, 1)  # warm-up + per-rep estimate
    reps = max(1, int(args.cpu_seconds / max(t, 1e-6)))
    t = O.time_reduce_local(op, dt, inp, inout, reps)
    es = inout.itemsize
    del inout, inp
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        pass
    _ = np
    return {"value": round(reps * args.n * es / t / GiB, 3), "unit": "GiB/s", "cores": 1,
            "kind": "port",
            "sample": f"reduce_local({args.op}, {args.dtype}) n={args.n} x {reps} reps, "
                      f"{t:.1f} s, oracle/sos_oracle.c gcc -O2 (SOS default flags), 1 thread; "
                      f"host: {model}, nproc={os.cpu_count()}"}


CURVE_SIZES = (1 << 20, 4 << 20, 16 << 20, 64 << 20, 128 << 20, 256 << 20)
MALL_BYTES = 256 << 20         # MI355X Infinity Cache (MALL), chip total
ROTATE_BYTES = 1 << 30         # operand bytes a rotation cycles through per size point


GRAPH_MAX_BYTES = 64 << 20  # graph-replayed curve points: 1Mi..16Mi fp32


def time_launches(torch, stream, launches, reps):
    """Mean HIP-event time per launch of `reps` back-to-back calls of launches[i % len]."""
    for k in range(min(3, len(launches))):
        launches[k]()
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s0.record(stream)
    for r in range(reps):
        launches[r % len(launches)]()
    s1.record(stream)
    torch.cuda.synchronize()
    return s0.elapsed_time(s1) / 1e3 / reps


def time_graph(torch, launch_on, ntargets, reps):
    """Mean time per launch of `reps` launches (target i % ntargets) captured into one HIP
    graph and replayed: the GPU runs them back to back with no host enqueue in between, so
    small sizes show the kernel and its dispatch gap rather than the host's launch rate.
    None if the capture fails."""
    try:
        side = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=side):
            h = torch.cuda.current_stream().cuda_stream
            for r in range(reps):
                launch_on(r % ntargets, h)
        with torch.cuda.stream(side):  # replay() launches on the current stream
            g.replay()
            torch.cuda.synchronize()
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record(side)
            g.replay()
            s1.record(side)
        torch.cuda.synchronize()
        t = s0.elapsed_time(s1) / 1e3 / reps
        del g
        return t
    except Exception as e:  # noqa: BLE001 -- the eager figure stands alone then
        log(f"[curve] graph capture failed: {e}")
        return None


def size_curve_n1(args, torch, cpu=True, cpu_seconds=1.0):
    """The north star's N = 1 curve: the device combine (sosx_combine) at nreduce =
    1Mi .. 256Mi on device-symmetric-heap operands, and beside it SOS's own CPU reduce_local (the oracle restatement of
    src/shmem_internal_op.h:23-33,305-339, gcc -O2, 1 pinned thread) on the same inputs,
    timed for about `cpu_seconds` per point.

    Two GPU timings per point, both the mean HIP-event kernel time over a batch of
    back-to-back launches:
      * HBM-streamed (`kernel_us`, `GBs`, `frac_hbm`): each launch takes the next of k
        operand pairs, k * 2 * n * s >= 1 GiB, so a pair's bytes have left the 256 MiB
        Infinity Cache before it comes round again -- every launch streams from HBM, and
        `frac_hbm` is an HBM fraction;
      * resident (`resident_kernel_us`, `resident_GBs`): the same pair every launch.  Where
        the three streams fit the Infinity Cache (`cache_resident`: 3 * n * s <= 256 MiB)
        this reads above the HBM rate and is not roofline evidence."""
    from sos_amd import _lib as L
    O = None
    if cpu:
        from oracle import oracle as O
    dt, op = L.dtype_id(args.dtype), L.op_id(args.op)
    es = L.dtype_size(dt)
    dist = L.DIST_PROD if args.op == "prod" else L.DIST_UNIFORM
    stream = torch.cuda.current_stream()
    S = stream.cuda_stream
    sizes = [m for m in CURVE_SIZES if m <= args.sweep_max]
    shmem_up(args)
    rows = []
    for m in sizes:
        nb = m * es
        npairs = max(1, -(-ROTATE_BYTES // (2 * nb)))
        bufs = []
        for _ in range(npairs):  # device symmetric heap, as the headline's operands
            a, b = DevBuf(torch, nb, True), DevBuf(torch, nb, True)
            L.fill(dt, dist, SEED, 0, a.ptr, m, 0, S)
            L.fill(dt, dist, SEED, 1, b.ptr, m, 0, S)
            bufs.append((a, b))
        launches = [(lambda a=a, b=b: L.combine(op, dt, a.ptr, b.ptr, m, S)) for a, b in bufs]
        reps = max(10, min(400, int(4e9 // (3 * nb))), 2 * npairs)
        kern = time_launches(torch, stream, launches, reps)
        resident = time_launches(torch, stream, launches[:1], max(10, min(200, int(4e9 // (3 * nb)))))
        graph = time_graph(torch, lambda i, h: L.combine(op, dt, bufs[i][0].ptr, bufs[i][1].ptr, m, h),
                           len(bufs), reps) if nb <= GRAPH_MAX_BYTES else None
        del launches
        for a, b in bufs:
            a.free()
            b.free()
        algo = 3 * nb
        row = {"nreduce": m, "kernel_us": round(kern * 1e6, 2),
               "GBs": round(algo / kern / 1e9, 1),
               "frac_hbm": round(algo / kern / 1e9 / HBM_PEAK_GBS, 4),
               "gpu_GiBs": round(nb / kern / GiB, 2),
               "operand_pairs_rotated": npairs,
               "resident_kernel_us": round(resident * 1e6, 2),
               "resident_GBs": round(algo / resident / 1e9, 1),
               "cache_resident": algo <= MALL_BYTES}
        if graph:
            row.update({"graph_kernel_us": round(graph * 1e6, 2), "graph_GBs": round(algo / graph / 1e9, 1),
                        "graph_frac_hbm": round(algo / graph / 1e9 / HBM_PEAK_GBS, 4)})
        if O is not None:
            inout = O.fill(dt, dist, SEED, 0, m)
            inp = O.fill(dt, dist, SEED, 1, m)
            t1 = O.time_reduce_local(op, dt, inp, inout, 1)
            creps = max(1, int(cpu_seconds / max(t1, 1e-6)))
            t = O.time_reduce_local(op, dt, inp, inout, creps)
            row["cpu_GiBs"] = round(creps * m * es / t / GiB, 3)
            row["cpu_reps"] = creps
            row["gpu_over_cpu"] = round(row["gpu_GiBs"] / row["cpu_GiBs"], 1)
            del inout, inp
        rows.append(row)
        log(f"[curve] n={m:>10} {row['kernel_us']:10.2f} us {row['GBs']:8.1f} GB/s "
            f"frac {row['frac_hbm']:.3f} ({npairs} pairs)  resident {row['resident_GBs']:8.1f} GB/s"
            f"  cpu {row.get('cpu_GiBs')} GiB/s")
    return {"op": args.op, "type": args.dtype, "kernel": "sos::k_combine3",
            "gpu": ("mean HIP-event kernel time over a batch of back-to-back launches; kernel_us / "
                    "GBs / frac_hbm with the launches rotating over operand pairs of >= 1 GiB in "
                    "all (HBM-streamed), resident_* on one pair (cache_resident: the three "
                    "streams fit the 256 MiB Infinity Cache, not an HBM figure); graph_* (up to "
                    "16Mi): the same rotating batch captured in one HIP graph and replayed, so the "
                    "host's launch rate does not bound the small sizes"),
            "cpu": (f"oracle/sos_oracle.c reduce_local (SOS's loop, gcc -O2), 1 thread, "
                    f"~{cpu_seconds:g} s per point, same inputs" if cpu else "skipped"),
            "rows": rows}


# ----------------------------------------------------------------------------------
# --gpus N > 1 without a launcher: this process spawns the N rank processes itself
# ----------------------------------------------------------------------------------
def free_port_base(span=16):
    """A port p with p .. p+span-1 free on 127.0.0.1 (the team leg uses MASTER_PORT, the
    shmem bootstrap MASTER_PORT + 1 and the preflight job MASTER_PORT + 12)."""
    import random
    import socket
    for _ in range(200):
        base = random.randint(20000, 60000 - span)
        socks = []
        try:
            for k in range(span):
                s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
                socks.append(s)
                s.bind(("127.0.0.1", base + k))
            return base
        except OSError:
            continue
        finally:
            for s in socks:
                s.close()
    raise RuntimeError("no free port range on 127.0.0.1")


def spawn_ranks(n, argv, grace_s=60.0):
    """Run `bench.py argv` as n rank processes (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT set as torch.distributed.run sets them), one per GPU.
    This parent never touches the GPU: it only starts the ranks, passes their stderr
    through, forwards rank 0's one JSON line to stdout and returns the worst exit code.
    When a rank fails, the others get `grace_s` to finish before they are killed (by
    PID).  Returns (rc, rank 0's JSON line or None)."""
    port = free_port_base()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                    "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0",
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out0 = []
    import threading
    reader = threading.Thread(target=lambda: out0.extend(procs[0].stdout.read().decode().splitlines()),
                              daemon=True)
    reader.start()
    failed_at = None
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs):
            break
        if failed_at is None and any(rc not in (None, 0) for rc in rcs):
            failed_at = time.time()
            log(f"[spawn] a rank exited with {[rc for rc in rcs if rc not in (None, 0)]}; "
                f"waiting up to {grace_s:.0f} s for the others")
        if failed_at is not None and time.time() - failed_at > grace_s:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(0.2)
    reader.join(timeout=30)
    rcs = [p.returncode for p in procs]
    lines = [ln for ln in out0 if ln.startswith("{")]
    rc = next((c for c in rcs if c != 0), 0)
    if rc == 0 and len(lines) != 1:
        log(f"[spawn] rank 0 printed {len(lines)} JSON lines, expected one")
        rc = 1
    return rc, (lines[0] if lines else None)


def launch_check(torch):
    """--launch-check (CPU, no GPU touched): every rank joins a gloo group from the
    launcher's environment and rank 0 prints the ranks it saw -- the plumbing of the
    N > 1 line without the library (tests/test_bench_launch.py)."""
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    seen = [None] * world
    dist.all_gather_object(seen, {"rank": rank, "local_rank": int(os.environ["LOCAL_RANK"]),
                                  "pid": os.getpid()})
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks": seen}), flush=True)
    dist.destroy_process_group()
    return 0


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1 and not args.child_pmc:
        # no launcher: run the N ranks from here (a line for N GPUs or none at all)
        rc, line = spawn_ranks(args.gpus, sys.argv[1:])
        if line is not None and rc == 0:
            print(line, flush=True)
        return rc
    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus and not args.child_pmc:
        # never report an N-GPU figure measured on another number of ranks
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world}: run with a matching launcher "
            f"(or none: bench.py --gpus N spawns its N ranks itself)")
        return 2
    import torch
    if args.launch_check:
        return launch_check(torch)
    if (world > 1 or args.team) and not args.child_pmc:
        sys.path.insert(0, os.path.join(HERE, "tools"))
        import team_bench   # the N > 1 leg (bench code: tools/team_bench.py)
        return team_bench.main(args, torch, pmc=pmc_traffic)
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    if args.sweep:
        print(json.dumps(sweep(args, torch)), flush=True)
        return 0
    res = run_combine(args, torch)
    if res is None:
        return 0
    if rank == 0 and not args.no_adjacent:
        res["fold_kernel"] = multi_stream_kernel(args, torch, "fold")
        res["scan_prefix_kernel"] = multi_stream_kernel(args, torch, "prefix")
    if rank == 0 and not args.no_pmc:
        traffic, info = pmc_traffic(args, save_dir=args.pmc_save)
        note = ("(2*FETCH_SIZE + WRITE_SIZE)*1024 B per launch, rocprofv3 --pmc (one pass "
                "per counter), gfx950 FETCH_SIZE halving corrected")
        if traffic is not None and "combine" in traffic:
            res["roofline"]["traffic"] = round(traffic["combine"])
            res["roofline"]["traffic_note"] = note
            res["roofline"]["traffic_over_algorithmic"] = round(
                traffic["combine"] / res["roofline"]["algorithmic_bytes_per_launch"], 5)
            for kind, key in (("fold", "fold_kernel"), ("prefix", "scan_prefix_kernel")):
                if key in res and kind in traffic:
                    res[key]["traffic"] = round(traffic[kind])
                    res[key]["traffic_over_algorithmic"] = round(
                        traffic[kind] / res[key]["algorithmic_bytes_per_launch"], 5)
        else:
            res["roofline"]["traffic_note"] = str(info)
    if rank == 0 and not args.no_host:
        res["host_resident"] = host_resident(args, torch)
    if rank == 0 and not args.no_curve:
        res["size_curve"] = size_curve_n1(args, torch, cpu=not args.no_cpu)
    if rank == 0 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(args)
    print(json.dumps(res), flush=True)
    if _SHMEM_UP:
        from sos_amd import shmem as SH
        SH.shmem_finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
