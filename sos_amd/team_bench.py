"""N > 1 leg of bench.py: shmem_<T>_<op>_reduce over one PE per GPU.

Launched by torchrun (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*).  torch.distributed
(gloo, CPU) is only the bench's control plane: it broadcasts the RCCL unique id and
takes the barrier / max-over-ranks of the timing.  The data path is libsos_amd.so:
RCCL over xGMI between PEs + the HIP fold kernels, behind the public C API.

Self-check: after the timed steps every rank regenerates all P inputs on its own GPU
and evaluates the schedule's element order with the fold kernel (ring: chunk c
folded from PE c rightwards, src/collectives.c:693-727; tree schedules: the recdbl_sw
tree), then compares its team result bit for bit.
"""
import json
import os
import sys
import time

GiB = float(1 << 30)
HBM_PEAK_GBS = 8000.0
XGMI_LINK_GBS = 153.0   # per link, per direction, nominal
XGMI_LINKS = 7


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main(args, torch):
    import torch.distributed as dist
    from sos_amd import _lib as L
    from sos_amd import shmem as S

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank)) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dist.init_process_group("gloo")
    uid = [S.get_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    os.environ.setdefault("SHMEMX_DEVICE", str(local))
    S.init_attr(rank, world, uid[0])
    alg = L.ALGS[args.alg]
    S.shmemx_set_reduce_algorithm(alg)

    dt = L.dtype_id(args.dtype)
    es = L.dtype_size(dt)
    n = args.n
    dist_kind = L.DIST_PROD if args.op == "prod" else L.DIST_UNIFORM
    seed = 0x5EED
    stream = S.lib().shmemx_get_stream()
    src = torch.empty(n * es, dtype=torch.uint8, device="cuda")
    dst = torch.empty(n * es, dtype=torch.uint8, device="cuda")
    L.fill(dt, dist_kind, seed, rank, src.data_ptr(), n, 0, stream)
    torch.cuda.synchronize()
    fn = getattr(S, f"shmem_{args.dtype}_{args.op}_reduce")
    team = S.team_world()

    def step():
        fn(team, dst.data_ptr(), src.data_ptr(), n)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    dist.barrier()
    el = torch.tensor([t1 - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    t_step = el.item() / args.steps

    # phase split (separate calls, so the timed loop above carries no events)
    S.prof_enable(True)
    for _ in range(3):
        step()
    prof = S.prof_get()
    S.prof_enable(False)

    mismatches = self_check(torch, L, S, dt, L.op_id(args.op), dist_kind, seed, world, n, es, alg,
                            dst, stream)
    mm = torch.tensor([mismatches], dtype=torch.int64)
    dist.all_reduce(mm, op=dist.ReduceOp.SUM)

    resolved = S.lib().sosx_resolve_alg(alg, n * es, 16384)
    name = {v: k for k, v in L.ALGS.items()}[resolved]
    fold_ms = prof["fold_ms"] / max(prof["nfold"], 1)
    xfer_ms = prof["xfer_ms"] / max(prof["ncall"], 1)
    P = world
    if resolved in (L.ALGS["ring"], L.ALGS["recdbl_direct"]):
        fold_bytes = (P + 1) * (n // P) * es       # P inputs of one chunk + the output
    else:
        fold_bytes = 3 * (n // 2) * es             # first (largest) pairwise step
    wire = 2 * (P - 1) / P * n * es if resolved != L.ALGS["recdbl"] else (P.bit_length() - 1) * n * es
    res = {
        "metric": "GiB/s device-resident sum_reduce combine, nreduce=128Mi fp32; 1/2/4/8 GPU",
        "value": round(world * n * es / t_step / GiB, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {"float": "f32", "double": "f64"}.get(args.dtype, args.dtype),
        "data": "synthetic (splitmix64 counter hash per PE, SURVEY.md 8(d)), resident in HBM",
        "config": {"workload": f"shmem_{args.dtype}_{args.op}_reduce(SHMEM_TEAM_WORLD) nreduce={n} "
                               f"per PE, {world} PEs (1 per MI355X), RCCL over xGMI + HIP fold",
                   "nreduce": n, "algorithm": name, "parallelism": f"pe{world}"},
        "roofline": {"bound": "hbm", "kernel": "sos::k_fold (fused P-way combine)",
                     "achieved": round(fold_bytes / (fold_ms / 1e3) / 1e9, 1) if fold_ms > 0 else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(fold_bytes / (fold_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if fold_ms > 0 else None,
                     "traffic": None, "algorithmic_bytes_per_launch": fold_bytes,
                     "mean_kernel_ms": round(fold_ms, 5)},
        "team_roofline": {"bound": "xgmi", "wire_bytes_per_pe": int(wire),
                          "busbw_GBs": round(wire / t_step / 1e9, 1),
                          "frac_one_link": round(wire / t_step / 1e9 / XGMI_LINK_GBS, 3),
                          "frac_7_links": round(wire / t_step / 1e9 / (XGMI_LINK_GBS * XGMI_LINKS), 3),
                          "xfer_ms_per_step": round(xfer_ms, 4), "fold_ms_per_step":
                          round(prof["fold_ms"] / max(prof["ncall"], 1), 4)},
        "check": {"bitwise_mismatches_all_ranks": int(mm.item()),
                  "against": "on-GPU regeneration of all PE inputs + schedule-order fold"},
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.barrier()
    S.shmem_finalize()
    dist.destroy_process_group()
    return 0


def self_check(torch, L, S, dt, opid, dist_kind, seed, world, n, es, alg, dst, stream):
    """Bitwise check of this rank's result against a local re-evaluation."""
    resolved = S.lib().sosx_resolve_alg(alg, n * es, 16384)
    ins = []
    for p in range(world):
        b = torch.empty(n * es, dtype=torch.uint8, device="cuda")
        L.fill(dt, dist_kind, seed, p, b.data_ptr(), n, 0, stream)
        ins.append(b)
    exp = torch.empty(n * es, dtype=torch.uint8, device="cuda")
    if resolved == L.ALGS["ring"]:
        q, r = divmod(n, world)
        for c in range(world):
            cnt = q + (c < r)
            first = c * cnt if c < r else c * cnt + r
            if cnt == 0:
                continue
            ptrs = [ins[(c + k) % world].data_ptr() + first * es for k in range(world)]
            L.fold(opid, dt, L.ORDER_LINEAR, exp.data_ptr() + first * es, ptrs, cnt, stream)
    else:
        L.fold(opid, dt, L.ORDER_TREE, exp.data_ptr(), [b.data_ptr() for b in ins], n, stream)
    torch.cuda.synchronize()
    bad = L.count_mismatch(exp.data_ptr(), dst.data_ptr(), n, es, stream)
    del ins
    return bad
