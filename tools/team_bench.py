"""N > 1 leg of bench.py: shmem_<T>_<op>_reduce over one PE per GPU.

Bench code, not product code: it lives in tools/ (it imports the CPU oracle for its
CPU-baseline leg, which the product package never does).

Launched by torchrun (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*).  torch.distributed
(gloo, CPU) is only the bench's control plane (barrier, max over ranks).  The data path
is libsos_amd.so behind the public C API: shmem_init() bootstraps over TCP
(MASTER_ADDR, MASTER_PORT + 1), source/target live in the device symmetric heap
(shmemx_malloc_device), and every step is one shmem_<T>_<op>_reduce(SHMEM_TEAM_WORLD).

Both inter-PE transports are measured (SHMEMX_TRANSPORT=both):
  rccl       : ncclSend/ncclRecv over xGMI + the HIP fold kernels (the library default)
  p2p        : the fold kernel reads the peers' chunks straight out of their IPC-mapped
               HBM; stream-ordered signals between rounds (one host sync per call)
  rccl_ag    : the same, the allgather round as one ncclAllGather when chunks are equal
  p2p_host   : p2p with the host moving the transfer counters every round
  rccl_ar    : RCCL's own ncclAllReduce (SHMEMX_RCCL_ALLREDUCE=2): the reference point
               for the SOS schedules; for fp sum its bits follow RCCL's order, so it is
               checked against the fp tolerance bound instead and never gives `value`
`value` is the fastest of the library's SOS-schedule transports (rccl, rccl_ag, p2p,
p2p_host) whose bitwise check is clean on every rank; null (with the reason) if none.
Self-check: after timing, every rank regenerates all P inputs on its own GPU and
re-evaluates the schedule's element order with the fold kernel (ring: chunk c folded
from PE c rightwards, src/collectives.c:693-727; tree schedules: the recdbl_sw tree),
then compares its team result bit for bit.
"""
import ctypes
import json
import os
import sys
import time

# bench code, not product code: it lives in tools/ and reaches the package from the repo root
_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

ctypes_u8 = ctypes.c_uint8

GiB = float(1 << 30)
HBM_PEAK_GBS = 8000.0
XGMI_LINK_GBS = 153.0   # per link, per direction, nominal
XGMI_LINKS = 7


# Measured transports: (name, shmemx_set_transport id, p2p signalling mode, RCCL native
# allgather, RCCL native allreduce mode).  rccl runs three ways: every round as grouped
# ncclSend/ncclRecv (the default), with the equal-chunk allgather round as one
# ncclAllGather (sosx_set_rccl_allgather), and as RCCL's own ncclAllReduce
# (sosx_set_rccl_allreduce(2)); p2p runs twice: counters moved between rounds by
# stream-ordered device signals (the default) and by the host every round
# (sosx_set_p2p_signal_mode(0)).
TRANSPORTS = (("rccl", 0, None, 0, 0), ("rccl_ag", 0, None, 1, 0), ("p2p", 1, 1, 0, 0),
              ("p2p_host", 1, 0, 0, 0), ("rccl_ar", 0, None, 0, 2))
T_NAMES = tuple(t[0] for t in TRANSPORTS)
# the SOS schedules (bit-exact); rccl_ar ignores the schedule, so the schedule, host and
# scan/broadcast legs skip it (the headline and the size curve measure it)
SCHEDULE_T = ("rccl", "rccl_ag", "p2p", "p2p_host")
# the transports `value` may come from: the library's own SOS schedules + HIP fold.
# rccl_ar is RCCL's ncclAllReduce (no library kernel on the data path): never `value`,
# even where its bits happen to equal SOS's ring (integer ops, fp sum at P = 2).
VALUE_T = SCHEDULE_T

# What `value` is at every N, stated in the line itself: the
# payload of ALL PEs per step, the same definition as the N = 1 line (one PE's payload).
VALUE_DEFINITION = ("value = N * nreduce * sizeof(T) / max-over-ranks step time (whole-job "
                    "payload; the 1->8 scaling curve plots this); algbw_GiBs = nreduce * "
                    "sizeof(T) / step time (one PE's vector per step, NCCL's algbw)")


def headline_fields(world, n, es, t_step, rccl_ranks):
    """The line's rate fields (t_step None: no clean transport).  `value` is the whole-job
    payload per step (every PE's nreduce * sizeof(T)), the N = 1 line's definition at N = 1;
    algbw_GiBs is one PE's vector per step; rccl_comm_ranks is what every rank's RCCL
    communicator reported (ncclCommCount; -1 without RCCL)."""
    ok = t_step is not None and t_step > 0
    return {"value": round(world * n * es / t_step / GiB, 3) if ok else None,
            "unit": "GiB/s",
            "algbw_GiBs": round(n * es / t_step / GiB, 3) if ok else None,
            "value_definition": VALUE_DEFINITION,
            "n_gpus": world,
            "rccl_comm_ranks": list(rccl_ranks)}


def xgmi_fields(wire, ts, world, ngpus):
    """busbw = wire bytes per PE / step time, and its fractions of one and of seven xGMI
    links.  When ranks share a GPU no xGMI link carries their bytes, so the link roofline
    does not describe the run: the fractions are null (a fraction above 1 would say the
    roofline is wrong, not that the code beat it) and the bound is "shared-gpu"."""
    bus = wire / ts / 1e9
    shared = ngpus < world
    return {"busbw_GBs": round(bus, 1),
            "frac_one_link": None if shared else round(bus / XGMI_LINK_GBS, 3),
            "frac_7_links": None if shared else round(bus / (XGMI_LINK_GBS * XGMI_LINKS), 3)}


def team_bound(world, ngpus):
    return "shared-gpu" if ngpus < world else "xgmi"


def select_primary(results):
    """(transport `value` comes from, None) or (None, reason).  Only a VALUE_T transport
    that was measured and whose bitwise check is clean on every rank qualifies; there is
    no fallback to a faster transport whose check failed."""
    measured = [k for k in VALUE_T if k in results and results[k].get("available", True)]
    if not measured:
        return None, "no SOS-schedule transport was available (preflight or bring-up failed)"
    clean = [k for k in measured if results[k]["mismatches"] == 0]
    if not clean:
        return None, ("every SOS-schedule transport failed its bitwise check: "
                      + ", ".join(f"{k} {results[k]['mismatches']}" for k in measured))
    return min(clean, key=lambda k: results[k]["t_step"]), None


def placement_text(world, ngpus):
    """How the PEs sat on GPUs, from the device map the ranks reported (distinct devices)."""
    if ngpus == world:
        return f"{world} PEs on {ngpus} GPUs (1 per MI355X)"
    return f"{world} PEs on {ngpus} GPU{'s' if ngpus != 1 else ''} (shared: not a 1-PE-per-GPU figure)"


def parallelism_text(world, ngpus):
    return f"pe{world}" if ngpus == world else f"pe{world}_on_{ngpus}gpu"


def device_ident(torch, local):
    """A string naming this rank's physical GPU (UUID, else PCI location)."""
    props = torch.cuda.get_device_properties(local)
    u = getattr(props, "uuid", None)
    if u is not None and str(u).strip("0-"):
        return str(u)
    loc = [getattr(props, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id")]
    if any(v is not None for v in loc):
        return ":".join(str(v) for v in loc)
    return f"{os.uname().nodename}/{local}"


def workload_text(tname, dtype, op, n, world, ngpus=None):
    """config.workload for what actually ran (ngpus: distinct GPUs the PEs ran on)."""
    ngpus = world if ngpus is None else ngpus
    head = f"shmem_{dtype}_{op}_reduce(SHMEM_TEAM_WORLD) nreduce={n} per PE, {placement_text(world, ngpus)}, "
    data_path = {
        "rccl": "ncclSend/ncclRecv over xGMI + HIP fold kernel",
        "rccl_ag": "ncclSend/ncclRecv + ncclAllGather over xGMI + HIP fold kernel",
        "p2p": "p2p reads of IPC-mapped peer HBM + HIP fold kernel, stream-signalled rounds",
        "p2p_host": "p2p reads of IPC-mapped peer HBM + HIP fold kernel, host-signalled rounds",
    }
    return head + data_path.get(tname, "no valid measurement")


# transports that failed the preflight on some rank (every leg skips them)
DISABLED = set()
PREFLIGHT_PORT_OFFSET = 11   # the preflight job bootstraps on MASTER_PORT + 12
PREFLIGHT_LIMIT_S = 150.0    # the preflight job is killed after this long


def use_transport(S, L, tname):
    """Switch every PE (collectively) to `tname`; False when it is unavailable."""
    if tname in DISABLED:
        return False
    _, tid, sig, ag, ar = next(t for t in TRANSPORTS if t[0] == tname)
    if S.lib().shmemx_set_transport(tid) < 0:
        return False
    L.lib().sosx_set_rccl_allgather(ag)
    L.lib().sosx_set_rccl_allreduce(ar)
    return sig is None or L.lib().sosx_set_p2p_signal_mode(sig) >= 0


def reset_transport(S, L):
    S.lib().shmemx_set_transport(0)
    L.lib().sosx_set_rccl_allgather(0)
    L.lib().sosx_set_rccl_allreduce(0)
    L.lib().sosx_set_p2p_signal_mode(1)


def tolerance_leg(tname, args):
    """rccl_ar on fp sum/prod: RCCL's own summation order, checked against the fp bound."""
    return tname == "rccl_ar" and args.dtype in ("float", "double") and args.op in ("sum", "prod")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main(args, torch, pmc=None):
    import torch.distributed as dist
    from sos_amd import _lib as L
    from sos_amd import shmem as S

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank)) % max(torch.cuda.device_count(), 1)
    # stdout carries rank 0's ONE JSON line and nothing else: what the native layers print
    # there (gloo's "[Gloo] Rank i is connected to ..." lines, an RCCL banner) goes to
    # stderr, and the line is written to the saved descriptor
    sys.stdout.flush()
    line_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    dt = L.dtype_id(args.dtype)
    es = L.dtype_size(dt)
    n = args.n
    user_transport = os.environ.get("SHMEMX_TRANSPORT")
    os.environ.setdefault("SHMEMX_TRANSPORT", "both")
    sweep_sizes = [] if getattr(args, "no_team_sweep", False) else \
        [m for m in (1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20)
         if m != n and m <= getattr(args, "sweep_max", 256 << 20)]
    nmax = max([n] + sweep_sizes)
    # p2p stage region: the scans' exchange scratch (2(P-1)/P * n * s) and staged host
    # operands must fit it, or those calls run on RCCL instead
    stage = 2 * n * es + (64 << 20)
    os.environ.setdefault("SHMEMX_STAGE_BYTES", str(stage))
    os.environ.setdefault("SHMEMX_DEVICE_HEAP_SIZE", str(2 * nmax * es + stage + (320 << 20)))
    os.environ.setdefault("SHMEMX_DEVICE", str(local))
    os.environ.setdefault("SHMEMX_P2P_TIMEOUT", "120")
    os.environ.setdefault("SHMEM_SYMMETRIC_SIZE", str(2 * (16 << 20) * es + (64 << 20)))
    dist.init_process_group("gloo")
    pre = preflight(torch, dist, rank, world)
    DISABLED.update(k for k, ok in pre["ok"].items() if not ok)
    if user_transport is None:
        # a transport that failed everywhere is not even brought up in this job
        p2p_any = pre["ok"]["p2p"] or pre["ok"]["p2p_host"]
        rccl_any = pre["ok"]["rccl"] or pre["ok"]["rccl_ag"] or pre["ok"]["rccl_ar"]
        if p2p_any != rccl_any:
            os.environ["SHMEMX_TRANSPORT"] = "p2p" if p2p_any else "rccl"
    if rank == 0 and DISABLED:
        log(f"[team] preflight: transports {sorted(DISABLED)} disabled ({pre['why']})")
    # the device is opened only now: during the preflight the child PE job is the only
    # process on each GPU (counting devices above does not initialise the runtime)
    torch.cuda.set_device(local)
    idents = [None] * world
    dist.all_gather_object(idents, device_ident(torch, local))
    ngpus = len(set(idents))
    S.shmem_init()
    assert S.shmem_n_pes() == world and S.shmem_my_pe() == rank
    # the rank count RCCL's communicator reports (-1: no RCCL in this job), every rank's
    rccl_ranks = [None] * world
    dist.all_gather_object(rccl_ranks, int(L.lib().sosx_rccl_comm_count()))
    alg = L.ALGS[args.alg]
    S.shmemx_set_reduce_algorithm(alg)

    dist_kind = L.DIST_PROD if args.op == "prod" else L.DIST_UNIFORM
    seed = 0x5EED
    stream = S.lib().shmemx_get_stream()
    src = S.shmemx_malloc_device(nmax * es)
    dst = S.shmemx_malloc_device(nmax * es)
    L.fill(dt, dist_kind, seed, rank, src, nmax, 0, stream)
    torch.cuda.synchronize()
    fn = getattr(S, f"shmem_{args.dtype}_{args.op}_reduce")
    team = S.team_world()
    resolved = S.lib().sosx_resolve_alg(alg, n * es, 16384)
    name = {v: k for k, v in L.ALGS.items()}[resolved]
    P = world

    def step():
        fn(team, dst, src, n)

    results = {}
    if rank == 0:
        log(f"[team] {world} PEs, nreduce {n}, alg {name}: heap {os.environ['SHMEMX_DEVICE_HEAP_SIZE']} B")
    for tid, tname in enumerate(T_NAMES):
        if not use_transport(S, L, tname):
            results[tname] = {"available": False, "preflight_failed": tname in DISABLED}
            continue
        if rank == 0:
            log(f"[team] {tname}: warmup + {args.steps} timed steps")
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
        # phase split (separate calls, so the timed loop carries no events)
        S.prof_enable(True)
        for _ in range(3):
            step()
        prof = S.prof_get()
        S.prof_enable(False)
        # fresh inputs for the checked call: a transport that returned bytes left over
        # from the timed loop (same inputs every step) would fail here
        check_seed = seed + 1 + tid
        L.fill(dt, dist_kind, check_seed, rank, src, n, 0, stream)
        torch.cuda.synchronize()
        dist.barrier()
        step()
        tol = tolerance_leg(tname, args)
        mm = self_check(torch, L, S, dt, L.op_id(args.op), dist_kind, check_seed, world, n, es,
                        alg, dst, stream, tolerance=tol)
        mm, tv = mm if tol else (mm, 0)
        L.fill(dt, dist_kind, seed, rank, src, n, 0, stream)
        torch.cuda.synchronize()
        mmt = torch.tensor([mm, tv], dtype=torch.int64)
        dist.all_reduce(mmt, op=dist.ReduceOp.SUM)
        results[tname] = {"t_step": t_step, "prof": prof, "mismatches": int(mmt[0].item())}
        if tol:
            results[tname]["tolerance_violations"] = int(mmt[1].item())

    curve = size_curve(args, torch, dist, L, S, fn, team, dt, es, dist_kind, seed, rank, world,
                       src, dst, stream, sorted(sweep_sizes + [n]), results, ngpus) if sweep_sizes else {}

    schedules = {} if getattr(args, "no_adjacent", False) else \
        other_schedules(args, torch, dist, L, S, fn, team, dt, es, dist_kind, seed, rank, world,
                        src, dst, stream, results)

    host_leg = {} if getattr(args, "no_host", False) else \
        host_resident_team(args, torch, dist, L, S, fn, team, dt, es, dist_kind, seed, rank,
                           world, stream, results)

    cpu_ring = {} if getattr(args, "no_cpu", False) else \
        cpu_ring_baseline(args, torch, dist, L, S, fn, team, dt, es, dist_kind, seed, rank, world,
                          src, dst, stream)

    adjacent = {}
    if not getattr(args, "no_adjacent", False):
        adjacent = adjacent_collectives(args, torch, dist, L, S, dt, es, n, src, dst, stream,
                                        seed, rank, world)

    local_leg = local_combine(args, torch, dist, L, dt, es, n, src, dst, stream, world)

    small = {} if (getattr(args, "no_small", False) or getattr(args, "no_cpu", False)) else \
        small_messages(args, torch, dist, L, S, team, rank, world, stream)

    # HBM traffic of the fold kernel: rank 0 runs bench.py's PMC passes (rocprofv3 --pmc
    # FETCH_SIZE, then WRITE_SIZE) over a one-process child launching the same kernel at
    # this call's shape (P inputs of n/P elements) on its GPU; the other ranks wait
    fold_traffic = None
    if (pmc is not None and not getattr(args, "no_pmc", False)
            and os.environ.get("SOSX_BENCH_PMC", "1") != "0"
            and resolved in (L.ALGS["ring"], L.ALGS["recdbl_direct"])):
        if rank == 0:
            log(f"[team] PMC passes over the fold kernel (P = {P}, {n // P} elements per input)")
            args.fold_p = P
            tr, info = pmc(args)
            fold_traffic = tr.get("fold") if tr else None
            if fold_traffic is None:
                log(f"[team] PMC: {info}")
        dist.barrier()

    # every measured transport is reported; `value` only from one of the library's SOS
    # schedules whose bitwise check is clean (select_primary)
    measured = [k for k in T_NAMES if results[k].get("available", True)]
    primary, why_null = select_primary(results)
    if resolved in (L.ALGS["ring"], L.ALGS["recdbl_direct"]):
        fold_bytes = (P + 1) * (n // P) * es       # P inputs of one chunk + the output
    else:
        fold_bytes = 3 * (n // 2) * es             # first (largest) pairwise step
    wire = 2 * (P - 1) / P * n * es if resolved != L.ALGS["recdbl"] else (P.bit_length() - 1) * n * es

    def team_roof(rr):
        ts = rr["t_step"]
        return {"ms_per_step": round(ts * 1e3, 4),
                "value_GiBs": round(world * n * es / ts / GiB, 3),
                "algbw_GiBs": round(n * es / ts / GiB, 3),
                **xgmi_fields(wire, ts, world, ngpus),
                "xfer_ms_per_step": round(rr["prof"]["xfer_ms"] / max(rr["prof"]["ncall"], 1), 4),
                "fold_ms_per_step": round(rr["prof"]["fold_ms"] / max(rr["prof"]["ncall"], 1), 4),
                "bitwise_mismatches_all_ranks": rr["mismatches"],
                **({"fp_tolerance_violations_all_ranks": rr["tolerance_violations"],
                    "note": "RCCL's own order: compared with the fp bound, not bit for bit"}
                   if "tolerance_violations" in rr else {})}

    r = results[primary] if primary else None
    t_step = r["t_step"] if r else None
    fold_ms = r["prof"]["fold_ms"] / max(r["prof"]["nfold"], 1) if r else 0.0
    res = {
        "metric": "GiB/s device-resident sum_reduce combine, nreduce=128Mi fp32; 1/2/4/8 GPU",
        **headline_fields(world, n, es, t_step, rccl_ranks),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4) if r else None,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {"float": "f32", "double": "f64"}.get(args.dtype, args.dtype),
        "data": "synthetic (splitmix64 counter hash per PE, SURVEY.md 8(d)), resident in HBM",
        "config": {"workload": workload_text(primary, args.dtype, args.op, n, world, ngpus),
                   "nreduce": n, "algorithm": name, "transport": primary,
                   "parallelism": parallelism_text(world, ngpus), "gpus_used": ngpus},
        "roofline": {"bound": "hbm", "kernel": "sos::k_fold (fused P-way combine)",
                     "achieved": round(fold_bytes / (fold_ms / 1e3) / 1e9, 1) if fold_ms > 0 else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(fold_bytes / (fold_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if fold_ms > 0 else None,
                     "traffic": round(fold_traffic) if fold_traffic else None,
                     **({"traffic_over_algorithmic": round(fold_traffic / fold_bytes, 5),
                         "traffic_note": "(2*FETCH_SIZE + WRITE_SIZE)*1024 B per launch, "
                                         "rocprofv3 --pmc over a one-process child running "
                                         "this kernel at this shape on GPU 0"}
                        if fold_traffic else {}),
                     "algorithmic_bytes_per_launch": fold_bytes,
                     "mean_kernel_ms": round(fold_ms, 5) if r else None,
                     **({"note": "p2p: the fold reads its P-1 peer inputs in place over xGMI, "
                                 "so this launch is link-bound (see team_roofline)"}
                        if primary and primary.startswith("p2p") else {})},
        "team_roofline": dict(bound=team_bound(world, ngpus), wire_bytes_per_pe=int(wire),
                              **team_roof(r)) if r else None,
        "check": {"bitwise_mismatches_all_ranks": r["mismatches"] if r else None,
                  "against": "on-GPU regeneration of all PE inputs + schedule-order fold"},
    }
    if why_null:
        res["value_null_reason"] = why_null
    res["transports"] = {k: team_roof(results[k]) for k in measured}
    res["transport_choice"] = ("value = the fastest of the library's SOS-schedule transports "
                               f"({', '.join(VALUE_T)}) whose bitwise check is clean on every "
                               "rank, else null; the library default is rccl "
                               "(SHMEMX_TRANSPORT selects; rccl_ag = rccl with "
                               "SHMEMX_RCCL_ALLGATHER=1, p2p_host = p2p with "
                               "SHMEMX_P2P_SIGNAL=host). rccl_ar = RCCL's own ncclAllReduce "
                               "(SHMEMX_RCCL_ALLREDUCE=2) is reported as the reference point "
                               "only: it measures RCCL's combine, not the library's fold")
    res["preflight"] = pre
    res["local_combine_all_pes"] = local_leg
    if curve:
        res["size_curve"] = curve
    if schedules:
        res["schedules"] = schedules
    if host_leg:
        res["host_resident"] = host_leg
    if adjacent:
        res["adjacent_collectives"] = adjacent
    if cpu_ring:
        res["cpu_ring_baseline"] = cpu_ring
    if small:
        res["small_messages"] = small
    if rank == 0:
        line_out.write(json.dumps(res) + "\n")
        line_out.flush()
    dist.barrier()
    S.shmemx_free_device(dst)
    S.shmemx_free_device(src)
    S.shmem_finalize()
    dist.destroy_process_group()
    return 0


def local_combine(args, torch, dist, L, dt, es, n, src, dst, stream, world):
    """The N = 1 headline kernel on every GPU at once (reduce_local: dst OP= src, nreduce
    per PE, no exchange): the local HBM roofline at N GPUs, beside the team line's xGMI
    one.  Whole-job GiB/s = world * n * s / max-over-ranks time per call."""
    opid = L.op_id(args.op)
    steps = max(5, min(args.steps, 50))
    for _ in range(3):
        L.combine(opid, dt, dst, src, n, stream)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        L.combine(opid, dt, dst, src, n, stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    el = torch.tensor([t1 - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    ts = el.item() / steps
    return {"kernel": "sos::k_combine3", "nreduce": n, "ms_per_call": round(ts * 1e3, 4),
            "value_GiBs": round(world * n * es / ts / GiB, 3),
            "hbm_GBs_per_pe": round(3 * n * es / ts / 1e9, 1),
            "frac_of_hbm_peak_per_pe": round(3 * n * es / ts / 1e9 / HBM_PEAK_GBS, 4),
            "note": "every PE's local combine at once, no exchange (host wall clock, "
                    "max over ranks): the HBM side of the 1->N curve; per PE = per GPU "
                    "with one PE per GPU"}


def cpu_ring_baseline(args, torch, dist, L, S, fn, team, dt, es, dist_kind, seed, rank, world,
                      src, dst, stream):
    """SOS's own CPU path beside the N > 1 line: the bench's P rank
    processes, each pinned to one host core, run the restated ring
    (oracle/sos_oracle.c oracle_pe_ring, src/collectives.c:647-764) over a /dev/shm
    segment -- memcpy puts and atomic pSync adds, SOS's XPMEM model -- on the same
    per-PE inputs, at nreduce = 1Mi, 16Mi and the headline size (`rows`; the top-level
    fields are the headline's).  Bounded sample per size: one untimed call, then as many
    calls as fit ~6 s at the headline size (~1.5 s below it), max over ranks.  At each
    size the CPU targets are compared byte for byte with the library's ring result on
    the GPU for the same inputs.
    Test infrastructure in the timed-baseline role only: the product path never calls it."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    from oracle import oracle as O
    m = args.n
    sizes = sorted({k for k in (1 << 20, 16 << 20) if k < m} | {m})
    opid = L.op_id(args.op)
    if rank == 0:
        log(f"[cpu ring] {world} processes x 1 core, nreduce {sizes}")

    # one physical core per PE, consecutive (as a by-core rank binding would place them):
    # the first hardware thread of each core in the allowed set
    allowed = sorted(os.sched_getaffinity(0))
    primaries = []
    for c in allowed:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                first = int(f.read().replace("-", ",").split(",")[0])
        except (OSError, ValueError):
            first = c
        if first == c or first not in allowed:
            primaries.append(c)
    core = primaries[rank % len(primaries)]
    path = f"/dev/shm/sosx_cpu_ring_{os.environ.get('MASTER_PORT', '0')}_{world}"
    ring = None
    why = ""

    def agreed(ok):  # every rank learns whether all ranks succeeded
        v = torch.tensor([0 if ok else 1], dtype=torch.int64)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        return v.item() == 0

    rows = []
    try:
        ok = True
        if rank == 0:
            try:
                if os.path.exists(path):
                    os.unlink(path)
                ring = O.PeRing(path, world, 0, m, dt, create=True)  # space reserved up front
            except OSError as e:
                ok, why = False, f"cannot create the {world}-PE segment: {e}"
                if os.path.exists(path):
                    os.unlink(path)
        if not agreed(ok):
            return {"skipped": why or "segment creation failed on rank 0"}
        if rank != 0:
            try:
                ring = O.PeRing(path, world, rank, m, dt, create=False)
            except OSError as e:
                ok, why = False, str(e)
        if not agreed(ok):
            return {"skipped": why or "segment attach failed on a rank"}
        if rank == 0:
            os.unlink(path)  # every PE has it mapped
        host_src = O.fill(dt, dist_kind, seed, rank, m)   # a prefix is the smaller sizes' input
        for mk in sizes:
            # the library's ring on the GPU for these inputs (src holds fill(seed, rank))
            S.shmemx_set_reduce_algorithm(L.ALGS["ring"])
            fn(team, dst, src, mk)
            torch.cuda.synchronize()
            S.shmemx_set_reduce_algorithm(L.ALGS[args.alg])
            os.sched_setaffinity(0, {core})
            ring.count = mk
            t_warm = ring.time(opid, host_src, 1)
            tw = torch.tensor([t_warm], dtype=torch.float64)
            dist.all_reduce(tw, op=dist.ReduceOp.MAX)
            budget = 6.0 if mk == m else 1.5
            reps = max(1, min(1000, int(budget / max(tw.item(), 1e-6))))
            t = ring.time(opid, host_src, reps)
            el = torch.tensor([t], dtype=torch.float64)
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            ts = el.item() / reps
            ring.barrier()  # every put into this PE's target has landed
            os.sched_setaffinity(0, set(allowed))
            tgt = ring.target()
            exp = torch.from_numpy(tgt.view("u1").copy()).to("cuda")
            del tgt
            torch.cuda.synchronize()
            mm = L.count_mismatch(exp.data_ptr(), dst, mk, es, stream)
            mmt = torch.tensor([mm], dtype=torch.int64)
            dist.all_reduce(mmt, op=dist.ReduceOp.SUM)
            del exp
            ring.barrier()  # nobody rewrites a target before every PE has read its own
            rows.append({"nreduce": mk, "ms_per_call": round(ts * 1e3, 4),
                         "value_GiBs": round(world * mk * es / ts / GiB, 3), "reps": reps,
                         "bitwise_mismatches_vs_gpu_ring_all_ranks": int(mmt.item())})
            if rank == 0:
                log(f"[cpu ring] n={mk} {rows[-1]['ms_per_call']} ms/call, "
                    f"{rows[-1]['value_GiBs']} GiB/s whole job, mismatches vs GPU ring "
                    f"{rows[-1]['bitwise_mismatches_vs_gpu_ring_all_ranks']}")
        del host_src
    finally:
        if ring is not None:
            ring.close()
        os.sched_setaffinity(0, set(allowed))
    cpu = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    head = rows[-1]
    out = {"value": head["value_GiBs"], "unit": "GiB/s", "cores": world,
           "kind": "port", "ms_per_call": round(head["ms_per_call"], 3),
           "sample": (f"SOS ring (oracle_pe_ring, src/collectives.c:647-764), "
                      f"shmem_{args.dtype}_{args.op}_reduce nreduce={m} per PE, {world} processes "
                      f"x 1 pinned physical core (consecutive cores from {primaries[0]}), "
                      f"memcpy puts over /dev/shm, {head['reps']} timed calls after 1 warm-up, "
                      f"gcc -O2; host: {cpu}, {len(primaries)} cores / {len(allowed)} threads allowed"),
           "bitwise_mismatches_vs_gpu_ring_all_ranks": sum(
               r["bitwise_mismatches_vs_gpu_ring_all_ranks"] for r in rows),
           "rows": rows}
    return out


def small_messages(args, torch, dist, L, S, team, rank, world, stream):
    """Small and medium shmem_float_sum_reduce(SHMEM_TEAM_WORLD) calls under SOS AUTO,
    microseconds per call (max over ranks), beside SOS's own CPU path on the same
    processes:
      host   : operands in the host symmetric heap (shmem_malloc), SOS's own case -- the
               small host-resident path (one kernel per PE over node shared memory);
      device : operands in the device symmetric heap (shmemx_malloc_device), as the
               library runs them: through node shared memory while team size * bytes
               <= SHMEMX_SMALL_DEVICE (128 KiB), else on the default transport;
      device_executor : the same calls with that limit at 0 (every call on the
               transport's executor);
      cpu    : SOS AUTO on the CPU -- recdbl_sw below 16 KiB, the ring above
               (oracle_pe_recdbl / oracle_pe_ring, src/collectives.c:850-984, :647-764),
               one pinned physical core per PE, memcpy puts over /dev/shm.
    At every size the host-heap and device-heap results are compared byte for byte with
    the CPU result.
    Test infrastructure in the timed-baseline role only."""
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    from oracle import oracle as O
    sizes = [1, 1024, 16384, 65536]          # fp32: 4 B .. 256 KiB
    nmax, dt, opid, es = max(sizes), L.dtype_id("float"), L.op_id("sum"), 4
    seed = 0x5A11
    S.shmemx_set_reduce_algorithm(L.ALGS["auto"])
    hsrc, hdst = S.lib().shmem_malloc(nmax * es), S.lib().shmem_malloc(nmax * es)
    dsrc, ddst = S.shmemx_malloc_device(nmax * es), S.shmemx_malloc_device(nmax * es)
    if not (hsrc and hdst and dsrc and ddst):
        return {"skipped": "symmetric allocation failed"}
    mine = O.fill(dt, L.DIST_UNIFORM, seed, rank, nmax)
    np.ctypeslib.as_array((ctypes_u8 * (nmax * es)).from_address(hsrc))[:] = mine.view(np.uint8)
    L.fill(dt, L.DIST_UNIFORM, seed, rank, dsrc, nmax, 0, stream)
    torch.cuda.synchronize()

    def timed(call, reps):
        for _ in range(10):
            call()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            call()
        t1 = time.perf_counter()
        el = torch.tensor([t1 - t0], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return el.item() / reps

    small_before = S.lib().sosx_small_path_calls()
    small_dev_before = S.lib().sosx_small_path_device_calls()
    rows = []
    for n in sizes:
        reps = 200 if n <= 16384 else 50
        th = timed(lambda: S.shmem_float_sum_reduce(team, hdst, hsrc, n), reps)
        td = timed(lambda: S.shmem_float_sum_reduce(team, ddst, dsrc, n), reps)
        rows.append({"nreduce": n, "bytes": n * es,
                     "schedule": "recdbl_sw" if n * es < 16384 else "ring",
                     "host_us": round(th * 1e6, 2), "device_us": round(td * 1e6, 2)})
    small_calls = S.lib().sosx_small_path_calls() - small_before
    small_dev_calls = S.lib().sosx_small_path_device_calls() - small_dev_before
    cap = S.lib().sosx_set_small_device_bytes(0)     # every rank: the choice is per PE
    for row in rows:
        n = row["nreduce"]
        tx = timed(lambda: S.shmem_float_sum_reduce(team, ddst, dsrc, n), 200 if n <= 16384 else 50)
        row["device_executor_us"] = round(tx * 1e6, 2)
    S.lib().sosx_set_small_device_bytes(cap)

    # SOS's CPU path on the same ranks, pinned one physical core each
    allowed = sorted(os.sched_getaffinity(0))
    primaries = []
    for c in allowed:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                first = int(f.read().replace("-", ",").split(",")[0])
        except (OSError, ValueError):
            first = c
        if first == c or first not in allowed:
            primaries.append(c)
    path = f"/dev/shm/sosx_small_{os.environ.get('MASTER_PORT', '0')}_{world}"
    ring = None
    try:
        if rank == 0:
            if os.path.exists(path):
                os.unlink(path)
            ring = O.PeRing(path, world, 0, nmax, dt, create=True, alg="recdbl")
        dist.barrier()
        if rank != 0:
            ring = O.PeRing(path, world, rank, nmax, dt, create=False, alg="recdbl")
        dist.barrier()
        if rank == 0:
            os.unlink(path)
        for row in rows:
            n = row["nreduce"]
            ring.count = n
            ring.alg = O.PeRing.ALGS["recdbl" if n * es < 16384 else "ring"]
            os.sched_setaffinity(0, {primaries[rank % len(primaries)]})
            reps = 2000 if n <= 16384 else 200
            ring.time(opid, mine, max(10, reps // 10))
            t = ring.time(opid, mine, reps) / reps
            ring.barrier()
            os.sched_setaffinity(0, set(allowed))
            el = torch.tensor([t], dtype=torch.float64)
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            row["cpu_us"] = round(el.item() * 1e6, 2)
            # the library's host-heap result for these inputs vs SOS's CPU result
            S.shmem_float_sum_reduce(team, hdst, hsrc, n)
            got = np.ctypeslib.as_array((ctypes_u8 * (n * es)).from_address(hdst)).copy()
            exp = ring.target().view(np.uint8)[:n * es].copy()
            # ... and the device-heap result (the path the device row timed)
            S.shmem_float_sum_reduce(team, ddst, dsrc, n)
            gd = torch.empty(n * es, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            L.check(S.lib().sosx_memcpy(gd.data_ptr(), ddst, n * es, None), "sosx_memcpy")
            gd = gd.cpu().numpy()
            mm = torch.tensor([int(np.count_nonzero(got.view(np.uint32) != exp.view(np.uint32))),
                               int(np.count_nonzero(gd.view(np.uint32) != exp.view(np.uint32)))],
                              dtype=torch.int64)
            dist.all_reduce(mm, op=dist.ReduceOp.SUM)
            row["host_bitwise_mismatches_vs_cpu_all_ranks"] = int(mm[0].item())
            row["device_bitwise_mismatches_vs_cpu_all_ranks"] = int(mm[1].item())
            ring.barrier()
    finally:
        if ring is not None:
            ring.close()
        os.sched_setaffinity(0, set(allowed))
    S.shmemx_free_device(ddst)
    S.shmemx_free_device(dsrc)
    S.lib().shmem_free(hdst)
    S.lib().shmem_free(hsrc)
    if rank == 0:
        for r in rows:
            log(f"[small] n={r['nreduce']} host {r['host_us']} us, device {r['device_us']} us "
                f"(executor {r['device_executor_us']} us), SOS CPU {r['cpu_us']} us, mismatches "
                f"{r['host_bitwise_mismatches_vs_cpu_all_ranks']}/{r['device_bitwise_mismatches_vs_cpu_all_ranks']}")
    return {"op": "float sum", "algorithm": "auto", "rows": rows,
            "small_path_calls_rank0_side": int(small_calls),
            "small_path_device_calls_rank0_side": int(small_dev_calls),
            "small_device_team_bytes": int(cap),
            "note": "us per call, max over ranks; host = host symmetric heap (small path through "
                    "node shared memory), device = device symmetric heap (that path while team size "
                    "* bytes <= small_device_team_bytes, else the default transport), "
                    "device_executor = device heap on the default transport, cpu = SOS AUTO "
                    "on the CPU (recdbl_sw < 16 KiB, ring above), one pinned core per PE"}


def host_resident_team(args, torch, dist, L, S, fn, team, dt, es, dist_kind, seed, rank, world,
                       stream, headline):
    """The same team reduction when source/dest live in the HOST symmetric heap (SOS's
    own case: shmem_malloc returns pinned host memory here): H2D staging, the device team
    reduction, D2H -- the PCIe-inclusive rate the north star asks to record beside
    `value`.  nreduce = min(n, 16Mi) (64 MiB fp32: the p2p stage region's size)."""
    import numpy as np
    m = min(args.n, 16 << 20)
    nbytes = m * es
    hsrc = S.lib().shmem_malloc(nbytes)
    hdst = S.lib().shmem_malloc(nbytes)
    if not hsrc or not hdst:
        return {"skipped": "shmem_malloc failed (SHMEM_SYMMETRIC_SIZE)"}
    tmp = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    L.fill(dt, dist_kind, seed, rank, tmp.data_ptr(), m, 0, stream)
    torch.cuda.synchronize()
    host = np.ctypeslib.as_array((ctypes_u8 * nbytes).from_address(hsrc))
    host[:] = tmp.cpu().numpy()
    out = {"nreduce": m, "buffers": "shmem_malloc (pinned host symmetric heap)"}
    for tid, tname in enumerate(SCHEDULE_T):
        if not headline.get(tname, {}).get("available", True) or not use_transport(S, L, tname):
            continue
        reps = max(3, min(args.steps, 10))
        fn(team, hdst, hsrc, m)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn(team, hdst, hsrc, m)
        t1 = time.perf_counter()
        el = torch.tensor([t1 - t0], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        ts = el.item() / reps
        out[tname] = {"ms_per_call": round(ts * 1e3, 4),
                      "value_GiBs": round(world * nbytes / ts / GiB, 3),
                      "payload_GiBs_per_pe": round(nbytes / ts / GiB, 3),
                      "pcie_bytes_per_pe": 2 * nbytes}
        log(f"[host resident] {tname} n={m} {out[tname]['ms_per_call']} ms/call")
    reset_transport(S, L)
    S.lib().shmem_free(hdst)
    S.lib().shmem_free(hsrc)
    return out


def size_curve(args, torch, dist, L, S, fn, team, dt, es, dist_kind, seed, rank, world, src, dst,
               stream, sizes, headline, ngpus):
    """The team reduction over nreduce = 1Mi .. 256Mi (SURVEY 8(d) config #5 / the north
    star's 1->8-GPU curve) on each transport: whole-job GiB/s (world * n * s / t, max over
    ranks), busbw = 2(P-1)/P * n * s / t and its fraction of one xGMI link and of all 7.
    The largest size also gets the bitwise self-check on fresh inputs."""
    P = world
    out = {}
    alg = L.ALGS[args.alg]
    for tid, tname in enumerate(T_NAMES):
        if not headline.get(tname, {}).get("available", True) or not use_transport(S, L, tname):
            continue
        rows = []
        for m in sizes:
            if m == args.n and "t_step" in headline.get(tname, {}):
                ts = headline[tname]["t_step"]
            else:
                reps = max(3, min(args.steps, int(4e9 // (m * es))))
                for _ in range(2):
                    fn(team, dst, src, m)
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(reps):
                    fn(team, dst, src, m)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                el = torch.tensor([t1 - t0], dtype=torch.float64)
                dist.all_reduce(el, op=dist.ReduceOp.MAX)
                ts = el.item() / reps
            wire = 2 * (P - 1) / P * m * es
            row = {"nreduce": m, "ms_per_call": round(ts * 1e3, 4),
                   "value_GiBs": round(world * m * es / ts / GiB, 3),
                   **xgmi_fields(wire, ts, world, ngpus)}
            if m == sizes[-1] and m != args.n:
                cseed = seed + 211 + tid
                L.fill(dt, dist_kind, cseed, rank, src, m, 0, stream)
                torch.cuda.synchronize()
                dist.barrier()
                fn(team, dst, src, m)
                tol = tolerance_leg(tname, args)
                mm = self_check(torch, L, S, dt, L.op_id(args.op), dist_kind, cseed, world, m, es,
                                alg, dst, stream, tolerance=tol)
                mm, tv = mm if tol else (mm, 0)
                mmt = torch.tensor([mm, tv], dtype=torch.int64)
                dist.all_reduce(mmt, op=dist.ReduceOp.SUM)
                row["bitwise_mismatches_all_ranks"] = int(mmt[0].item())
                if tol:
                    row["fp_tolerance_violations_all_ranks"] = int(mmt[1].item())
                L.fill(dt, dist_kind, seed, rank, src, args.n, 0, stream)
                torch.cuda.synchronize()
            rows.append(row)
            log(f"[team curve] {tname} n={m} {row['ms_per_call']} ms/call {row['value_GiBs']} GiB/s "
                f"busbw {row['busbw_GBs']} GB/s")
        out[tname] = rows
    reset_transport(S, L)
    return out


def other_schedules(args, torch, dist, L, S, fn, team, dt, es, dist_kind, seed, rank, world, src,
                    dst, stream, headline):
    """The headline reduction under the other bit-exact-for-sum schedules
    (SHMEM_REDUCE_ALGORITHM): the north star's recursive halving + doubling (pairwise,
    one link per step) and recdbl_direct (recdbl_sw tree after a direct exchange), on each
    transport, with the bitwise self-check (recdbl_sw tree order) on fresh inputs."""
    n, P = args.n, world
    out = {}
    steps = max(3, min(args.steps, 10))
    for tid, tname in enumerate(SCHEDULE_T):
        if not headline.get(tname, {}).get("available", True) or not use_transport(S, L, tname):
            continue
        for sname in ("rechalving", "recdbl_direct"):
            alg = L.ALGS[sname]
            S.shmemx_set_reduce_algorithm(alg)
            if rank == 0:
                log(f"[team] schedule {sname} on {tname}")
            for _ in range(2):
                fn(team, dst, src, n)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(steps):
                fn(team, dst, src, n)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            el = torch.tensor([t1 - t0], dtype=torch.float64)
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            ts = el.item() / steps
            cseed = seed + 307 + tid
            L.fill(dt, dist_kind, cseed, rank, src, n, 0, stream)
            torch.cuda.synchronize()
            dist.barrier()
            fn(team, dst, src, n)
            mm = self_check(torch, L, S, dt, L.op_id(args.op), dist_kind, cseed, world, n, es, alg,
                            dst, stream)
            mmt = torch.tensor([mm], dtype=torch.int64)
            dist.all_reduce(mmt, op=dist.ReduceOp.SUM)
            L.fill(dt, dist_kind, seed, rank, src, n, 0, stream)
            torch.cuda.synchronize()
            wire = 2 * (P - 1) / P * n * es
            out.setdefault(tname, {})[sname] = {
                "ms_per_call": round(ts * 1e3, 4),
                "value_GiBs": round(world * n * es / ts / GiB, 3),
                "busbw_GBs": round(wire / ts / 1e9, 1),
                "bitwise_mismatches_all_ranks": int(mmt.item())}
    S.shmemx_set_reduce_algorithm(L.ALGS[args.alg])
    reset_transport(S, L)
    return out


def adjacent_collectives(args, torch, dist, L, S, dt, es, n, src, dst, stream, seed, rank, world):
    """shmemx_<T>_sum_inscan and shmem_<T>_broadcast (root 0) at the bench size, on each
    transport: time per call (max over ranks), the bytes each PE puts on xGMI, and a
    bitwise check on fresh inputs (scan: one prefix launch over every PE's regenerated
    source; broadcast: the root's regenerated source)."""
    import time as _t
    team = S.team_world()
    P = world
    steps = max(min(args.steps, 10), 2)
    out = {}
    scan_fn = getattr(S, f"shmemx_{args.dtype}_sum_inscan", None)
    bcast_fn = getattr(S, f"shmem_{args.dtype}_broadcast", None)
    colls = []
    if scan_fn is not None:
        colls.append(("inscan", lambda: scan_fn(team, dst, src, n),
                      2 * (P - 1) / P * n * es))
    # broadcast: the root puts the payload on its links once (scattered over P-1 links
    # above 64 KiB); each non-root forwards its 1/(P-1) share to the P-2 others
    colls.append(("broadcast_root0", lambda: bcast_fn(team, dst, src, n, 0), n * es))
    for tid, tname in enumerate(SCHEDULE_T):
        if not use_transport(S, L, tname):
            continue
        for cname, call, wire in colls:
            for _ in range(2):
                call()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = _t.perf_counter()
            for _ in range(steps):
                call()
            torch.cuda.synchronize()
            t1 = _t.perf_counter()
            dist.barrier()
            el = torch.tensor([t1 - t0], dtype=torch.float64)
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            ts = el.item() / steps
            # check on fresh inputs
            cseed = seed + 101 + tid
            L.fill(dt, L.DIST_UNIFORM, cseed, rank, src, n, 0, stream)
            torch.cuda.synchronize()
            dist.barrier()
            call()
            if cname == "inscan":
                ins = []
                for p in range(P):
                    b = torch.empty(n * es, dtype=torch.uint8, device="cuda")
                    L.fill(dt, L.DIST_UNIFORM, cseed, p, b.data_ptr(), n, 0, stream)
                    ins.append(b)
                outs = [torch.empty_like(x) for x in ins]
                L.prefix("sum", dt, [o.data_ptr() for o in outs], [x.data_ptr() for x in ins],
                         n, -1, stream)
                exp = outs[rank]
            else:
                exp = torch.empty(n * es, dtype=torch.uint8, device="cuda")
                L.fill(dt, L.DIST_UNIFORM, cseed, 0, exp.data_ptr(), n, 0, stream)
            torch.cuda.synchronize()
            mm = L.count_mismatch(exp.data_ptr(), dst, n, es, stream)
            mmt = torch.tensor([mm], dtype=torch.int64)
            dist.all_reduce(mmt, op=dist.ReduceOp.SUM)
            if cname == "inscan":
                del ins, outs
            del exp
            L.fill(dt, L.DIST_UNIFORM, seed, rank, src, n, 0, stream)
            torch.cuda.synchronize()
            out.setdefault(tname, {})[cname] = {
                "ms_per_call": round(ts * 1e3, 4),
                "payload_GiBs_per_pe": round(n * es / ts / GiB, 3),
                "wire_bytes_per_pe": int(wire),
                "wire_GBs_per_pe": round(wire / ts / 1e9, 1),
                "bitwise_mismatches_all_ranks": int(mmt.item())}
    reset_transport(S, L)
    return out


def self_check(torch, L, S, dt, opid, dist_kind, seed, world, n, es, alg, dst, stream,
               tolerance=False):
    """Bitwise check of this rank's result against a local re-evaluation.  With
    `tolerance` (fp sum/prod, for results in another order than the schedule's) it
    returns (bitwise mismatches, elements outside the fp bound of DESIGN.md section 5:
    |got - exp| <= (P-1) eps sum_p |x_p| for sum, 2 (P-1) eps |exp| for prod)."""
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
    bad = L.count_mismatch(exp.data_ptr(), dst, n, es, stream)
    if not tolerance:
        del ins
        return bad
    ft = {4: torch.float32, 8: torch.float64}[es]
    got = torch.empty(n * es, dtype=torch.uint8, device="cuda")
    L.check(L.lib().sosx_memcpy(got.data_ptr(), dst, n * es, stream), "sosx_memcpy")
    torch.cuda.synchronize()
    eps = torch.finfo(ft).eps
    g = got.view(ft).double()
    e = exp.view(ft).double()
    if opid == L.op_id("sum"):
        bound = torch.zeros_like(e)
        for b in ins:
            bound += b.view(ft).double().abs()
        bound *= (world - 1) * eps
    else:
        bound = 2 * (world - 1) * eps * e.abs()
    tol_bad = int(((g - e).abs() > bound).sum().item())
    del ins
    return bad, tol_bad


def preflight(torch, dist, rank, world):
    """Run every transport once in a short-lived child PE job before the bench brings
    them up in this one.  A transport that hangs, times out (the p2p waits end the process
    with _exit) or returns wrong bytes there is disabled on every rank here, so that one
    broken transport cannot take the whole N > 1 line with it.  The child job is the same
    library and the same torchrun ranks, bootstrapped on MASTER_PORT + 12, with the p2p
    wait bound at 20 s; its results are agreed over gloo (a transport counts only when
    it passed on every rank).  The child is killed after PREFLIGHT_LIMIT_S (a transport
    that hangs without a bound, e.g. in RCCL init).  SOSX_BENCH_PREFLIGHT=0 skips it."""
    import subprocess
    ok = {k: True for k in T_NAMES}
    if os.environ.get("SOSX_BENCH_PREFLIGHT", "1") == "0":
        return {"ran": False, "ok": ok, "why": "SOSX_BENCH_PREFLIGHT=0"}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.update(MASTER_PORT=str(int(os.environ["MASTER_PORT"]) + PREFLIGHT_PORT_OFFSET),
               SHMEMX_TRANSPORT=os.environ.get("SHMEMX_TRANSPORT", "both"),
               SHMEMX_P2P_TIMEOUT="20", SHMEM_BOOTSTRAP_TIMEOUT="60",
               SHMEMX_DEVICE_HEAP_SIZE=str(512 << 20), SHMEMX_STAGE_BYTES=str(64 << 20),
               SHMEM_SYMMETRIC_SIZE=str(64 << 20))
    t0 = time.perf_counter()
    why = ""
    import tempfile
    with tempfile.TemporaryFile("w+") as fo, tempfile.TemporaryFile("w+") as fe:
        child = subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), "--preflight"],
                                 cwd=root, env=env, stdout=fo, stderr=fe)
        next_note = 20.0
        while child.poll() is None:
            el = time.perf_counter() - t0
            if el > PREFLIGHT_LIMIT_S:
                child.kill()
                child.wait()
                why = f"child killed after {PREFLIGHT_LIMIT_S:.0f} s"
                break
            if el > next_note:      # progress lines: a silent wait looks like a hang
                if rank == 0:
                    log(f"[team] preflight job still running ({el:.0f} s)")
                next_note += 20.0
            time.sleep(0.2)
        rc = child.returncode
        fo.seek(0)
        fe.seek(0)
        out, err = fo.read(), fe.read()
    seen = {}
    for line in out.splitlines():
        if line.startswith("{"):
            try:
                d = json.loads(line)
            except ValueError:
                continue
            if d.get("t") in ok:
                seen[d["t"]] = bool(d.get("ok"))
    for k in T_NAMES:       # a transport the child never reported (it died first) failed
        ok[k] = seen.get(k, False)
    if rc != 0 and not why:
        why = f"child rc={rc}"
    if rc != 0 or not all(ok.values()):
        tail = "\n".join((err or "").strip().splitlines()[-6:])
        log(f"[team] rank {rank} preflight: {seen} ({why or 'check failed'})\n{tail}")
    flags = torch.tensor([1 if ok[k] else 0 for k in T_NAMES], dtype=torch.int64)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    agreed = {k: bool(v) for k, v in zip(T_NAMES, flags.tolist())}
    return {"ran": True, "ok": agreed, "seconds": round(time.perf_counter() - t0, 1),
            "why": why or ("ok" if all(agreed.values()) else "bitwise check or availability")}


def preflight_child():
    """The preflight job (one PE per torchrun rank): each transport in turn runs a
    recdbl-sized (1Ki) and a ring-sized (4Mi) float sum reduce on fresh inputs, checked
    bit for bit; one JSON line per transport as soon as it is done."""
    import torch
    from sos_amd import _lib as L
    from sos_amd import shmem as S
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank)) % max(torch.cuda.device_count(), 1)
    os.environ.setdefault("SHMEMX_DEVICE", str(local))
    S.shmem_init()
    dt = L.dtype_id("float")
    es = L.dtype_size(dt)
    stream = S.lib().shmemx_get_stream()
    nmax = 4 << 20
    src = S.shmemx_malloc_device(nmax * es)
    dst = S.shmemx_malloc_device(nmax * es)
    team = S.team_world()
    alg = L.ALGS["auto"]
    S.shmemx_set_reduce_algorithm(alg)
    # test hook (tests/test_gpu_fakerccl.py): SOSX_PREFLIGHT_FAULT=<transport>:<rank> makes
    # that rank vanish when it reaches that transport, so its peers meet a real p2p timeout
    fault_t, _, fault_r = os.environ.get("SOSX_PREFLIGHT_FAULT", "").partition(":")
    for tid, tname in enumerate(T_NAMES):
        if tname == fault_t and fault_r and int(fault_r) == rank:
            os._exit(0)
        if not use_transport(S, L, tname):
            print(json.dumps({"t": tname, "ok": False, "why": "unavailable"}), flush=True)
            continue
        bad = 0
        for k, n in enumerate((1024, nmax)):
            seed = 0x9F1E + 16 * tid + k
            L.fill(dt, L.DIST_UNIFORM, seed, rank, src, n, 0, stream)
            torch.cuda.synchronize()
            S.shmem_float_sum_reduce(team, dst, src, n)
            if tname == "rccl_ar":   # RCCL's order: the fp bound, not the bits
                bad += self_check(torch, L, S, dt, L.op_id("sum"), L.DIST_UNIFORM, seed, world,
                                  n, es, alg, dst, stream, tolerance=True)[1]
            else:
                bad += self_check(torch, L, S, dt, L.op_id("sum"), L.DIST_UNIFORM, seed, world,
                                  n, es, alg, dst, stream)
        print(json.dumps({"t": tname, "ok": bad == 0, "mismatches": bad}), flush=True)
    reset_transport(S, L)
    S.shmemx_free_device(dst)
    S.shmemx_free_device(src)
    S.shmem_finalize()
    return 0


if __name__ == "__main__" and "--preflight" in sys.argv:
    sys.exit(preflight_child())
