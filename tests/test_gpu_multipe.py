"""GPU, multiple processes on one MI355X: the peer-to-peer transport end to end.

tools/oshrun starts P PEs (P = 2, 3, 4, 8) on the box's single GPU with
SHMEMX_TRANSPORT=p2p: each PE maps every other PE's device heap through IPC and the
plans' transfers become direct reads of peer HBM, synchronised through node shared
memory -- the same code that reads xGMI peer memory on the 8-GPU node.  (RCCL refuses
two ranks on one GPU; tests/test_gpu_fakerccl.py runs the RCCL executor's multi-PE cases.)
"""
import json
import os
import re
import subprocess
import sys
import time

import numpy as np
import pytest

from oracle import oracle as O
from sos_amd import _lib as L

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OSHRUN = os.path.join(ROOT, "tools", "oshrun")


def oshrun(np_, cmd, timeout=600, extra_env=None):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update({"SHMEMX_TRANSPORT": "p2p", "SHMEMX_DEVICE_HEAP_SIZE": "256M",
                "SHMEMX_STAGE_BYTES": "64M", "SHMEMX_DEVICE": "0", "PYTHONPATH": ROOT})
    if np_ >= 8:
        # eight PE processes on the box's one GPU, next to this pytest process's own
        # queues, oversubscribe the device's hardware queues and every call then waits on
        # queue time-slicing: one hardware queue per PE process
        # (the full suite measured test_coll_check[8] at 110 s with the default, 4 s alone)
        env["GPU_MAX_HW_QUEUES"] = "1"
    env.update(extra_env or {})
    return subprocess.run([sys.executable, OSHRUN, "-np", str(np_), "--timeout", str(timeout - 30),
                           *cmd], capture_output=True, text=True, timeout=timeout, env=env)


@pytest.fixture(scope="module")
def examples():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples")], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    return os.path.join(ROOT, "examples")


GOLDEN_PI = {2: "Pi from 20000 points on 2 PEs: 3.164400",
             4: "Pi from 40000 points on 4 PEs: 3.154100",
             8: "Pi from 80000 points on 8 PEs: 3.150200"}


@pytest.mark.parametrize("np_", [2, 4, 8])
def test_pi_reduce_multi_pe(examples, np_):
    r = oshrun(np_, [os.path.join(examples, "pi_reduce_amd")], timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("Pi from")]
    assert lines == [GOLDEN_PI[np_]], r.stdout


@pytest.mark.parametrize("alg", ["auto", "linear", "tree", "recdbl", "ring", "bogus"])
def test_reduce_algorithm_env_matrix(examples, alg):
    """SOS's CI runs `make check` once per SHMEM_REDUCE_ALGORITHM = auto, linear, tree,
    recdbl, ring on 2 processes (.github/workflows/ci.yml:86-124, :246-252).  The same
    matrix here over the C programs: pi_reduce's golden line (an integer sum, the same under
    every schedule) and reduce_types' closed forms, 2 PE processes.  linear and tree run
    recdbl_sw, as SOS does without NIC atomics (src/shmem_collectives.h:200-229); an unknown
    name is ignored with SOS's warning (src/collectives.c:195-210)."""
    env = {"SHMEM_REDUCE_ALGORITHM": alg}
    r = oshrun(2, [os.path.join(examples, "pi_reduce_amd")], timeout=180, extra_env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert [ln for ln in r.stdout.splitlines() if ln.startswith("Pi from")] == [GOLDEN_PI[2]], r.stdout
    if alg == "bogus":
        assert "Ignoring bad reduction algorithm 'bogus'" in r.stderr, r.stderr[-2000:]
    r = oshrun(2, [os.path.join(examples, "reduce_types")], timeout=180, extra_env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert "reduce_types: OK (2 PEs)" in r.stdout


@pytest.mark.parametrize("crossover,want", [(None, "ring"), ("1M", "recdbl"), ("32768", "ring"),
                                            ("32769", "recdbl")])
def test_coll_size_crossover_env(crossover, want):
    """SHMEM_COLL_SIZE_CROSSOVER moves AUTO's switch from recdbl_sw to the ring
    (src/shmem_collectives.h:179-200: recdbl_sw below the crossover, the ring at or above
    it): a 32 KiB float sum over 4 PE processes gives the ring's bits by default (16 KiB)
    and at a crossover of exactly 32 KiB, recdbl_sw's bits one byte above; on device-heap
    operands (the executor) and host-heap ones (the small shared-memory path)."""
    env = {} if crossover is None else {"SHMEM_COLL_SIZE_CROSSOVER": crossover}
    r = oshrun(4, [sys.executable, os.path.join(ROOT, "tests", "crossover_pe.py"), want], timeout=180,
               extra_env=env)
    ok = re.findall(r"PE (\d)/4: (\w+) bits on device and host heap", r.stdout)
    assert r.returncode == 0 and sorted(int(p) for p, _ in ok) == [0, 1, 2, 3], r.stdout + r.stderr[-2000:]


def test_reduce_types_4_pes(examples):
    r = oshrun(4, [os.path.join(examples, "reduce_types")], timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert "reduce_types: OK (4 PEs)" in r.stdout


@pytest.mark.parametrize("np_,signal,small_dev", [(2, "stream", True), (3, "stream", False),
                                                   (4, "stream", True), (8, "stream", True),
                                                   (3, "host", False), (8, "host", False),
                                                   (12, "host", True), (1, "host", False)])
def test_team_check(np_, signal, small_dev):
    """Every schedule across np_ PE processes, with the p2p transport's counters moved by
    stream-ordered device signals (the default) or by the host every round
    (SHMEMX_P2P_SIGNAL=host); small device operands through node shared memory (the
    default) or, with SHMEMX_SMALL_DEVICE=0, on the p2p executor like larger ones."""
    env = {"SHMEMX_P2P_SIGNAL": signal}
    if not small_dev:
        env["SHMEMX_SMALL_DEVICE"] = "0"
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "team_check_pe.py")], timeout=900,
               extra_env=env)
    # PEs print concurrently, so lines may interleave: count the reports, not lines
    ok = re.findall(r"PE (\d+)/\d+: \d+ checks OK \(p2p signal (\w+), small-path calls (\d+), "
                    r"device (\d+)\)", r.stdout)
    assert r.returncode == 0 and sorted(int(p) for p, _, _, _ in ok) == list(range(np_)), \
        r.stdout + r.stderr[-3000:]
    if np_ > 1:  # one PE has no p2p peers to signal
        assert {m for _, m, _, _ in ok} == {signal}, ok
    # the host-resident recdbl_sw calls below 64 KiB took the shared-memory path, and the
    # small device-resident ones did when it was on (a 1-PE job has no team to meet)
    assert all((int(c) > 0) == (np_ > 1) for _, _, c, _ in ok), ok
    assert all((int(d) > 0) == small_dev for _, _, _, d in ok), ok


@pytest.mark.parametrize("np_", [2, 3])
def test_team_check_small_path_off(np_):
    """SHMEMX_SMALL_HOST=0: the same checks with every host-resident call on the general
    (staged) path -- both paths give the oracle's bits."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "team_check_pe.py")], timeout=900,
               extra_env={"SHMEMX_SMALL_HOST": "0"})
    ok = re.findall(r"PE (\d+)/\d+: \d+ checks OK \(p2p signal \w+, small-path calls (\d+),", r.stdout)
    assert r.returncode == 0 and sorted(int(p) for p, _ in ok) == list(range(np_)), \
        r.stdout + r.stderr[-3000:]
    assert all(int(c) == 0 for _, c in ok), ok


def test_team_check_small_path_bytes():
    """SHMEMX_SMALL_HOST_BYTES=4096: host operands up to 4 KiB take the small path, larger
    ones the staged path, in the same job -- every result the oracle's bits, and the small
    path did run."""
    r = oshrun(3, [sys.executable, os.path.join(ROOT, "tests", "team_check_pe.py")], timeout=900,
               extra_env={"SHMEMX_SMALL_HOST_BYTES": "4096"})
    ok = re.findall(r"PE (\d+)/\d+: \d+ checks OK \(p2p signal \w+, small-path calls (\d+),", r.stdout)
    assert r.returncode == 0 and sorted(int(p) for p, _ in ok) == [0, 1, 2], \
        r.stdout + r.stderr[-3000:]
    assert all(int(c) > 0 for _, c in ok), ok


def test_team_reduction_past_2_31_elements():
    """shmem_uint8_sum_reduce of 2^31 + 4101 elements per PE across 2 PE processes
    (tests/big_count_pe.py): SOS's int count stops below this, this build's size_t does
    not; the AUTO ring's chunks, exchange and fold against the oracle's ring, bit for
    bit.  Device heap 9 GiB per PE: the operands plus the p2p exchange scratch."""
    r = oshrun(2, [sys.executable, os.path.join(ROOT, "tests", "big_count_pe.py")], timeout=400,
               extra_env={"SHMEMX_DEVICE_HEAP_SIZE": "9G", "SHMEMX_STAGE_BYTES": "4200M"})
    ok = re.findall(r"PE (\d+)/2: \d+ elements OK", r.stdout)
    assert r.returncode == 0 and sorted(map(int, ok)) == [0, 1], r.stdout + r.stderr[-3000:]


@pytest.mark.parametrize("np_", [2, 4, 5])
def test_small_path_stress(np_):
    """400 seeded small reductions over interleaved teams (world, even PEs, odd PEs),
    host-heap and device-heap operands, both sides of the crossover
    (tests/small_stress_pe.py): the shared-memory slots and per-pair post counters under
    every reuse order, each result bit for bit against the CPU oracle."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "small_stress_pe.py")], timeout=300)
    ok = re.findall(r"PE (\d+)/\d+: \d+ checks OK \(small-path calls (\d+), device (\d+)\)", r.stdout)
    assert r.returncode == 0 and sorted(int(p) for p, _, _ in ok) == list(range(np_)), \
        r.stdout + r.stderr[-3000:]
    assert all(int(c) > 0 and int(d) > 0 for _, c, d in ok), ok


@pytest.mark.parametrize("np_,signal,small_dev", [(2, "host", True), (3, "host", True),
                                                   (4, "host", False), (8, "host", True),
                                                   (3, "stream", True), (8, "stream", False)])
def test_coll_check(np_, signal, small_dev):
    """Scans and broadcasts through the public API (tests/coll_check_pe.py), p2p counters
    moved by the host or by stream-ordered device signals; small device operands through
    node shared memory or (SHMEMX_SMALL_DEVICE=0) on the executor."""
    env = {"SHMEMX_P2P_SIGNAL": signal}
    if not small_dev:
        env["SHMEMX_SMALL_DEVICE"] = "0"
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "coll_check_pe.py")], timeout=900,
               extra_env=env)
    ok = re.findall(r"PE (\d+)/\d+: \d+ checks OK \(p2p signal (\w+), small-path device calls (\d+)\)",
                    r.stdout)
    assert r.returncode == 0 and sorted(int(p) for p, _, _ in ok) == list(range(np_)), \
        r.stdout + r.stderr[-3000:]
    assert {m for _, m, _ in ok} == {signal}, ok
    assert all((int(d) > 0) == small_dev for _, _, d in ok), ok


@pytest.mark.parametrize("signal", ["stream", "host"])
def test_p2p_wait_is_bounded(signal):
    """A PE that never arrives ends the job with the p2p timeout error (SHMEMX_P2P_TIMEOUT)
    on the waiting PE, in both signalling modes, instead of a hang."""
    t0 = time.monotonic()
    r = oshrun(2, [sys.executable, os.path.join(ROOT, "tests", "p2p_timeout_pe.py")], timeout=150,
               extra_env={"SHMEMX_P2P_TIMEOUT": "3", "SHMEMX_P2P_SIGNAL": signal})
    assert r.returncode != 0, r.stdout
    assert "p2p transport: timed out" in r.stderr, r.stderr[-2000:]
    assert "reduction returned" not in r.stdout
    assert time.monotonic() - t0 < 55, "the job outlived the late PE's sleep"


@pytest.mark.parametrize("mode", ["host", "devsmall"])
def test_small_path_wait_is_bounded(mode):
    """The same late PE with 64-float operands in the host heap or the device heap: the
    call takes the small path through node shared memory, whose waits for a peer's operand
    are bounded by SHMEMX_P2P_TIMEOUT too."""
    t0 = time.monotonic()
    env = {"SHMEMX_P2P_TIMEOUT": "3"}
    r = oshrun(2, [sys.executable, os.path.join(ROOT, "tests", "p2p_timeout_pe.py"), mode],
               timeout=150, extra_env=env)
    assert r.returncode != 0, r.stdout
    assert "small shared-memory path: timed out" in r.stderr, r.stderr[-2000:]
    assert "reduction returned" not in r.stdout
    assert time.monotonic() - t0 < 55, "the job outlived the late PE's sleep"


def test_route_mismatch_ends_the_job_at_once():
    """PE 0 with host-heap operands (small path), PE 1 with device-heap operands above
    SHMEMX_SMALL_DEVICE (executor) in the same call: the small-path PE reads the peer's
    route word while it waits for its post and ends the job with both residencies named,
    long before SHMEMX_P2P_TIMEOUT (60 s here)."""
    r = oshrun(2, [sys.executable, os.path.join(ROOT, "tests", "route_mismatch_pe.py")], timeout=150,
               extra_env={"SHMEMX_P2P_TIMEOUT": "60", "SHMEMX_SMALL_DEVICE": "16K"})
    t_end = time.time()
    assert r.returncode != 0, r.stdout
    assert "reduction returned" not in r.stdout
    msg = [ln for ln in r.stderr.splitlines() if "took different paths" in ln]
    assert msg, r.stderr[-2000:]
    assert "PE 0 the small shared-memory path (source host, target host)" in msg[0], msg
    assert "PE 1 the executor (source device, target device)" in msg[0], msg
    starts = [float(x) for x in re.findall(r"call starts at ([\d.]+)", r.stdout)]
    assert len(starts) == 2, r.stdout
    assert t_end - max(starts) < 10, t_end - max(starts)  # teardown included; 60 s if missed


def test_device_heap_colours():
    """Large device-heap allocations step through the 32 KiB channel interleave in 4 KiB
    colours (consecutive ones an odd multiple of 4 KiB apart), at the same offsets on
    every PE (symmetric)."""
    r = oshrun(2, [sys.executable, os.path.join(ROOT, "tests", "heap_colour_pe.py")], timeout=120,
               extra_env={"SHMEMX_DEVICE_HEAP_SIZE": "1G", "SHMEMX_STAGE_BYTES": "64M",
                          "HEAP_REGION_BYTES": str(960 << 20)})
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    # PEs print concurrently: match the reports, not lines
    lines = re.findall(r"PE \d: (colours \[[\d, ]+\] offsets \[[\d, ]+\])", r.stdout)
    assert len(lines) == 2 and lines[0] == lines[1], r.stdout
    assert "colours [0, 1, 2, 3, 4, 5, 6, 7, 0, 1]" in lines[0], lines


@pytest.mark.parametrize("np_", [2, 3])
def test_calls_end_with_system_release(np_):
    """Every executor call (reductions under four schedules in both p2p signalling modes, a
    scan, a broadcast, reduce_local, a barrier) issues a system-scope release before it
    returns, so its results are in HBM for DMA reads, the host and peer GPUs (DESIGN.md
    section 5, the 12-PE wrong results); each result is the oracle's."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "sys_release_pe.py")], timeout=180)
    ok = re.findall(r"PE (\d+)/\d+: (\d+) calls, each ended with a system-scope release", r.stdout)
    assert r.returncode == 0 and sorted(int(p) for p, _ in ok) == list(range(np_)), \
        r.stdout + r.stderr[-2000:]


@pytest.mark.parametrize("np_", [2, 3, 4])
def test_peer_reads_follow_system_acquire(np_):
    """The consumer half of the visibility rule: every launch that
    read a peer's bytes -- p2p gathers and in-place folds under four schedules in both
    signalling modes, a scan, a broadcast, the small path with host and device operands --
    followed a system-scope acquire issued after the wait for the peer's post (the
    library's own classification, sosx_acquire_stats), each result the oracle's read back
    by a plain D2H copy; the acquire kernels reached all 8 XCDs."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "acquire_pe.py")], timeout=180)
    ok = re.findall(r"PE (\d+)/\d+: (\d+) calls, (\d+) peer reads, (\d+) acquires, 0 unacquired, "
                    r"\d+ acquire kernels, xcc mask 0x([0-9a-f]{2})", r.stdout)
    assert r.returncode == 0 and sorted(int(p) for p, *_ in ok) == list(range(np_)), \
        r.stdout + r.stderr[-2000:]
    assert all(int(reads) > 0 and int(acq) > 0 for _, _, reads, acq, _ in ok), ok
    assert {m for *_, m in ok} == {"ff"}, ok


def _static_inputs(n, pe):
    i = np.arange(n, dtype=np.uint64)
    k = (i * np.uint64(2654435761) + np.uint64(pe * 40503)) % np.uint64(1000003)
    return k.astype(np.float32) * np.float32(0.001)


@pytest.mark.parametrize("np_", [1, 2])
def test_static_data_team_reduce(examples, np_, tmp_path):
    """shmem_float_sum_reduce on STATIC source/dest arrays of 16Mi floats (.bss of
    examples/static_reduce.c), which shmem_init registered with HIP as SOS registers its
    data segment (src/init.c:341-346): every PE's bytes equal the oracle's (the ring under
    AUTO; one PE copies), and the segment was registered."""
    n = 16 << 20
    out = str(tmp_path / "static")
    cmd = [os.path.join(examples, "static_reduce"), "team", str(n), out]
    if np_ == 1:
        env = dict(os.environ)
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            env.pop(k, None)
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=env)
    else:
        r = oshrun(np_, cmd, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    reg = re.findall(r"PE (\d+)/\d+: static team reduce of \d+ floats written; data segment "
                     r"registered (\d+) B", r.stdout)
    assert sorted(int(p) for p, _ in reg) == list(range(np_)), r.stdout
    assert all(int(b) >= 2 * n * 4 for _, b in reg), reg
    ins = [_static_inputs(n, q) for q in range(np_)]
    dt = L.dtype_id("float")
    exp = O.ring(L.op_id("sum"), dt, ins) if np_ > 1 else [ins[0]]
    for q in range(np_):
        got = np.fromfile(f"{out}.{q}", dtype=np.float32)
        assert got.size == n and got.tobytes() == exp[q].tobytes(), q


@pytest.mark.parametrize("register", [True, False])
def test_static_data_local_combine(examples, register):
    """shmemx_reduce_local on static arrays (the H2D || combine || D2H pipeline) on the
    registered data segment, and with SHMEMX_REGISTER_DATA=0 (pageable): exact results."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    if not register:
        env["SHMEMX_REGISTER_DATA"] = "0"
    r = subprocess.run([os.path.join(examples, "static_reduce"), "local", str(16 << 20), "3"],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["wrong"] == 0, res
    if register:
        assert res["registered_bytes"] >= 2 * (16 << 20) * 4, res
    else:
        assert res["registered_bytes"] == 0, res


def test_small_device_setter_is_collective():
    """sosx_set_small_device_bytes with different limits on two PEs is refused."""
    r = oshrun(2, [sys.executable, os.path.join(ROOT, "tests", "route_mismatch_pe.py"), "setter"],
               timeout=120)
    assert r.returncode != 0, r.stdout
    assert "every PE passes the same limit" in r.stderr, r.stderr[-2000:]


def test_p2p_stall_mid_call_costs_one_timeout():
    """A peer that stops after a call's entry boundary (test hook SOSX_P2P_TEST_STALL_PE):
    the waiting PEs' device waits time out in the call's first device step, and the
    call's two later device steps give up at once instead of each waiting out
    SHMEMX_P2P_TIMEOUT again (one timeout per call, not one per step)."""
    T = 5
    # the hook is compiled into the test build only (the fakerccl twin of the library,
    # here on the p2p transport, so its RCCL stand-in is never called)
    r = oshrun(4, [sys.executable, os.path.join(ROOT, "tests", "p2p_stall_pe.py")], timeout=150,
               extra_env={"SHMEMX_P2P_TIMEOUT": str(T), "SHMEMX_P2P_SIGNAL": "stream",
                          "SOSX_P2P_TEST_STALL_PE": "1",
                          "SOSX_LIBRARY": os.path.join(ROOT, "tests", "fakerccl",
                                                       "libsos_amd_fakerccl.so")})
    t_end = time.time()
    assert r.returncode != 0, r.stdout
    assert "timed out" in r.stderr and "device wait" in r.stderr, r.stderr[-2000:]
    assert "reduction returned" not in r.stdout
    starts = [float(x) for x in re.findall(r"call starts at ([\d.]+)", r.stdout)]
    assert len(starts) == 4, r.stdout
    # one timeout (+ launch, abort and teardown slack); three would be >= 15 s
    assert t_end - max(starts) < 2 * T + 1, (t_end - max(starts), r.stderr[-2000:])


@pytest.mark.parametrize("np_", [1, 2, 3, 4, 6])
def test_team_management(np_):
    """split_strided / split_2d / team-slot pool / translate / config (tools/team_mgmt_check.py)."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tools", "team_mgmt_check.py")], timeout=300)
    ok = re.findall(r"PE (\d+)/\d+: \d+ checks OK", r.stdout)
    assert r.returncode == 0 and sorted(map(int, ok)) == list(range(np_)), r.stdout + r.stderr[-3000:]


def _fracs_above_one(obj, path=""):
    """Every key named frac* whose value is a number above 1, with its path."""
    out = []
    if isinstance(obj, dict):
        for k, v in obj.items():
            if k.startswith("frac") and isinstance(v, (int, float)) and v > 1:
                out.append((path + "/" + k, v))
            out += _fracs_above_one(v, path + "/" + k)
    elif isinstance(obj, list):
        for i, v in enumerate(obj):
            out += _fracs_above_one(v, f"{path}[{i}]")
    return out


@pytest.mark.parametrize("np_", [2, 4])
def test_bench_team_leg(np_):
    """The driver's N > 1 bench path (torch.distributed.run -> bench.py -> team_bench) with
    np_ ranks on this one GPU over the p2p transport: one JSON line whose bitwise self-check
    and adjacent-collective checks are clean on every rank.  (The RCCL leg needs one GPU
    per rank; it reports itself unavailable here.)"""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update({"SHMEMX_TRANSPORT": "p2p", "SHMEMX_DEVICE": "0", "PYTHONPATH": ROOT})
    port = 29400 + np_ * 7 + os.getpid() % 500
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        f"--nproc-per-node={np_}", "--master-addr", "127.0.0.1",
                        "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", str(np_), "--steps", "3", "--warmup", "1",
                        "--nreduce", str((1 << 20) + 3), "--sweep-max", str(4 << 20)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    # the driver reads stdout: rank 0's JSON line and nothing else (gloo's connection
    # lines and any RCCL banner go to stderr)
    assert [ln for ln in r.stdout.splitlines() if ln.strip()] == lines, r.stdout[:2000]
    import json
    res = json.loads(lines[0])
    assert res["n_gpus"] == np_ and res["value"] > 0
    assert res["config"]["transport"] in ("p2p", "p2p_host")
    # np_ ranks on this box's one GPU: the line says so (device map, not a fixed text)
    assert res["config"]["gpus_used"] == 1 and res["config"]["parallelism"] == f"pe{np_}_on_1gpu"
    assert f"{np_} PEs on 1 GPU (shared" in res["config"]["workload"], res["config"]
    assert res["check"]["bitwise_mismatches_all_ranks"] == 0
    # no xGMI link carried these bytes: no link roofline, and no fraction above 1 anywhere
    assert res["team_roofline"]["bound"] == "shared-gpu", res["team_roofline"]
    assert res["team_roofline"]["frac_one_link"] is None, res["team_roofline"]
    assert _fracs_above_one(res) == [], _fracs_above_one(res)
    # both p2p signalling modes measured and checked in every leg
    assert list(res["transports"]) == ["p2p", "p2p_host"], res["transports"]
    for t in ("p2p", "p2p_host"):
        assert res["transports"][t]["bitwise_mismatches_all_ranks"] == 0, res["transports"]
        for coll in res["adjacent_collectives"][t].values():
            assert coll["bitwise_mismatches_all_ranks"] == 0, res["adjacent_collectives"]
        assert res["host_resident"][t]["value_GiBs"] > 0, res["host_resident"]
        for sched in ("rechalving", "recdbl_direct"):
            assert res["schedules"][t][sched]["bitwise_mismatches_all_ranks"] == 0, res["schedules"]
        curve = res["size_curve"][t]
        assert [r["nreduce"] for r in curve] == [1 << 20, (1 << 20) + 3, 4 << 20]
        assert curve[-1]["bitwise_mismatches_all_ranks"] == 0
    # the local combine on every PE at once (the HBM side of the curve)
    assert res["local_combine_all_pes"]["value_GiBs"] > 0, res["local_combine_all_pes"]
    # small / medium calls beside SOS's CPU path, host-heap results equal to the CPU's
    small = res["small_messages"]["rows"]
    assert [r["nreduce"] for r in small] == [1, 1024, 16384, 65536]
    for row in small:
        assert row["host_us"] > 0 and row["device_us"] > 0 and row["cpu_us"] > 0, row
        assert row["device_executor_us"] > 0, row
        assert row["host_bitwise_mismatches_vs_cpu_all_ranks"] == 0, row
        assert row["device_bitwise_mismatches_vs_cpu_all_ranks"] == 0, row
    # the device-heap calls with team size * bytes <= 128 KiB took the shared-memory path
    assert res["small_messages"]["small_path_device_calls_rank0_side"] > 0, res["small_messages"]
    # SOS's ring on np_ host processes beside the line, equal to the GPU ring byte for byte
    cpu = res["cpu_ring_baseline"]
    assert cpu["cores"] == np_ and cpu["value"] > 0 and cpu["kind"] == "port", cpu
    assert cpu["bitwise_mismatches_vs_gpu_ring_all_ranks"] == 0, cpu


@pytest.mark.parametrize("np_", [3, 4])
def test_api_sweep_every_typed_reduction(np_):
    """All 198 typed reductions (154 *_reduce + 44 *_to_all), the 52 typed scans and the 24
    typed broadcasts across np_ real PE processes, host and device buffers, recdbl and
    ring sizes, bit for bit vs the oracle schedules."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "api_sweep_pe.py")], timeout=600)
    ok = re.findall(r"PE (\d+)/\d+: (\d+) checks OK", r.stdout)
    assert r.returncode == 0 and sorted(int(p) for p, _ in ok) == list(range(np_)), \
        r.stdout[-3000:] + r.stderr[-3000:]
    assert all(int(c) == 396 + 104 + 48 for _, c in ok), ok


def test_p2p_stage_overflow_is_an_error(tmp_path):
    """p2p-only transport: a scan whose exchange scratch exceeds SHMEMX_STAGE_BYTES ends the
    job with a message (with RCCL also up -- SHMEMX_TRANSPORT=both -- the call runs on RCCL
    instead; that needs one GPU per PE)."""
    script = tmp_path / "ovf.py"
    script.write_text(
        "import torch\nfrom sos_amd import shmem as S\nS.shmem_init()\n"
        "n = 1 << 20\nsrc = S.shmemx_malloc_device(n * 4)\ndst = S.shmemx_malloc_device(n * 4)\n"
        "S.shmemx_float_sum_inscan(S.team_world(), dst, src, n)\nprint('no error')\n")
    env_stage = dict(os.environ, SHMEMX_STAGE_BYTES="1M")
    env = dict(env_stage)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update({"SHMEMX_TRANSPORT": "p2p", "SHMEMX_DEVICE_HEAP_SIZE": "64M", "SHMEMX_DEVICE": "0",
                "PYTHONPATH": ROOT})
    r = subprocess.run([sys.executable, OSHRUN, "-np", "2", "--timeout", "100", sys.executable,
                        str(script)], capture_output=True, text=True, timeout=150, env=env)
    assert r.returncode != 0 and "no error" not in r.stdout
    assert "exceed the p2p stage region" in r.stderr, r.stderr[-2000:]


@pytest.mark.parametrize("heap", ["2G", "3400M"])
def test_ipc_heap_sizes_with_bit31(heap):
    """torch's HIP 7.0.2 hangs in hipIpcOpenMemHandle for exported sizes with bit 31 set;
    the library rounds such heaps up (tests/heap_init_pe.py; /opt/rocm 7.2 maps them all)."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update({"SHMEMX_TRANSPORT": "p2p", "SHMEMX_DEVICE_HEAP_SIZE": heap, "SHMEMX_DEVICE": "0",
                "SHMEMX_STAGE_BYTES": "64M", "PYTHONPATH": ROOT})
    r = subprocess.run([sys.executable, OSHRUN, "-np", "2", "--timeout", "60", sys.executable,
                        os.path.join(ROOT, "tests", "heap_init_pe.py")],
                       capture_output=True, text=True, timeout=90, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert r.stdout.count("PE done") == 2, r.stdout


@pytest.mark.parametrize("np_,signal", [(2, "host"), (3, "host"), (8, "host"), (3, "stream")])
def test_team_check_host_stripes(np_, signal):
    """Host-resident ring reductions pipelined in stripes (striped_host_ring): with 256-B
    chunk slices the host-buffer calls of tests/team_check_pe.py run as many stripes plus
    the n mod P remainder stripe (p2p stripes only when SHMEMX_HOST_STRIPE_BYTES is set),
    bit for bit against the CPU oracle."""
    env = {"SHMEMX_HOST_STRIPE_BYTES": "256", "SHMEMX_P2P_SIGNAL": signal}
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "team_check_pe.py")], timeout=900,
               extra_env=env)
    ok = re.findall(r"PE (\d+)/\d+: \d+ checks OK \(p2p signal (\w+)[,)]", r.stdout)
    assert r.returncode == 0 and sorted(int(p) for p, _ in ok) == list(range(np_)), \
        r.stdout + r.stderr[-3000:]
    assert {m for _, m in ok} == {signal}, ok


def test_bench_team_leg_default_transport():
    """bench.py's N > 1 default (SHMEMX_TRANSPORT=both, what the driver's 8-GPU run uses),
    here with 2 ranks on one GPU: RCCL refuses a second rank on the device, so in the
    preflight job init falls back -- on every PE, agreed over the bootstrap -- to the p2p
    transport; the bench job then brings up p2p only, and the line comes out with clean
    checks."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "SHMEMX_TRANSPORT"):
        env.pop(k, None)
    env.update({"SHMEMX_DEVICE": "0", "PYTHONPATH": ROOT})
    port = 29700 + os.getpid() % 500
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr", "127.0.0.1",
                        "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--nreduce", str((1 << 20) + 3), "--sweep-max", str(4 << 20)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    import json
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["config"]["transport"] in ("p2p", "p2p_host")
    assert list(res["transports"]) == ["p2p", "p2p_host"]
    assert res["check"]["bitwise_mismatches_all_ranks"] == 0
    # the preflight job found RCCL down (init refused, every PE fell back) and p2p clean,
    # so this job brought up p2p only
    assert res["preflight"]["ran"] and res["preflight"]["ok"] == \
        {"rccl": False, "rccl_ag": False, "p2p": True, "p2p_host": True,
         "rccl_ar": False}, res["preflight"]
    assert "preflight: transports ['rccl', 'rccl_ag', 'rccl_ar'] disabled" in r.stderr
