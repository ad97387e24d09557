"""GPU, several PE processes on one MI355X: the RCCL executor end to end.

Real RCCL refuses two ranks on one GPU, so these runs load a test build of the library,
tests/fakerccl/libsos_amd_fakerccl.so: the same objects as sos_amd/libsos_amd.so, with the
ten RCCL entry points it calls bound to tests/fakerccl/fake_rccl.cpp, which moves each
ncclSend/ncclRecv through a /dev/shm file with RCCL's per-pair FIFO matching.  Everything
above those calls is the product code the 8-GPU node runs with SHMEMX_TRANSPORT=rccl: the
plans, exec_rccl's byte offsets and groups, the folds between rounds, the striped
host-resident ring, the RCCL device barrier.  The checkers are the ones the p2p runs use
(bit-exact against an on-GPU re-evaluation of each schedule's element order).
"""
import glob
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OSHRUN = os.path.join(ROOT, "tools", "oshrun")
FAKE = os.path.join(ROOT, "tests", "fakerccl", "libsos_amd_fakerccl.so")


def _env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update({"SOSX_LIBRARY": FAKE, "SHMEMX_TRANSPORT": "rccl", "SHMEMX_DEVICE": "0",
                "SHMEMX_DEVICE_HEAP_SIZE": "256M", "FAKERCCL_TIMEOUT": "60", "FAKERCCL_STATS": "1", "PYTHONPATH": ROOT})
    return env


@pytest.fixture(autouse=True)
def _no_leftover_messages():
    assert os.path.exists(FAKE), "tests/fakerccl/libsos_amd_fakerccl.so is not built"
    yield
    left = glob.glob("/dev/shm/fakerccl_*")
    for f in left:
        os.unlink(f)
    assert not left, f"unreceived messages: {left[:4]}"


def oshrun(np_, cmd, timeout=600, **extra):
    env = _env()
    env.update(extra)
    return subprocess.run([sys.executable, OSHRUN, "-np", str(np_), "--timeout", str(timeout - 30),
                           *cmd], capture_output=True, text=True, timeout=timeout, env=env)


def _ok(r, np_):
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    ok = re.findall(r"PE (\d+)/\d+: \d+ checks OK", r.stdout)
    assert sorted(int(p) for p in ok) == list(range(np_)), r.stdout[-3000:]
    _used_fake(r, np_)


def _used_fake(r, np_):
    """Every rank moved data through the stand-in (so the RCCL executor ran) without error."""
    assert "fakerccl error" not in r.stderr, r.stderr[-2000:]
    sent = {int(rk): int(m) for rk, m in
            re.findall(r"fakerccl stats: rank (\d+) sent (\d+) messages", r.stderr)}
    assert sorted(sent) == list(range(np_)) and min(sent.values()) > 0, r.stderr[-2000:]


@pytest.mark.parametrize("np_", [2, 3, 4])
def test_team_check_rccl_executor(np_):
    """Every schedule, 8 type/op pairs, heap / device / host buffers, in place, a split team
    (small device operands on the executor too: SHMEMX_SMALL_DEVICE=0)."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "team_check_pe.py")], timeout=900,
               SHMEMX_SMALL_DEVICE="0")
    _ok(r, np_)


@pytest.mark.parametrize("np_", [2, 4])
def test_team_check_rccl_native_allgather(np_):
    """SHMEMX_RCCL_ALLGATHER=1: equal-chunk allgather rounds of world-team plans go through
    ncclAllGather (counted by the stand-in); every check stays bit-exact."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "team_check_pe.py")], timeout=900,
               SHMEMX_RCCL_ALLGATHER="1")
    _ok(r, np_)
    ag = {int(rk): int(a) for rk, a in
          re.findall(r"fakerccl stats: rank (\d+) sent \d+ messages, \d+ bytes, (\d+) allgathers",
                     r.stderr)}
    assert sorted(ag) == list(range(np_)) and min(ag.values()) > 0, r.stderr[-2000:]


@pytest.mark.parametrize("np_", [3])
def test_coll_check_rccl_executor(np_):
    """Scans and broadcasts over the RCCL executor (small device operands included)."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "coll_check_pe.py")], timeout=600,
               SHMEMX_SMALL_DEVICE="0")
    _ok(r, np_)


def test_team_management_rccl(np_=4):
    """Team management with its reductions on the RCCL executor (their host operands would
    otherwise take the shared-memory small path, which moves nothing through RCCL)."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tools", "team_mgmt_check.py")], timeout=300,
               SHMEMX_SMALL_HOST="0")
    _ok(r, np_)


def test_team_management_small_path(np_=4):
    """The same checks with the default small host-resident path: every reduction of the
    checker (8-byte host operands) runs through node shared memory, none through RCCL."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tools", "team_mgmt_check.py")], timeout=300)
    ok = re.findall(r"PE (\d+)/\d+: \d+ checks OK", r.stdout)
    assert r.returncode == 0 and sorted(map(int, ok)) == list(range(np_)), r.stdout + r.stderr[-3000:]
    assert "fakerccl error" not in r.stderr, r.stderr[-2000:]


def test_api_sweep_rccl(np_=2):
    """All 154 typed reductions and 44 to_all entry points through the public API (small
    device operands on the executor too: SHMEMX_SMALL_DEVICE=0)."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "api_sweep_pe.py")], timeout=600,
               SHMEMX_SMALL_DEVICE="0")
    _ok(r, np_)


@pytest.mark.parametrize("np_", [2, 3])
def test_api_sweep_rccl_native_allreduce(np_):
    """SHMEMX_RCCL_ALLREDUCE=1: every integer sum/prod/min/max of an 8/32/64-bit type over
    the world team runs as one ncclAllReduce (counted by the stand-in, which folds in rank
    order), and all 198 typed reductions still match the oracle's SOS schedules bit for
    bit (integer results do not depend on the order); 16-bit, bitwise, fp, complex and
    long double calls keep their schedules."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "api_sweep_pe.py")], timeout=600,
               SHMEMX_RCCL_ALLREDUCE="1")
    _ok(r, np_)
    ar = {int(rk): int(a) for rk, a in
          re.findall(r"fakerccl stats: rank (\d+) .* (\d+) allreduces", r.stderr)}
    assert sorted(ar) == list(range(np_)) and min(ar.values()) > 0, r.stderr[-2000:]


@pytest.mark.parametrize("np_", [2, 4])
def test_team_check_rccl_native_allreduce(np_):
    """The same switch under tests/team_check_pe.py: world-team integer calls through
    ncclAllReduce, split-team calls (not world-shaped) on their schedules, all bit-exact."""
    r = oshrun(np_, [sys.executable, os.path.join(ROOT, "tests", "team_check_pe.py")], timeout=900,
               SHMEMX_RCCL_ALLREDUCE="1")
    _ok(r, np_)


def test_bench_team_leg_rccl():
    """bench.py's N > 1 line as the driver runs it on the 8-GPU node, transport forced to
    RCCL: the headline ring, the size curve, rechalving / recdbl_direct, and the
    host-resident (striped) leg, each with a bitwise check on every rank."""
    env = _env()
    port = 29200 + os.getpid() % 500
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr", "127.0.0.1",
                        "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--nreduce", str((1 << 20) + 3), "--sweep-max", str(4 << 20)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    _used_fake(r, 2)
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["config"]["transport"] in ("rccl", "rccl_ag"), res["config"]
    assert res["check"]["bitwise_mismatches_all_ranks"] == 0, res["check"]
    assert list(res["transports"]) == ["rccl", "rccl_ag", "rccl_ar"], res["transports"]
    # RCCL's own allreduce (the stand-in folds in rank order): within the fp bound; at
    # P = 2 the two orders are a commutative swap, so also bit for bit
    ar = res["transports"]["rccl_ar"]
    assert ar["fp_tolerance_violations_all_ranks"] == 0 and ar["bitwise_mismatches_all_ranks"] == 0, ar
    assert res["size_curve"]["rccl_ar"][-1]["fp_tolerance_violations_all_ranks"] == 0
    assert "rccl_ar" not in res["schedules"] and "rccl_ar" not in res["host_resident"]
    for t in ("rccl", "rccl_ag"):
        assert res["transports"][t]["bitwise_mismatches_all_ranks"] == 0, res["transports"]
        for coll in res["adjacent_collectives"][t].values():
            assert coll["bitwise_mismatches_all_ranks"] == 0, res["adjacent_collectives"]
        assert res["host_resident"][t]["value_GiBs"] > 0, res["host_resident"]
        for sched in ("rechalving", "recdbl_direct"):
            assert res["schedules"][t][sched]["bitwise_mismatches_all_ranks"] == 0, res["schedules"]
        curve = res["size_curve"][t]
        assert curve[-1]["bitwise_mismatches_all_ranks"] == 0   # 4Mi: equal chunks


def test_bench_spawns_ranks_without_launcher():
    """`python bench.py --gpus 2` with no launcher environment (as the driver may call it):
    bench.py starts both rank processes itself, and the one line says n_gpus 2 with the
    communicator's rank count (the stand-in's ncclCommCount) 2 on both ranks."""
    env = _env()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "2", "--warmup", "1", "--no-cpu", "--no-host", "--no-adjacent",
                        "--no-team-sweep", "--no-small", "--no-pmc", "--nreduce", str((1 << 20) + 3)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    _used_fake(r, 2)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["rccl_comm_ranks"] == [2, 2], res
    assert res["check"]["bitwise_mismatches_all_ranks"] == 0
    assert abs(res["algbw_GiBs"] * 2 - res["value"]) < 0.01 * res["value"], res


def test_bench_rccl_allreduce_is_checked_by_tolerance():
    """Four PEs: RCCL's own allreduce order (the stand-in folds in rank order) differs
    from SOS's ring for fp sum, so rccl_ar shows bitwise mismatches, stays inside the fp
    bound, and is never the transport `value` comes from.  (Not 3: the bench's inputs
    are multiples of 2^-23 in [-1, 1), so every partial sum of two is exact and 3-PE sums
    agree in any order.)"""
    env = _env()
    port = 29050 + os.getpid() % 500
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=4", "--master-addr", "127.0.0.1",
                        "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "4", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-host",
                        "--no-adjacent", "--nreduce", str((1 << 20) + 3),
                        "--sweep-max", str(4 << 20)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    ar = res["transports"]["rccl_ar"]
    assert ar["bitwise_mismatches_all_ranks"] > 0, ar
    assert ar["fp_tolerance_violations_all_ranks"] == 0, ar
    assert res["size_curve"]["rccl_ar"][-1]["fp_tolerance_violations_all_ranks"] == 0
    assert res["config"]["transport"] in ("rccl", "rccl_ag"), res["config"]
    assert res["check"]["bitwise_mismatches_all_ranks"] == 0
    assert res["preflight"]["ok"]["rccl_ar"], res["preflight"]


def test_bench_preflight_drops_a_hanging_transport():
    """The N > 1 bench's preflight against a transport that hangs: both transports are up
    (SHMEMX_TRANSPORT=both, RCCL through the stand-in), and in the preflight job PE 1
    vanishes when it reaches p2p, so PE 0's p2p call meets the real bounded wait (20 s in
    the preflight) and ends that process.  The bench job must then bring up RCCL only and
    print a clean line from both RCCL variants."""
    env = _env()
    env["SOSX_PREFLIGHT_FAULT"] = "p2p:1"
    env.pop("SHMEMX_TRANSPORT")   # the bench's own default (both), as the driver runs it
    port = 29100 + os.getpid() % 500
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr", "127.0.0.1",
                        "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu",
                        "--nreduce", str((1 << 20) + 3), "--sweep-max", str(4 << 20)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["preflight"]["ok"] == {"rccl": True, "rccl_ag": True, "p2p": False,
                                      "p2p_host": False, "rccl_ar": False}, res["preflight"]
    assert "timed out" in r.stderr, r.stderr[-3000:]
    assert list(res["transports"]) == ["rccl", "rccl_ag"], res["transports"]
    assert res["config"]["transport"] in ("rccl", "rccl_ag")
    assert res["check"]["bitwise_mismatches_all_ranks"] == 0, res["check"]


@pytest.mark.parametrize("script", ["tests/team_check_pe.py", "tools/team_mgmt_check.py"])
def test_init_attr_multi_pe(tmp_path, script, np_=3):
    """shmemx_init_attr across 3 processes (unique id passed out of band, no bootstrap hub):
    RCCL barriers and the RCCL team-word agreement under the team checkers."""
    procs = []
    for pe in range(np_):
        env = _env()
        for k in ("SHMEM_PE", "SHMEM_NPES", "SHMEM_BOOTSTRAP_ADDR", "SHMEM_BOOTSTRAP_PORT"):
            env.pop(k, None)
        env.update({"INIT_ATTR_PE": str(pe), "INIT_ATTR_NPES": str(np_),
                    "INIT_ATTR_UID_FILE": str(tmp_path / "uid")})
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "tests", "init_attr_pe.py"),
             os.path.join(ROOT, script)],
            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=400))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    out = "".join(o for o, _ in outs)
    err = "".join(e for _, e in outs)
    rcs = [p.returncode for p in procs]

    class R:
        returncode = max(rcs, key=abs)
        stdout, stderr = out, err
    _ok(R, np_)
