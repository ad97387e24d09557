"""CPU: `python bench.py --gpus N` with no launcher environment starts its N rank
processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets
them, from a parent that never touches the GPU) and forwards rank 0's one JSON line; a
launcher whose WORLD_SIZE differs from --gpus is an error, never an N = 1 line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_bench_spawns_its_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--launch-check"], capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["launch_check"] and res["n_gpus"] == 2
    assert sorted(x["rank"] for x in res["ranks"]) == [0, 1]
    assert sorted(x["local_rank"] for x in res["ranks"]) == [0, 1]
    assert len({x["pid"] for x in res["ranks"]}) == 2


def test_bench_rejects_a_mismatched_launcher():
    env = _env()
    env.update({"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8",
                        "--launch-check"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and r.stdout.strip() == "", (r.returncode, r.stdout)
    assert "WORLD_SIZE=1" in r.stderr


def test_bench_spawn_reports_a_failed_rank(tmp_path):
    """A rank that fails makes the whole run fail, with no line on stdout."""
    sys.path.insert(0, ROOT)
    import bench
    rc, line = bench.spawn_ranks(2, ["--launch-check", "--nreduce", "not-a-number"], grace_s=5)
    assert rc != 0 and line is None
