"""GPU: bench.py's N = 1 line (the driver's BENCH run), shortened: the contract keys, a
roofline fraction that is an HBM fraction, and a size curve whose frac_hbm comes from
HBM-streamed launches (operand pairs rotated past the Infinity Cache), never above 1,
with the cache-resident timings labelled as such."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_n1_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "10", "--warmup", "2",
                        "--no-pmc", "--no-host", "--no-adjacent", "--cpu-seconds", "0.5",
                        "--sweep-max", str(16 << 20)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    # the driver reads stdout: the JSON line and nothing else
    assert [ln for ln in r.stdout.splitlines() if ln.strip()] == lines, r.stdout[:2000]
    res = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in res, k
    assert res["n_gpus"] == 1 and res["steps"] == 10 and res["dtype"] == "f32"
    roof = res["roofline"]
    assert roof["bound"] == "hbm" and 0 < roof["frac"] <= 1 and roof["peak"] == 8000.0
    rows = res["size_curve"]["rows"]
    assert [row["nreduce"] for row in rows] == [1 << 20, 4 << 20, 16 << 20]
    for row in rows:
        assert 0 < row["frac_hbm"] <= 1, row
        assert row["operand_pairs_rotated"] * 2 * row["nreduce"] * 4 >= 1 << 30, row
        assert row["cache_resident"] == (3 * row["nreduce"] * 4 <= 256 << 20), row
        assert row["cpu_GiBs"] > 0
    # operands from the device symmetric heap, started an odd multiple of 4 KiB apart in
    # the 32 KiB channel interleave; the torch-allocator pair is reported beside it
    assert res["operands"]["in_minus_inout_mod_32KiB"] % 8192 == 4096, res["operands"]
    assert 0 < res["torch_allocator_buffers"]["frac"] <= 1
    cpu = res["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["cores"] == 1 and cpu["value"] > 0
