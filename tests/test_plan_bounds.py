"""CPU: the plan builder under AddressSanitizer + UBSan (host code only).

tests/plan_bounds.cpp is compiled with g++ -fsanitize=address,undefined together with
sos_amd/csrc/plan.cpp and checks, for every schedule, team size, PE, ragged count and
element size, that each transfer and local op stays inside its buffer (the executors
turn these offsets into raw device pointers) and that sends and receives pair up FIFO
per ordered PE pair.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_plan_bounds_under_asan(tmp_path):
    exe = tmp_path / "plan_bounds"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=undefined", f"-I{ROOT}/include",
                        f"-I{ROOT}/sos_amd/csrc", f"{ROOT}/tests/plan_bounds.cpp",
                        f"{ROOT}/sos_amd/csrc/plan.cpp", "-o", str(exe)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "plans OK" in r.stdout
