"""CPU: the -m gpu run grades BASELINE.json's configs first (conftest.py
pytest_collection_modifyitems), so a cut-short or partly failing driver run still has
every config's parity result: the golden known answers of configs #1-#5, then the
full-size configs, then pi_reduce as PE processes, then everything else in file order
(no test is moved to the end: round 4's run-it-last ordering of the 12-PE team check is
gone with the cause it hid)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpu_collection_starts_with_the_configs():
    r = subprocess.run([sys.executable, "-m", "pytest", "tests", "--collect-only", "-q", "-m", "gpu",
                        "-p", "no:cacheprovider"], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    ids = [ln for ln in r.stdout.splitlines() if "::" in ln]
    files = [i.split("::")[0].rsplit("/", 1)[-1] for i in ids]
    n_golden = files.count("test_golden.py")
    n_cfg = files.count("test_gpu_configs.py")
    assert n_golden >= 8 and n_cfg >= 20
    assert set(files[:n_golden]) == {"test_golden.py"}, ids[:n_golden]
    assert set(files[n_golden:n_golden + n_cfg]) == {"test_gpu_configs.py"}
    pi = [i for i in ids if "test_pi_reduce_multi_pe" in i]
    assert ids[n_golden + n_cfg:n_golden + n_cfg + len(pi)] == pi and len(pi) == 3
    # every config is named by a golden test, #1 as the pi_reduce known answer
    golden = " ".join(ids[:n_golden])
    for cfg in ("#2", "#3", "#4", "#5"):
        assert f"test_gpu_reproduces_golden[{cfg}]" in golden
    assert "test_gpu_pi_reduce_known_answer[2]" in golden
    # after the configs, file order: the 12-PE team check sits among its own file's tests
    mp = [i for i in ids if "test_gpu_multipe.py::" in i]
    assert any("test_team_check[12-" in i for i in mp)
    assert not ids[-1].rsplit("/", 1)[-1].startswith("test_gpu_multipe.py::test_team_check[12-")
