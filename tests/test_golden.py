"""Known-answer vectors (tests/golden/reductions.json, made by tests/golden/make_golden.py).

CPU : the oracle still reproduces every stored answer (inputs and outputs, SHA-256 and
      the full bytes of the n <= 7 cases) -- an oracle change cannot move silently.
GPU : the device path reproduces the stored answers with no oracle in the loop: inputs
      from the device generator (sosx_fill), combine = sosx_combine, ring / recdbl = the
      per-PE plans on the single-GPU loopback team (the RCCL executor's plans and kernels).
"""
import hashlib
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "reductions.json")))
CASES = GOLDEN["cases"]
SEED = GOLDEN["seed"]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_golden_covers_survey_8c():
    kinds = {(c["kind"], c["P"]) for c in CASES}
    assert {("combine", 2)} | {(k, p) for k in ("ring", "recdbl") for p in (1, 2, 3, 4, 8)} == kinds
    assert {c["n"] for c in CASES} == {1, 7, 4097, 65536}
    assert {c["config"] for c in CASES} == {"#2", "#3", "#4", "#5"}


def test_oracle_reproduces_golden():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden as G
    for c in CASES:
        ins, outs = G.compute(c["kind"], c["type"], c["op"], c["n"], c["P"])
        assert [sha(a.tobytes()) for a in ins] == c["in_sha256"], c
        assert [sha(a.tobytes()) for a in outs] == c["out_sha256"], c
        if "out_hex" in c:
            assert [a.tobytes().hex() for a in outs] == c["out_hex"], c


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["#2", "#3", "#4", "#5"])
def test_gpu_reproduces_golden(torch_cuda, sos, config):
    """One test per BASELINE config, so a failure names the config it broke."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import golden_gpu
    cases = [c for c in CASES if c["config"] == config]
    bad = golden_gpu.run_cases(torch_cuda, sos, cases, SEED)
    assert not bad, f"{len(bad)} of {len(cases)} golden cases of {config} differ: {bad[:10]}"
    _ = np


@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 2, 4, 8])
def test_gpu_pi_reduce_known_answer(torch_cuda, sos, P):
    """BASELINE config #1: examples/pi_reduce.c's golden line per PE count, with its two
    long long sum reductions through the GPU loopback recdbl_sw."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import golden_gpu
    assert golden_gpu.pi_lines_gpu(torch_cuda, P) == [golden_gpu.GOLDEN_PI[P]] * P
