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
def test_gpu_reproduces_golden(torch_cuda, sos):
    from sos_amd import shmem as S
    torch = torch_cuda
    ESZ = {4: 4, 11: 8, 23: 4, 24: 8, 27: 16}
    bad = []
    for c in CASES:
        dt, op, n, P = c["type"], c["op"], c["n"], c["P"]
        es = ESZ[dt]
        dist = 1 if op == 6 else 0
        npe = 2 if c["kind"] == "combine" else P
        src = []
        for pe in range(npe):
            t = torch.empty(n * es, dtype=torch.uint8, device="cuda")
            sos.fill(dt, dist, SEED, pe, t.data_ptr(), n)
            src.append(t)
        torch.cuda.synchronize()
        if [sha(t.cpu().numpy().tobytes()) for t in src] != c["in_sha256"]:
            bad.append(("inputs", c["kind"], dt, op, n, P))
            continue
        if c["kind"] == "combine":
            sos.combine(op, dt, src[0].data_ptr(), src[1].data_ptr(), n)
            outs = [src[0]]
        else:
            outs = [torch.zeros_like(t) for t in src]
            S.loopback_allreduce(c["kind"], op, dt, [t.data_ptr() for t in src],
                                 [t.data_ptr() for t in outs], n)
        torch.cuda.synchronize()
        got = [sha(t.cpu().numpy().tobytes()) for t in outs]
        if got != c["out_sha256"]:
            bad.append((c["kind"], dt, op, n, P))
    assert not bad, f"{len(bad)} of {len(CASES)} golden cases differ: {bad[:10]}"
    _ = np
