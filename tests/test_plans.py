"""CPU: every per-PE plan, simulated across P PEs, reproduces the SOS schedule.

  ring          == SOS ring (src/collectives.c:647-764) bit for bit, every type/op
  recdbl        == SOS recdbl_sw (src/collectives.c:850-984) bit for bit, per PE
  recdbl_gather == SOS recdbl_sw bit for bit, per PE, after one all-gather round
  rechalving    == SOS recdbl_sw for commutative element semantics
  recdbl_direct == SOS recdbl_sw for commutative element semantics
Also: SOS AUTO crossover, chunk math, in-place calls, ragged/empty chunks.
"""
import numpy as np
import pytest

from oracle import oracle as O
from sos_amd import shmem as S

import plansim

CASES = [  # (dtype, op, dist)
    (23, 5, 0),   # float sum
    (24, 6, 1),   # double prod
    (11, 2, 0),   # int64 xor
    (11, 0, 0),   # int64 and
    (4, 4, 0),    # int max
    (18, 3, 0),   # uint8 min (SOS maps uint8 -> INT8: signed compare)
    (1, 5, 0),    # char sum (signed, wraps)
    (27, 6, 1),   # complexd prod
    (26, 5, 0),   # complexf sum
    (16, 1, 0),   # ulong or
]


def bits(a):
    return np.frombuffer(a.tobytes(), np.uint8)


@pytest.mark.parametrize("P", [2, 3, 4, 5, 7, 8])
@pytest.mark.parametrize("dt,op,dist", CASES)
def test_ring_plan_matches_sos_ring(P, dt, op, dist):
    for n in (1, 5, 64, 1001):
        srcs = [O.fill(dt, dist, 11 + n, p, n) for p in range(P)]
        ref = O.ring(op, dt, srcs)
        got = plansim.simulate("ring", op, dt, srcs)
        for p in range(P):
            assert np.array_equal(bits(got[p]), bits(ref[p])), (P, n, p)


@pytest.mark.parametrize("alg", ["recdbl", "recdbl_gather"])
@pytest.mark.parametrize("P", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("dt,op,dist", CASES)
def test_recdbl_plan_matches_sos_recdbl(alg, P, dt, op, dist):
    for n in (1, 7, 300):
        srcs = [O.fill(dt, dist, 3 + n, p, n) for p in range(P)]
        ref = O.recdbl(op, dt, srcs)
        got = plansim.simulate(alg, op, dt, srcs)
        for p in range(P):
            assert np.array_equal(bits(got[p]), bits(ref[p])), (alg, P, n, p)


@pytest.mark.parametrize("alg", ["rechalving", "recdbl_direct"])
@pytest.mark.parametrize("P", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("dt,op,dist", [c for c in CASES if c[:2] != (4, 4) and c[:2] != (18, 3)])
def test_tree_plans_match_sos_recdbl(alg, P, dt, op, dist):
    """Commutative element semantics: every PE ends with recdbl_sw's value."""
    for n in (1, 3, 100, 1027):
        srcs = [O.fill(dt, dist, 5 + n, p, n) for p in range(P)]
        ref = O.recdbl(op, dt, srcs)
        got = plansim.simulate(alg, op, dt, srcs)
        for p in range(P):
            assert np.array_equal(bits(got[p]), bits(ref[0])), (alg, P, n, p)


@pytest.mark.parametrize("alg", ["ring", "recdbl", "rechalving", "recdbl_direct", "recdbl_gather"])
def test_in_place(alg):
    P, n, dt, op = 5, 333, 23, 5
    srcs = [O.fill(dt, 0, 77, p, n) for p in range(P)]
    ref = O.ring(op, dt, srcs) if alg == "ring" else O.recdbl(op, dt, srcs)
    got = plansim.simulate(alg, op, dt, srcs, in_place=True)
    for p in range(P):
        assert np.array_equal(bits(got[p]),
                              bits(ref[p if alg in ("ring", "recdbl", "recdbl_gather") else 0]))


@pytest.mark.parametrize("alg", ["recdbl", "recdbl_gather"])
@pytest.mark.parametrize("P", [3, 4, 6, 8])
@pytest.mark.parametrize("op", [3, 4, 5])
def test_minmax_ties_recdbl_per_pe(alg, P, op):
    """fp min/max/sum with +-0 ties and NaNs: recdbl keeps every PE's own perspective."""
    n = 256
    rng = np.random.default_rng(3 + P)
    pool = np.array([0.0, -0.0, np.nan, -np.nan, 1.0, -1.0], dtype=np.float32)
    srcs = [rng.choice(pool, n).astype(np.float32) for _ in range(P)]
    # distinct NaN payloads per PE, so the x86 first-operand NaN rule shows too
    for p, a in enumerate(srcs):
        v = a.view(np.uint32)
        v[np.isnan(a)] |= np.uint32(p + 1)
    ref = O.recdbl(op, 23, srcs)
    got = plansim.simulate(alg, op, 23, srcs)
    for p in range(P):
        assert np.array_equal(bits(got[p]), bits(ref[p])), (alg, P, op, p)
    # and the PEs genuinely disagree (perspective matters), so the check has teeth
    assert any(not np.array_equal(bits(ref[0]), bits(ref[p])) for p in range(1, P))


def test_auto_crossover():
    # SOS AUTO without NIC atomics: recdbl_sw below COLL_SIZE_CROSSOVER (16 KiB), else ring;
    # the recdbl_sw results come from the one-round gather form (same bits per PE)
    lib = S.lib()
    assert lib.sosx_resolve_alg(0, 16383, 16384) == 5
    assert lib.sosx_resolve_alg(0, 16384, 16384) == 2
    assert lib.sosx_resolve_alg(3, 16, 16384) == 3


def test_ring_chunks_follow_sos():
    """Owner chunk sizes/offsets of the ring plans are SOS's (src/collectives.c:697-709)."""
    for P in (2, 3, 5, 8):
        for n in (1, 7, 8, 9, 1000):
            ts = 4
            for me in range(P):
                pl = S.plan("ring", P, me, n, ts)
                q, r = divmod(n, P)
                cnt = q + (me < r)
                first = me * cnt if me < r else me * cnt + r
                folds = [o for rd in pl["rounds"] for o in rd["ops"]]
                if cnt == 0:
                    assert not folds
                else:
                    assert folds[0]["count"] == cnt and folds[0]["out"] == (1, first * ts)


def test_wire_bytes():
    """Bytes sent per PE: 2(P-1)/P n s for ring/rechalving (P pow2), log2(P) n s for recdbl."""
    n, ts = 4096, 4
    for P in (2, 4, 8):
        for alg, expect in (("ring", 2 * (P - 1) * n * ts // P), ("rechalving", 2 * (P - 1) * n * ts // P),
                            ("recdbl", int(np.log2(P)) * n * ts)):
            pl = S.plan(alg, P, 0, n, ts)
            sent = sum(x["bytes"] for rd in pl["rounds"] for x in rd["xfers"] if x["send"])
            assert sent == expect, (alg, P, sent, expect)
        pl = S.plan("recdbl_gather", P, 0, n, ts)
        assert len(pl["rounds"]) == 1  # one exchange round whatever P
        sent = sum(x["bytes"] for rd in pl["rounds"] for x in rd["xfers"] if x["send"])
        assert sent == (P - 1) * n * ts
