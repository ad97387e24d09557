"""CPU: the scan and broadcast plans, simulated across P PEs, reproduce SOS.

  inscan / exscan == SOS scan_ring (src/collectives.c:1111-1209) bit for bit: the
                     in-order prefix ((s_0 OP s_1) OP ...) OP s_i, PE 0 zero for exscan
  broadcast       == SOS bcast (src/collectives.c:429-485): every non-root receives the
                     root's source; the root's target is written only by the team forms
Also: in-place scans, misaligned operands, ragged/empty chunks, teams above the
direct reductions' 8 PEs, wire bytes of the split broadcast.
"""
import numpy as np
import pytest

from oracle import oracle as O
from sos_amd import _lib, shmem as S

import plansim

SCAN_CASES = [  # (dtype, dist): the sum scans exist for the SUM_PROD types
    (23, 0),   # float
    (24, 0),   # double
    (4, 0),    # int
    (1, 0),    # char (signed, wraps)
    (18, 0),   # uint8
    (27, 0),   # complexd
    (26, 0),   # complexf
    (25, 0),   # long double (x87)
]


def bits(a):
    return np.frombuffer(a.tobytes(), np.uint8)


def src_of(dt, dist, seed, pe, n):
    if dt == 25:  # long double: the synthetic generator has no x87 leg; numpy's is x87
        return np.random.default_rng(seed * 131 + pe).standard_normal(n).astype(np.longdouble)
    return O.fill(dt, dist, seed, pe, n)


@pytest.mark.parametrize("exclusive", [False, True])
@pytest.mark.parametrize("P", [1, 2, 3, 5, 8, 12])
@pytest.mark.parametrize("dt,dist", SCAN_CASES)
def test_scan_plan_matches_sos_scan(exclusive, P, dt, dist):
    alg = _lib.PLAN_EXSCAN if exclusive else _lib.PLAN_INSCAN
    for n in (1, 5, 64, 1001):
        srcs = [src_of(dt, dist, 7 + n, p, n) for p in range(P)]
        ref = O.scan(5, dt, srcs, exclusive)
        got = plansim.simulate(alg, 5, dt, srcs)
        for p in range(P):
            assert np.array_equal(bits(got[p]), bits(ref[p])), (P, n, p)


@pytest.mark.parametrize("exclusive", [False, True])
@pytest.mark.parametrize("P", [2, 3, 4, 9])
def test_scan_in_place_and_misaligned(exclusive, P):
    alg = _lib.PLAN_EXSCAN if exclusive else _lib.PLAN_INSCAN
    dt = 24
    for n in (3, 257):
        srcs = [O.fill(dt, 0, 3, p, n) for p in range(P)]
        ref = O.scan(5, dt, srcs, exclusive)
        for in_place, mis in ((True, (0, 0)), (False, (8, 8)), (True, (8, 8))):
            got = plansim.simulate(alg, 5, dt, srcs, in_place=in_place, mis=mis)
            for p in range(P):
                assert np.array_equal(bits(got[p]), bits(ref[p])), (P, n, p, in_place, mis)


def test_scan_prefix_local_owns_alias():
    # the PREFIX op marks the input that aliases this PE's target chunk (in-place scans)
    for exclusive, alg in ((False, _lib.PLAN_INSCAN), (True, _lib.PLAN_EXSCAN)):
        for P in (3, 12):
            for me in range(P):
                pl = S.plan(alg, P, me, 1000, 4)
                pre = [l for r in pl["rounds"] for l in r["ops"] if l["kind"] == plansim.PREFIX]
                assert len(pre) == 1
                ins = pre[0]["ins"]
                assert len(ins) == (P - 1 if exclusive else P)
                assert len(pre[0]["outs"]) == len(ins)
                srcs = [i for i, (b, _) in enumerate(ins) if b == plansim.SRC]
                assert srcs == ([me] if me < len(ins) else [])


@pytest.mark.parametrize("P", [1, 2, 3, 4, 7, 8, 9])
@pytest.mark.parametrize("copy_root", [False, True])
def test_bcast_plan_matches_sos_bcast(P, copy_root):
    rng = np.random.default_rng(P)
    for nbytes in (1, 100, 65535, 65536, 200001):
        for dtype in (np.uint8, np.uint32, np.uint64):
            n = max(1, nbytes // np.dtype(dtype).itemsize)
            for root in sorted({0, P - 1, P // 2}):
                srcs = [rng.integers(0, 255, n * np.dtype(dtype).itemsize, dtype=np.uint8).view(dtype)
                        for _ in range(P)]
                init = [np.full(n, 0xA5, dtype) for _ in range(P)]
                ref = O.bcast(srcs, root, copy_root, [a.copy() for a in init])
                got = plansim.simulate(_lib.plan_bcast(root, copy_root), 5, 13, srcs,
                                       dsts=[a.copy() for a in init])
                for p in range(P):
                    assert np.array_equal(got[p], ref[p]), (P, nbytes, dtype, root, p)


def test_bcast_plan_flags_and_errors():
    P = 4
    for me in range(P):
        pl = S.plan(_lib.plan_bcast(2, False), P, me, 10, 1)
        assert pl["rounds"]
    with pytest.raises(_lib.SosError):
        S.plan(_lib.plan_bcast(4, True), P, 0, 10, 1)   # root outside the team
    with pytest.raises(_lib.SosError):
        S.plan(_lib.PLAN_INSCAN, 65, 0, 10, 4)           # more than 64 PEs


def _wire(alg, P, n, ts):
    sent = [0] * P
    for me in range(P):
        for r in S.plan(alg, P, me, n, ts)["rounds"]:
            for x in r["xfers"]:
                if x["send"]:
                    sent[me] += x["bytes"]
    return sent


def test_bcast_split_wire_bytes():
    # large payloads: the root sends the payload once (scattered), each non-root
    # forwards its chunk to the P-2 other non-roots -> ~ (P-1) * bytes in total,
    # no link carries more than ~ bytes / (P-1) per round
    P, nbytes = 8, 1 << 20
    sent = _wire(_lib.plan_bcast(3, True), P, nbytes, 1)
    assert sent[3] == nbytes
    for p in range(P):
        if p != 3:
            assert abs(sent[p] - nbytes * (P - 2) / (P - 1)) <= 64 * (P - 2)
    # small payloads: direct root -> all
    sent = _wire(_lib.plan_bcast(0, True), P, 1000, 1)
    assert sent[0] == 1000 * (P - 1) and sum(sent) == 1000 * (P - 1)


def test_scan_wire_bytes():
    # gather + all-to-all: every PE sends 2 (P-1)/P of the vector (ragged chunks aside)
    P, n, ts = 8, 8000, 4
    for alg in (_lib.PLAN_INSCAN, _lib.PLAN_EXSCAN):
        sent = _wire(alg, P, n, ts)
        for p in range(P):
            assert sent[p] == 2 * (P - 1) * (n // P) * ts


@pytest.mark.parametrize("P", [9, 12, 16])
def test_ring_plan_beyond_eight_pes(P):
    # teams above 8 PEs run the same direct ring with the runtime-P fold kernel
    dt, op = 23, 5
    for n in (7, 1001):
        srcs = [O.fill(dt, 0, n, p, n) for p in range(P)]
        ref = O.ring(op, dt, srcs)
        got = plansim.simulate("ring", op, dt, srcs)
        for p in range(P):
            assert np.array_equal(bits(got[p]), bits(ref[p])), (P, n, p)
