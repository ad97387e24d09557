"""CPU: pin the oracle (oracle/sos_oracle.c).

1. Known answers of SURVEY.md 8(c): SOS's examples/pi_reduce.c output for 1/2/4/8 PEs
   (glibc rand() seeded 1+pe, long long sums through shmem_sum_reduce).  Computed here
   with the host glibc's rand() and the oracle's ring and recdbl schedules.
2. An independent numpy restatement of reduce_local's element semantics (ternary
   min/max, wrapping integer arithmetic, SOS's signed mapping of uint8..64) agrees
   with the compiled oracle bit for bit.
3. The synthetic-input generator is deterministic and shaped as SURVEY.md 8(d) says.
"""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN_PI = {1: "Pi from 10000 points on 1 PEs: 3.171200",
             2: "Pi from 20000 points on 2 PEs: 3.164400",
             4: "Pi from 40000 points on 4 PEs: 3.154100",
             8: "Pi from 80000 points on 8 PEs: 3.150200"}


def pi_counts(me, npoints=10000):
    libc = ctypes.CDLL("libc.so.6")
    libc.rand.restype = ctypes.c_int
    libc.srand(1 + me)
    rand_max = 2147483647
    inside = 0
    for _ in range(npoints):
        x = libc.rand() / float(rand_max)
        y = libc.rand() / float(rand_max)
        if x * x + y * y < 1:
            inside += 1
    return inside, npoints


@pytest.mark.parametrize("P", [1, 2, 4, 8])
@pytest.mark.parametrize("sched", ["ring", "recdbl"])
def test_pi_reduce_known_answers(P, sched):
    counts = [pi_counts(me) for me in range(P)]
    inside = [np.array([c[0]], dtype=np.int64) for c in counts]
    total = [np.array([c[1]], dtype=np.int64) for c in counts]
    fn = O.ring if sched == "ring" else O.recdbl
    # in place, as the example does (shmem_sum_reduce(team, &x, &x, 1))
    fn(5, 6, inside, inside)
    fn(5, 6, total, total)
    for p in range(P):
        line = "Pi from %d points on %d PEs: %f" % (total[p][0], P, 4.0 * inside[p][0] / total[p][0])
        assert line == GOLDEN_PI[P]


def np_reduce_local(op, dt, inp, inout):
    """Independent restatement of src/shmem_internal_op.h:37-43 in numpy."""
    a, b = inout, inp
    if op == 0:
        return a & b
    if op == 1:
        return a | b
    if op == 2:
        return a ^ b
    if op == 3:
        return np.where(a < b, a, b)   # (a) < (b) ? (a) : (b)
    if op == 4:
        return np.where(a > b, a, b)
    with np.errstate(over="ignore", invalid="ignore"):
        if op == 5:
            return (a + b).astype(a.dtype)
        return (a * b).astype(a.dtype)


@pytest.mark.parametrize("dt", [1, 2, 3, 4, 5, 8, 9, 10, 11, 13, 14, 15, 16, 18, 19, 20, 21, 22, 23, 24])
def test_oracle_matches_numpy_restatement(dt):
    ops = [3, 4, 5, 6] if dt in (1, 2, 23, 24) else list(range(7))
    for op in ops:
        n = 4099
        a = O.fill(dt, 1 if op == 6 else 0, 1234 + op, 0, n)
        b = O.fill(dt, 1 if op == 6 else 0, 1234 + op, 1, n)
        ref = a.copy()
        O.reduce_local(op, dt, b, ref)
        mine = np_reduce_local(op, dt, b, a.copy())
        assert np.array_equal(ref.view(np.uint8), mine.view(np.uint8)), (dt, op)


def test_uint_maps_to_signed_compare_only_via_bindings():
    """reduce_local itself compares UINT32 unsigned; SOS's binding passes INT32 for
    uint32_t, so shmem_uint32_max_reduce compares signed."""
    a = np.array([0x80000000], dtype=np.uint32)
    b = np.array([1], dtype=np.uint32)
    r_unsigned = a.copy()
    O.reduce_local(4, 20, b, r_unsigned)                  # UINT32: 0x80000000
    r_signed = a.copy()
    O.reduce_local(4, 10, b.view(np.int32), r_signed.view(np.int32))  # INT32 (binding): 1
    assert r_unsigned[0] == 0x80000000 and r_signed[0] == 1


def test_fill_shapes():
    f = O.fill(23, 0, 1, 0, 100000)
    assert f.dtype == np.float32 and f.min() >= -1 and f.max() < 1
    p = O.fill(24, 1, 1, 0, 100000)
    assert p.min() >= 0.5 and p.max() < 2
    c = O.fill(27, 1, 1, 0, 1000).view(np.float64)
    assert np.all((np.abs(c) >= 0.5) & (np.abs(c) < 1))
    i = O.fill(4, 1, 1, 0, 1000)
    assert i.min() >= -3 and i.max() <= 3
    assert np.array_equal(O.fill(11, 0, 9, 3, 50, 10), O.fill(11, 0, 9, 3, 60)[10:])


def test_ring_vs_recdbl_fp_tolerance():
    """SOS ring and recdbl disagree in the last bits for fp sums; within (P-1) eps sum|x|."""
    P, n = 8, 100000
    srcs = [O.fill(23, 0, 42, p, n) for p in range(P)]
    r = O.ring(5, 23, srcs)[0].astype(np.float64)
    d = O.recdbl(5, 23, srcs)[0].astype(np.float64)
    bound = (P - 1) * np.finfo(np.float32).eps * np.sum(np.abs(np.stack(srcs).astype(np.float64)), 0)
    assert np.all(np.abs(r - d) <= bound)
    assert np.count_nonzero(r != d) > 0
