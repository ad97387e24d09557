"""TEST INFRASTRUCTURE: replay tests/golden/reductions.json on the GPU with no oracle in
the loop.  Shared by tests/test_golden.py (-m gpu) and __graft_entry__.smoke().

Inputs come from the device generator (sosx_fill), combine cases run sosx_combine
(shmem_internal_reduce_local, src/shmem_internal_op.h:305-339), ring / recdbl cases run
the per-PE plans on the single-GPU loopback team (the RCCL executor's plans and kernels;
src/collectives.c:647-764 ring, :850-984 recdbl_sw).  Every input and output is compared
by SHA-256 with the stored answer.

Also the BASELINE config #1 known answer: examples/pi_reduce.c's "Pi from ..." lines
(SURVEY 8(c)), with the per-PE counts from the host glibc rand() seeded 1 + pe and the
long long sums through the GPU loopback recdbl_sw (SOS AUTO below the crossover).
"""
import ctypes
import hashlib
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "reductions.json")
ESZ = {4: 4, 6: 8, 11: 8, 23: 4, 24: 8, 27: 16}

GOLDEN_PI = {1: "Pi from 10000 points on 1 PEs: 3.171200",
             2: "Pi from 20000 points on 2 PEs: 3.164400",
             4: "Pi from 40000 points on 4 PEs: 3.154100",
             8: "Pi from 80000 points on 8 PEs: 3.150200"}


def load():
    with open(GOLDEN) as f:
        return json.load(f)


def sha(b):
    return hashlib.sha256(b).hexdigest()


def run_cases(torch, sos, cases, seed):
    """Replay `cases` on cuda; returns the list of (what, kind, type, op, n, P) that differ."""
    from sos_amd import shmem as S
    bad = []
    for c in cases:
        dt, op, n, P = c["type"], c["op"], c["n"], c["P"]
        es = ESZ[dt]
        dist = 1 if op == 6 else 0
        npe = 2 if c["kind"] == "combine" else P
        src = []
        for pe in range(npe):
            t = torch.empty(n * es, dtype=torch.uint8, device="cuda")
            sos.fill(dt, dist, seed, pe, t.data_ptr(), n)
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
        if [sha(t.cpu().numpy().tobytes()) for t in outs] != c["out_sha256"]:
            bad.append(("outputs", c["kind"], dt, op, n, P))
    return bad


def pi_counts(me, npoints=10000):
    """examples/pi_reduce.c's per-PE loop: srand(1 + me), npoints pairs of rand()."""
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


def pi_lines_gpu(torch, P):
    """Every PE's pi_reduce line with the two shmem_longlong_sum_reduce calls (n = 1, in
    place) run as the GPU loopback recdbl_sw over P PEs."""
    import numpy as np
    from sos_amd import shmem as S
    counts = [pi_counts(me) for me in range(P)]
    vals = []
    for which in range(2):
        bufs = [torch.from_numpy(np.array([c[which]], dtype=np.int64)).cuda() for c in counts]
        outs = [torch.zeros_like(t) for t in bufs]
        # sum over SHM_INTERNAL_LONG_LONG (shmem_longlong_sum_reduce)
        S.loopback_allreduce("recdbl", 5, 6, [t.data_ptr() for t in bufs],
                             [t.data_ptr() for t in outs], 1)
        torch.cuda.synchronize()
        vals.append([int(t.cpu()[0]) for t in outs])
    inside, total = vals
    return ["Pi from %d points on %d PEs: %f" % (total[p], P, 4.0 * inside[p] / total[p])
            for p in range(P)]
