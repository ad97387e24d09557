"""CPU: the multi-process PEs of the oracle -- oracle_pe_ring (bench.py's N > 1 CPU
baseline) and oracle_pe_recdbl (the small-message latency comparison).

P real processes, one per PE, run SOS's ring (src/collectives.c:647-764) or recdbl_sw
(:850-984) over one shared segment (memcpy puts + atomic pSync adds / flag stores, as
XPMEM).  Every PE's target must equal the single-process simulation (oracle_ring /
oracle_recdbl) bit for bit: same chunk math, same in/inout roles, same per-PE tree.
Repeated calls through the timing entry (barrier per call) must leave the same
result, and the pSync words back at SHMEM_SYNC_VALUE (0).
"""
import multiprocessing as mp
import os

import numpy as np
import pytest

from oracle import oracle as O

FLOAT, DOUBLE, INT64, INT = 23, 24, 11, 4
SUM, PROD, BXOR, MAX = 5, 6, 2, 4


def _pe(path, P, me, count, dt, op, dist, reps, q, alg):
    try:
        ring = O.PeRing(path, P, me, count, dt, create=False, alg=alg)
        src = O.fill(dt, dist, 0x5EED, me, count)
        ring.barrier()  # every PE mapped
        if reps:
            ring.time(op, src, reps)
        else:
            ring.run(op, src)
        ring.barrier()  # every put into this target has landed
        out = ring.target().copy()
        q.put((me, out.tobytes()))
        ring.barrier()  # nobody unmaps before the others read
        ring.close()
    except Exception as e:  # pragma: no cover - reported through the queue
        q.put((me, repr(e)))


@pytest.mark.parametrize("alg", ["ring", "recdbl"])
@pytest.mark.parametrize("P,count,dt,op,dist,reps", [
    (2, 1001, FLOAT, SUM, 0, 0),
    (3, 4097, DOUBLE, PROD, 1, 0),
    (4, 7, INT64, BXOR, 0, 0),
    (5, 65536 + 3, FLOAT, SUM, 0, 3),
    (8, 12345, INT, MAX, 0, 2),
    (3, 2, DOUBLE, SUM, 0, 0),   # fewer elements than PEs: empty chunks
])
def test_pe_matches_simulated_schedule(tmp_path, P, count, dt, op, dist, reps, alg):
    path = f"/dev/shm/sosx_pe_{alg}_test_{os.getpid()}_{P}_{count}"
    owner = O.PeRing(path, P, 0, count, dt, create=True, alg=alg)
    try:
        ctx = mp.get_context("fork")
        q = ctx.Queue()
        procs = [ctx.Process(target=_pe, args=(path, P, me, count, dt, op, dist, reps, q, alg))
                 for me in range(P)]
        for p in procs:
            p.start()
        got = dict(q.get(timeout=120) for _ in range(P))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        srcs = [O.fill(dt, dist, 0x5EED, me, count) for me in range(P)]
        exp = (O.ring if alg == "ring" else O.recdbl)(op, dt, srcs)
        for me in range(P):
            assert isinstance(got[me], bytes), got[me]
            assert got[me] == exp[me].tobytes(), f"PE {me} differs from oracle_{alg}"
        words = np.frombuffer(owner.mm, dtype=np.int64, count=owner.hdr // 8)
        assert not words[8:].any(), "pSync words not restored to 0"
        del words
    finally:
        owner.close()
        os.unlink(path)
