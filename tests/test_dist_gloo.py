"""CPU, multi-process: the per-PE plans exchanged between real processes.

world_size 2, 3 and 4 with torch.distributed (gloo, 127.0.0.1): each rank runs ITS
OWN plan (from libsos_amd.so's plan builder) with isend/irecv per round (posted as one
group, like ncclGroupStart/End) and the oracle's reduce_local for the folds, and must
end with exactly the oracle's SOS ring / recdbl result.  This checks that the plans
of different PEs agree on every transfer (peer, order, size) when each process only
knows its own plan, as on the 8-GPU node.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, alg, dt, op, n, in_place, outq):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from oracle import oracle as O
    from sos_amd import shmem as S
    import plansim

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    src = O.fill(dt, 1 if op == 6 else 0, 1000 + n, rank, n)
    ts = src.itemsize
    plan = S.plan(alg, world, rank, n, ts)
    bufs = {0: bytearray(src.tobytes())}
    bufs[1] = bufs[0] if in_place else bytearray(n * ts)
    bufs[2] = bytearray(max(plan["scratch_bytes"], 1))
    for r in plan["rounds"]:
        reqs, recvs = [], []
        for x in r["xfers"]:
            if x["send"]:
                t = torch.frombuffer(bytearray(bufs[x["buf"]][x["off"]:x["off"] + x["bytes"]]),
                                     dtype=torch.uint8)
                reqs.append(dist.isend(t, x["peer"]))
            else:
                t = torch.empty(x["bytes"], dtype=torch.uint8)
                reqs.append(dist.irecv(t, x["peer"]))
                recvs.append((x, t))
        for q in reqs:
            q.wait()
        for x, t in recvs:
            bufs[x["buf"]][x["off"]:x["off"] + x["bytes"]] = t.numpy().tobytes()
        for l in r["ops"]:
            ob, ooff = l["out"]
            if l["kind"] == plansim.COPY:
                ib, ioff = l["ins"][0]
                bufs[ob][ooff:ooff + l["count"]] = bytes(bufs[ib][ioff:ioff + l["count"]])
                continue
            cnt = l["count"]
            ins = [np.frombuffer(bytes(bufs[b][o:o + cnt * ts]), dtype=src.dtype) for b, o in l["ins"]]
            bufs[ob][ooff:ooff + cnt * ts] = plansim.fold_values(op, dt, ins, l["order"]).tobytes()
    outq.put((rank, bytes(bufs[1])))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,alg,dt,op,n,in_place", [
    (2, "ring", 23, 5, 1000, False),
    (3, "ring", 11, 2, 777, True),
    (4, "ring", 27, 6, 513, False),
    (3, "recdbl", 23, 4, 200, False),
    (3, "recdbl_gather", 23, 4, 200, False),
    (4, "recdbl_gather", 24, 6, 333, True),
    (2, "rechalving", 24, 5, 1001, False),
    (3, "rechalving", 11, 5, 99, True),
    (4, "recdbl_direct", 10, 6, 640, False),
])
def test_plans_across_processes(world, alg, dt, op, n, in_place):
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, alg, dt, op, n, in_place, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    srcs = [O.fill(dt, 1 if op == 6 else 0, 1000 + n, r, n) for r in range(world)]
    ref = O.ring(op, dt, srcs) if alg == "ring" else O.recdbl(op, dt, srcs)
    for r in range(world):
        want = ref[r] if alg in ("ring", "recdbl", "recdbl_gather") else ref[0]
        assert got[r] == want.tobytes(), (alg, world, r)
