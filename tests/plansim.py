"""CPU simulator of the per-PE reduction plans (test infrastructure).

Executes every PE's plan (decoded from libsos_amd.so's plan builder) with numpy byte
buffers: transfers are matched FIFO per (sender, receiver) pair as RCCL matches
ncclSend/ncclRecv, folds are evaluated with the oracle's reduce_local in the plan's
order.  The result must equal the oracle's restatement of the SOS schedule.
"""
import numpy as np

from oracle import oracle as O
from sos_amd import shmem as S

SRC, DST, SCR = 0, 1, 2
FOLD, COPY, PREFIX, ZERO = 0, 1, 2, 3
LINEAR, TREE = 0, 1


def fold_values(op, dt, ins, order):
    """Fold the input arrays in the plan's order with the oracle's reduce_local."""
    if order == LINEAR:
        acc = ins[0].copy()
        for x in ins[1:]:
            O.reduce_local(op, dt, x, acc)
        return acc
    P = len(ins)
    w = [x.copy() for x in ins]
    p2 = 1
    while p2 * 2 <= P:
        p2 *= 2
    for k in range(P - p2):
        O.reduce_local(op, dt, w[k + p2], w[k])
    d = 1
    while d < p2:
        for k in range(0, p2, 2 * d):
            O.reduce_local(op, dt, w[k + d], w[k])
        d *= 2
    return w[0]


def simulate(alg, op, dt, srcs, in_place=False, dsts=None, mis=(0, 0)):
    """Run all PEs' plans; returns the list of per-PE target arrays.

    `dsts` gives the targets' initial contents (default zeros); `mis` the (src, dst)
    addresses mod 16 the plans are built for."""
    P = len(srcs)
    n = srcs[0].size
    ts = srcs[0].itemsize
    np_t = srcs[0].dtype
    plans = [S.plan(alg, P, p, n, ts, mis[0], mis[1]) for p in range(P)]
    bufs = []
    for p in range(P):
        src = bytearray(srcs[p].tobytes())
        if in_place:
            dst = src
        elif dsts is not None:
            dst = bytearray(dsts[p].tobytes())
        else:
            dst = bytearray(n * ts)
        bufs.append({SRC: src, DST: dst, SCR: bytearray(max(plans[p]["scratch_bytes"], 1))})
    fifo = {}
    k = [0] * P
    posted = [False] * P
    outstanding = [0] * P
    done_recv = [None] * P
    while True:
        progress = False
        all_done = True
        for p in range(P):
            if k[p] >= len(plans[p]["rounds"]):
                continue
            all_done = False
            r = plans[p]["rounds"][k[p]]
            if not posted[p]:
                for x in r["xfers"]:
                    if x["send"]:
                        data = bytes(bufs[p][x["buf"]][x["off"]:x["off"] + x["bytes"]])
                        fifo.setdefault((p, x["peer"]), []).append((data, p))
                        outstanding[p] += 1
                done_recv[p] = [False] * len(r["xfers"])
                posted[p] = True
                progress = True
            ok = True
            for i, x in enumerate(r["xfers"]):
                if x["send"] or done_recv[p][i]:
                    continue
                if any(not r["xfers"][j]["send"] and r["xfers"][j]["peer"] == x["peer"]
                       and not done_recv[p][j] for j in range(i)):
                    ok = False
                    continue
                q = fifo.get((x["peer"], p), [])
                if not q:
                    ok = False
                    continue
                data, frm = q.pop(0)
                assert len(data) == x["bytes"], "plan size mismatch between PEs"
                bufs[p][x["buf"]][x["off"]:x["off"] + x["bytes"]] = data
                outstanding[frm] -= 1
                done_recv[p][i] = True
                progress = True
            if ok and outstanding[p] == 0:
                for l in r["ops"]:
                    ob, ooff = l["out"]
                    if l["kind"] == COPY:
                        ib, ioff = l["ins"][0]
                        bufs[p][ob][ooff:ooff + l["count"]] = bytes(bufs[p][ib][ioff:ioff + l["count"]])
                        continue
                    if l["kind"] == ZERO:
                        bufs[p][ob][ooff:ooff + l["count"]] = bytes(l["count"])
                        continue
                    cnt = l["count"]
                    ins = [np.frombuffer(bytes(bufs[p][b][o:o + cnt * ts]), dtype=np_t)
                           for b, o in l["ins"]]
                    if l["kind"] == PREFIX:
                        # all inputs are read before any output is written (kernel contract)
                        acc = ins[0].copy()
                        outs = [acc.copy()]
                        for x in ins[1:]:
                            O.reduce_local(op, dt, x, acc)
                            outs.append(acc.copy())
                        for (b, o), v in zip(l["outs"], outs):
                            bufs[p][b][o:o + cnt * ts] = v.tobytes()
                        continue
                    res = fold_values(op, dt, ins, l["order"])
                    bufs[p][ob][ooff:ooff + cnt * ts] = res.tobytes()
                k[p] += 1
                posted[p] = False
                progress = True
        if all_done:
            break
        assert progress, "plans deadlock"
    return [np.frombuffer(bytes(bufs[p][DST]), dtype=np_t).copy() for p in range(P)]
