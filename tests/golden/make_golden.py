"""Generate tests/golden/reductions.json: known-answer vectors of the SOS reduction path.

TEST INFRASTRUCTURE.  The values come from the CPU oracle (oracle/sos_oracle.c), the
restatement of shmem_internal_reduce_local (src/shmem_internal_op.h:305-339), the ring
schedule (src/collectives.c:647-764) and recdbl_sw (:850-984), which is itself pinned by
the reference's examples/pi_reduce.c known answers (tests/test_oracle_kat.py).  The
fixture freezes those answers, so that (a) an oracle change that moves any result fails
tests/test_golden.py on CPU, and (b) the GPU path is checked against stored answers with
no oracle in the loop (tests/test_golden.py, -m gpu).

Cases follow SURVEY.md 8(c): the (type, op) pairs of BASELINE configs #2-#5,
nreduce in {1, 7, 4097, 65536}, P in {1, 2, 3, 4, 8}; kinds:
  combine : inout = fill(pe 0) OP fill(pe 1)           (reduce_local)
  ring    : every PE's target after the SOS ring       (P simulated PEs)
  recdbl  : every PE's target after SOS recdbl_sw
Inputs are the 8(d) synthetic streams fill(type, dist, seed, pe, n) (splitmix64 of the
element index; dist 1 for prod).  Per case: SHA-256 of every input and output, and the
full hex bytes when n <= 7.

Usage: python tests/golden/make_golden.py   (rewrites reductions.json next to it)
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

SEED = 0x5EED
PAIRS = [  # (config, datatype id, op id) -- ids are SOS's enums (src/transport.h, transport_none.h)
    ("#2", 24, 5),                                   # double sum
    ("#3", 11, 0), ("#3", 11, 1), ("#3", 11, 2),     # int64 and / or / xor
    ("#4", 23, 5),                                   # float sum
    ("#5", 4, 3), ("#5", 4, 4), ("#5", 4, 6),        # int min / max / prod
    ("#5", 24, 3), ("#5", 24, 4), ("#5", 24, 6),     # double min / max / prod
    ("#5", 27, 6), ("#5", 27, 5),                    # complexd prod / sum
]
SIZES = [1, 7, 4097, 65536]
PES = [1, 2, 3, 4, 8]


def digest(a):
    return hashlib.sha256(a.tobytes()).hexdigest()


def inputs(dt, op, n, P):
    dist = 1 if op == 6 else 0
    return [O.fill(dt, dist, SEED, pe, n) for pe in range(P)]


def compute(kind, dt, op, n, P):
    """(inputs, outputs) of one case, both lists of arrays."""
    if kind == "combine":
        ins = inputs(dt, op, n, 2)
        out = ins[0].copy()
        O.reduce_local(op, dt, ins[1], out)
        return ins, [out]
    ins = inputs(dt, op, n, P)
    outs = (O.ring if kind == "ring" else O.recdbl)(op, dt, ins)
    return ins, outs


def cases():
    for cfg, dt, op in PAIRS:
        for n in SIZES:
            yield {"config": cfg, "type": dt, "op": op, "n": n, "P": 2, "kind": "combine"}
            for P in PES:
                for kind in ("ring", "recdbl"):
                    yield {"config": cfg, "type": dt, "op": op, "n": n, "P": P, "kind": kind}


def record(c):
    ins, outs = compute(c["kind"], c["type"], c["op"], c["n"], c["P"])
    r = dict(c)
    r["in_sha256"] = [digest(a) for a in ins]
    r["out_sha256"] = [digest(a) for a in outs]
    if c["n"] <= 7:
        r["in_hex"] = [a.tobytes().hex() for a in ins]
        r["out_hex"] = [a.tobytes().hex() for a in outs]
    return r


def main():
    doc = {"what": "SOS reduction known answers (see make_golden.py)", "seed": SEED,
           "dist": "fill(type, 1 if op == prod else 0, seed, pe, n)",
           "cases": [record(c) for c in cases()]}
    with open(os.path.join(HERE, "reductions.json"), "w") as f:
        json.dump(doc, f, indent=0, sort_keys=True)
        f.write("\n")
    print(f"{len(doc['cases'])} cases")


if __name__ == "__main__":
    main()
