"""CPU: the schedules' index arithmetic pinned to the reference's source TEXT (VERDICT r5
item 5).

test_reference_text.py pins the op macros, enums and type tables; this file pins the
ring's chunk/displacement expressions (src/collectives.c:693-756) and recdbl_sw's
pow2/log2 loop, extra-peer and pairwise-peer expressions (:850-977).  The expressions are
extracted from the C text with regular expressions, translated to Python by a small
C-expression translator and evaluated over P = 1..12 and nreduce in {0, 1, 7, 4097}.  A
symbolic run of each schedule over those tables (lists of PE ids instead of values) gives
every chunk's extent, every chunk's fold order and every PE's pairing sequence.  The same
is done with oracle/sos_oracle.c's restatement (ring_chunk and the loops of oracle_ring /
oracle_recdbl, also parsed from text) and with the product's plans (libsos_amd.so's plan
builder, decoded by sos_amd.shmem.plan): all three must agree.  Nothing of the reference
is compiled or executed.

Skipped where /root/reference is absent (the GPU box)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_C = "/root/reference/src/collectives.c"
ORACLE = os.path.join(ROOT, "oracle", "sos_oracle.c")

pytestmark = pytest.mark.skipif(not os.path.exists(REF_C), reason="reference checkout not present")

PS = range(1, 13)
NS = (0, 1, 7, 4097)
TS = 4


def _strip_comments(t):
    return re.sub(r"/\*.*?\*/", "", t, flags=re.S)


def _function(text, name, end_marker):
    a = text.index(name + "(")
    return text[a:text.index(end_marker, a + len(name))]


def _split_top(expr, ch):
    """Index of the first `ch` at parenthesis depth 0, or -1."""
    d = 0
    for k, c in enumerate(expr):
        if c == "(":
            d += 1
        elif c == ")":
            d -= 1
        elif c == ch and d == 0:
            return k
    return -1


def c_to_py(expr):
    """A C integer expression of these schedules as Python: casts dropped, `/` as floor
    division (every operand is non-negative), `a ? b : c` as a conditional, `x++` not
    allowed (statements are translated by the callers)."""
    e = " ".join(expr.split())
    e = re.sub(r"\((?:size_t|int|long|unsigned)\)\s*", "", e)
    q = _split_top(e, "?")
    if q >= 0:
        rest = e[q + 1:]
        c = _split_top(rest, ":")
        assert c >= 0, expr
        return f"(({c_to_py(rest[:c])}) if ({c_to_py(e[:q])}) else ({c_to_py(rest[c + 1:])}))"
    # a parenthesised sub-expression may hold a ternary of its own
    out, k = "", 0
    while k < len(e):
        if e[k] == "(":
            d, j = 0, k
            while True:
                d += e[j] == "("
                d -= e[j] == ")"
                if d == 0:
                    break
                j += 1
            out += "(" + c_to_py(e[k + 1:j]) + ")"
            k = j + 1
        else:
            out += e[k]
            k += 1
    return out.replace("/", "//")


def ev(expr, **env):
    return int(eval(c_to_py(expr), {"__builtins__": {}}, env))


def assigns(text, names):
    """{name: C expression} of `size_t name = expr;` for each name (first occurrence)."""
    out = {}
    for nm in names:
        m = re.search(r"size_t\s+" + nm + r"\s*=\s*(.*?);", text, re.S)
        assert m, nm
        out[nm] = m.group(1)
    return out


# ------------------------------------------------------------------------------------
# the ring, src/collectives.c:647-764
# ------------------------------------------------------------------------------------
def ref_ring_text():
    body = _strip_comments(_function(open(REF_C).read(), "shmem_internal_op_to_all_ring",
                                     "shmem_internal_op_to_all_tree"))
    loops = [m.start() for m in re.finditer(r"for \(int i = 0; i < PE_size - 1; i\+\+\)", body)]
    assert len(loops) == 2, "the ring has a reduce-scatter and an allgather loop"
    rs, ag = body[loops[0]:loops[1]], body[loops[1]:]
    peer = re.search(r"int peer = (.*?);", body).group(1)
    # the step-0 put sends from source, later ones from target; reduce_local(in = source,
    # inout = target): the received value is the left operand
    assert re.search(r"i == 0 \?\s*\(\(uint8_t \*\) source\) \+ chunk_out_disp :", rs), "put source"
    assert re.search(r"shmem_internal_reduce_local\(op, datatype, chunk_in_count,\s*\(\(uint8_t \*\) source\) "
                     r"\+ chunk_in_disp,\s*\(\(uint8_t \*\) target\) \+ chunk_in_disp\)", rs), "combine"
    assert re.search(r"if \(count == 0\) return;", body) and re.search(r"if \(PE_size == 1\)", body)
    rs_x = assigns(rs, ["chunk_in", "chunk_out", "chunk_in_extra", "chunk_out_extra", "chunk_in_count",
                        "chunk_out_count", "chunk_out_disp", "chunk_in_disp"])
    ag_x = assigns(ag, ["chunk_out", "chunk_out_extra", "chunk_out_count", "chunk_out_disp"])
    return peer, rs_x, ag_x


def ref_ring_step(rs_x, r, i, P, n):
    env = dict(group_rank=r, i=i, PE_size=P, count=n, type_size=TS)
    v = {}
    for nm in ("chunk_in", "chunk_out", "chunk_in_extra", "chunk_out_extra", "chunk_in_count",
               "chunk_out_count", "chunk_out_disp", "chunk_in_disp"):
        v[nm] = ev(rs_x[nm], **env, **v)
    return v


def ref_ring_ag(ag_x, r, i, P, n):
    env = dict(group_rank=r, i=i, PE_size=P, count=n, type_size=TS)
    v = {}
    for nm in ("chunk_out", "chunk_out_extra", "chunk_out_count", "chunk_out_disp"):
        v[nm] = ev(ag_x[nm], **env, **v)
    return v


def run_ring(P, n, peer_of, step, ag_step):
    """Symbolic ring: every PE's target chunks as the list of PEs folded into them, in
    order; extents {chunk: (byte offset, bytes)}.  P == 1 or n == 0: nothing moves."""
    if P == 1 or n == 0:
        return None, {}
    tgt = [[None] * P for _ in range(P)]
    ext = {}

    def note(c, disp, cnt):
        assert ext.setdefault(c, (disp, cnt * TS)) == (disp, cnt * TS), (P, n, c)

    for i in range(P - 1):
        puts = []
        for r in range(P):
            v = step(r, i, P, n)
            note(v["chunk_out"], v["chunk_out_disp"], v["chunk_out_count"])
            note(v["chunk_in"], v["chunk_in_disp"], v["chunk_in_count"])
            puts.append((peer_of(r, P), v["chunk_out"], [r] if i == 0 else tgt[r][v["chunk_out"]]))
        for p, c, payload in puts:
            tgt[p][c] = list(payload)
        for r in range(P):
            c = step(r, i, P, n)["chunk_in"]
            tgt[r][c] = tgt[r][c] + [r]          # target = target OP source
    for i in range(P - 1):
        puts = []
        for r in range(P):
            v = ag_step(r, i, P, n)
            note(v["chunk_out"], v["chunk_out_disp"], v["chunk_out_count"])
            puts.append((peer_of(r, P), v["chunk_out"], tgt[r][v["chunk_out"]]))
        for p, c, payload in puts:
            tgt[p][c] = list(payload)
    return tgt, ext


def ref_ring(P, n):
    peer, rs_x, ag_x = ref_ring_text()
    return run_ring(P, n, lambda r, P_: ev(peer, PE_start=0, group_rank=r, PE_size=P_, PE_stride=1),
                    lambda r, i, P_, n_: ref_ring_step(rs_x, r, i, P_, n_),
                    lambda r, i, P_, n_: ref_ring_ag(ag_x, r, i, P_, n_))


def oracle_ring_text():
    t = _strip_comments(open(ORACLE).read())
    rc = _function(t, "static void ring_chunk", "int oracle_ring")
    extra = re.search(r"size_t extra = (.*?);", rc).group(1)
    cnt = re.search(r"size_t cnt = (.*?);", rc).group(1)
    disp = re.search(r"\*disp = (.*?);", rc).group(1)
    body = _function(t, "int oracle_ring", "int oracle_recdbl")
    outs = re.findall(r"size_t chunk_out = (.*?), n, disp;", body)
    cin = re.search(r"size_t chunk_in = (.*?), n, disp;", body).group(1)
    peer = re.search(r"int peer = (.*?);", body).group(1)
    assert len(outs) == 2
    assert "i == 0 ? (uint8_t *) s[r] + disp : (uint8_t *) dst[r] + disp" in body
    assert re.search(r"oracle_reduce_local\(op, dt, \(int\) n, \(uint8_t \*\) s\[r\] \+ disp,\s*"
                     r"\(uint8_t \*\) dst\[r\] \+ disp\)", body)

    def chunk(c, P, n):
        x = ev(extra, c=c, count=n, P=P)
        k = ev(cnt, count=n, P=P, extra=x)
        return k, ev(disp, extra=x, c=c, cnt=k, ts=TS, count=n, P=P)

    def step(r, i, P, n):
        co, ci = ev(outs[0], r=r, i=i, P=P), ev(cin, r=r, i=i, P=P)
        (ko, do), (ki, di) = chunk(co, P, n), chunk(ci, P, n)
        return {"chunk_out": co, "chunk_out_count": ko, "chunk_out_disp": do,
                "chunk_in": ci, "chunk_in_count": ki, "chunk_in_disp": di}

    def ag(r, i, P, n):
        co = ev(outs[1], r=r, i=i, P=P)
        k, d = chunk(co, P, n)
        return {"chunk_out": co, "chunk_out_count": k, "chunk_out_disp": d}

    return lambda r, P: ev(peer, r=r, P=P), step, ag


def test_ring_text_tables_parse():
    peer, rs_x, ag_x = ref_ring_text()
    assert ev(peer, PE_start=0, group_rank=2, PE_size=3, PE_stride=1) == 0
    v = ref_ring_step(rs_x, 0, 0, 4, 7)
    assert (v["chunk_out"], v["chunk_in"]) == (0, 3)


@pytest.mark.parametrize("P", PS)
def test_oracle_ring_tables_equal_reference_text(P):
    peer, step, ag = oracle_ring_text()
    for n in NS:
        want = ref_ring(P, n)
        got = run_ring(P, n, peer, step, ag)
        assert got == want, (P, n)
        if want[0] is not None:
            tgt, ext = want
            # every PE ends with every chunk, chunk c folded from PE c onward, in ring order
            for r in range(P):
                for c in range(P):
                    assert tgt[r][c] == [(c + k) % P for k in range(P)], (P, n, r, c)
            # the chunks tile [0, n * ts)
            spans = sorted(ext.values())
            assert spans[0][0] == 0 and sum(b for _, b in spans) == n * TS
            for (o1, b1), (o2, _) in zip(spans, spans[1:]):
                assert o1 + b1 == o2


def _plan(alg, P, me, n):
    from sos_amd import shmem as S
    return S.plan(alg, P, me, n, TS)


SRC, DST, SCR = 0, 1, 2


@pytest.mark.parametrize("P", PS)
def test_product_ring_plan_equals_reference_text(P):
    """The product's ring plans (a direct exchange: PE c folds chunk c) move exactly the
    reference's chunks, and fold chunk c from PE c onward in the reference's order."""
    for n in NS:
        want = ref_ring(P, n)
        for me in range(P):
            plan = _plan("ring", P, me, n)
            if want[0] is None:
                assert not any(r["xfers"] for r in plan["rounds"]), (P, n, me)
                continue
            tgt, ext = want
            chunks = {(o, b) for o, b in ext.values() if b}
            moved = {(x["off"], x["bytes"]) for r in plan["rounds"] for x in r["xfers"]
                     if x["buf"] in (SRC, DST)}
            assert moved <= chunks, (P, n, me, moved - chunks)
            # the fold of chunk me: its inputs in order, each mapped to the PE it came from
            recv = {(x["buf"], x["off"]): x["peer"] for r in plan["rounds"] for x in r["xfers"]
                    if not x["send"]}
            folds = [o for r in plan["rounds"] for o in r["ops"] if o["kind"] == 0]
            off, nbytes = ext[me]
            if nbytes == 0:
                continue
            assert len(folds) == 1, (P, n, me)
            order = [me if b == SRC else recv[(b, o)] for b, o in folds[0]["ins"]]
            assert order == tgt[(me + P - 1) % P][me], (P, n, me, order)
            assert folds[0]["count"] * TS == nbytes


# ------------------------------------------------------------------------------------
# recdbl_sw, src/collectives.c:850-977
# ------------------------------------------------------------------------------------
def _exec_c_loop(init, cond, body, env):
    """Run `init; while (cond) { body }` with statements `x >>= k;` `x <<= k;` `x++;`."""
    for name, val in init:
        env[name] = ev(val, **env)
    guard = 0
    while ev(cond, **env):
        for st in [s.strip() for s in body.split(";") if s.strip()]:
            m = re.fullmatch(r"(\w+)\s*(>>=|<<=|\+=|-=)\s*(.+)", st)
            if m:
                v = ev(m.group(3), **env)
                env[m.group(1)] = {">>=": env[m.group(1)] >> v, "<<=": env[m.group(1)] << v,
                                   "+=": env[m.group(1)] + v, "-=": env[m.group(1)] - v}[m.group(2)]
            else:
                m = re.fullmatch(r"(\w+)\+\+", st)
                assert m, st
                env[m.group(1)] += 1
        guard += 1
        assert guard < 64
    return env


def _decls(decl):
    """`int a = 1, b = 2` -> [('a', '1'), ('b', '2')]."""
    return [tuple(p.split("=", 1)[0].split()[-1:] + [p.split("=", 1)[1].strip()])
            for p in decl.split(",")]


def ref_recdbl(P):
    body = _strip_comments(_function(open(REF_C).read(), "shmem_internal_op_to_all_recdbl_sw",
                                     "SCAN"))
    d1 = re.search(r"int (log2_proc = .*?);", body).group(1)
    d2 = re.search(r"int (i = PE_size >> 1);", body).group(1)
    loop = re.search(r"while \((.*?)\) \{(.*?)\}", body, re.S)
    env = _exec_c_loop(_decls(d1) + _decls(d2), loop.group(1), loop.group(2), {"PE_size": P})
    pow2, log2 = env["pow2_proc"], env["log2_proc"]
    extra_peer = re.search(r"if \(my_id >= pow2_proc\) \{\s*int peer = (.*?);", body).group(1)
    partners = re.findall(r"if \(my_id < PE_size - pow2_proc\) \{\s*int peer = (.*?);", body)
    assert len(partners) == 2 and partners[0] == partners[1]
    pair = re.search(r"for \(i = 0; i < log2_proc; i\+\+\) \{.*?int peer = (.*?);", body, re.S).group(1)
    seq = {}
    for me in range(P):
        e = dict(my_id=me, pow2_proc=pow2, PE_stride=1, PE_start=0, PE_size=P)
        if me >= pow2:
            q = ev(extra_peer, **e)
            seq[me] = [("send", q), ("recv", q)]
            continue
        s = []
        if me < P - pow2:
            s.append(("recv", ev(partners[0], **e)))
        for i in range(log2):
            s.append(("xchg", ev(pair, i=i, **e)))
        if me < P - pow2:
            s.append(("send", ev(partners[1], **e)))
        seq[me] = s
    return pow2, log2, seq


def oracle_recdbl(P):
    t = _strip_comments(open(ORACLE).read())
    body = _function(t, "int oracle_recdbl", "int oracle_scan")
    d = re.search(r"int (pow2 = .*?);", body).group(1)
    loop = re.search(r"while \((.*?)\) \{(.*?)\}", body, re.S)
    env = _exec_c_loop(_decls(d), loop.group(1), loop.group(2), {"P": P})
    pow2, log2 = env["pow2"], env["log2p"]
    partner = re.search(r"for \(int p = pow2; p < P; p\+\+\) \{\s*int partner = (.*?);", body).group(1)
    pair = re.search(r"for \(int s = 0; s < log2p; s\+\+\) \{\s*for \(int r = 0; r < pow2; r\+\+\) "
                     r"memcpy\(dst\[(.*?)\], cur\[r\], bytes\);", body).group(1)
    final = re.search(r"for \(int p = pow2; p < P; p\+\+\) memcpy\(dst\[p\], cur\[(.*?)\], bytes\);",
                      body).group(1)
    seq = {}
    for me in range(P):
        if me >= pow2:
            seq[me] = [("send", ev(partner, p=me, pow2=pow2)), ("recv", ev(final, p=me, pow2=pow2))]
            continue
        s = []
        xs = [p for p in range(pow2, P) if ev(partner, p=p, pow2=pow2) == me]
        s += [("recv", p) for p in xs]
        for k in range(log2):
            s.append(("xchg", ev(pair, r=me, s=k)))
        s += [("send", p) for p in range(pow2, P) if ev(final, p=p, pow2=pow2) == me]
        seq[me] = s
    return pow2, log2, seq


@pytest.mark.parametrize("P", range(2, 13))
def test_oracle_recdbl_pairings_equal_reference_text(P):
    assert oracle_recdbl(P) == ref_recdbl(P)
    pow2, log2, _ = ref_recdbl(P)
    assert pow2 <= P < 2 * pow2 and pow2 == 1 << log2


def _flat(plan):
    out = []
    for r in plan["rounds"]:
        by = {}
        for x in r["xfers"]:
            by.setdefault(x["peer"], set()).add("send" if x["send"] else "recv")
        for p, k in by.items():
            out.append(("xchg" if k == {"send", "recv"} else k.pop(), p))
    return out


@pytest.mark.parametrize("P", range(2, 13))
def test_product_recdbl_plan_pairings_equal_reference_text(P):
    """The product's recdbl_sw plan (SHMEM_REDUCE_ALGORITHM=recdbl) makes the reference's
    transfers with the reference's peers in the reference's order, at every n > 0."""
    _, _, want = ref_recdbl(P)
    for n in NS:
        for me in range(P):
            got = _flat(_plan("recdbl", P, me, n))
            assert got == (want[me] if n else []), (P, n, me, got, want[me])
