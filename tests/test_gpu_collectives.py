"""GPU: the team scans and broadcast, and the runtime-P fold (teams above 8 PEs).

Every result is compared bit for bit with the CPU oracle (oracle/sos_oracle.c):
  sosx_prefix                 == in-order prefix of oracle reduce_local
  loopback inscan / exscan    == oracle_scan   (SOS scan_ring, src/collectives.c:1111-1209)
  loopback broadcast          == oracle_bcast  (src/collectives.c:429-485)
  sosx_fold with 9..64 inputs == the plan simulator's LINEAR / TREE fold
  loopback ring over 12 PEs   == oracle_ring   (src/collectives.c:647-764)
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from sos_amd import _lib, shmem as S

import plansim

pytestmark = pytest.mark.gpu


def to_dev(torch, a, pad=0):
    """Device copy of array a (bytes), optionally `pad` bytes into a larger buffer."""
    raw = np.frombuffer(a.tobytes(), np.uint8)
    t = torch.zeros(raw.size + pad + 16, dtype=torch.uint8, device="cuda")
    t[pad:pad + raw.size].copy_(torch.from_numpy(raw.copy()))
    return t


def from_dev(t, like, pad=0):
    raw = t[pad:pad + like.nbytes].cpu().numpy()
    return np.frombuffer(raw.tobytes(), like.dtype).copy()


def bits(a):
    return np.frombuffer(a.tobytes(), np.uint8)


def src_of(dt, seed, pe, n):
    if dt == 25:
        return np.random.default_rng(seed * 131 + pe).standard_normal(n).astype(np.longdouble)
    return O.fill(dt, 0, seed, pe, n)


def cpu_prefix(op, dt, ins):
    acc = ins[0].copy()
    outs = [acc.copy()]
    for x in ins[1:]:
        O.reduce_local(op, dt, x, acc)
        outs.append(acc.copy())
    return outs


@pytest.mark.parametrize("np_", [1, 2, 3, 8, 9, 12, 64])
@pytest.mark.parametrize("dt", [23, 24, 4, 1, 27, 25])
def test_prefix_kernel(torch_cuda, np_, dt):
    torch = torch_cuda
    for n in (1, 999, (1 << 18) + 5):
        if np_ > 12 and n > 999:
            continue
        ins = [src_of(dt, n, k, n) for k in range(np_)]
        ref = cpu_prefix(5, dt, ins)
        di = [to_dev(torch, a) for a in ins]
        do = [torch.zeros_like(t) for t in di]
        _lib.prefix(5, dt, [t.data_ptr() for t in do], [t.data_ptr() for t in di], n)
        torch.cuda.synchronize()
        for k in range(np_):
            assert np.array_equal(bits(from_dev(do[k], ref[k])), bits(ref[k])), (np_, n, k)


@pytest.mark.parametrize("np_", [1, 2, 3, 8])
@pytest.mark.parametrize("dt", [23, 24, 4, 1, 27])
def test_prefix_realigned_inputs(torch_cuda, np_, dt):
    """SUM prefix whose inputs sit at other 16-B offsets than its (congruent) outputs
    (a scan with source and target at different offsets): input 0 only, every input at
    its own offset (k_prefix_realign_np), every input at one offset (k_prefix_outshift,
    the outputs realigned), ragged sizes; bit for bit against the in-order prefix of the
    oracle's reduce_local."""
    torch = torch_cuda
    es = O.lib().oracle_type_size(dt)
    for n in (999, (1 << 18) + 5):
        ins = [src_of(dt, n + 7, k, n) for k in range(np_)]
        ref = cpu_prefix(5, dt, ins)
        for offs in ([es % 16] + [0] * (np_ - 1), [(es * (k + 1)) % 16 for k in range(np_)],
                     [es % 16] * np_):
            di = [to_dev(torch, a, off) for a, off in zip(ins, offs)]
            do = [torch.zeros_like(to_dev(torch, a)) for a in ins]
            _lib.prefix(5, dt, [t.data_ptr() for t in do], [t.data_ptr() + off for t, off in zip(di, offs)], n)
            torch.cuda.synchronize()
            for k in range(np_):
                assert np.array_equal(bits(from_dev(do[k], ref[k])), bits(ref[k])), (np_, n, offs, k)


@pytest.mark.parametrize("np_", [3, 8, 12])
@pytest.mark.parametrize("op", [5, 4, 6])
def test_prefix_kernel_aliasing(torch_cuda, np_, op):
    """An in-place exscan: output k-1 is input k's buffer.  np <= 8 may alias any input,
    for every op (SUM through the vector kernel, MAX/PROD through the element loop, which
    loads every input of an element before its first store); larger np names the aliased
    input `own` (one per call)."""
    torch = torch_cuda
    dt, n = 24, 4099
    ins = [src_of(dt, 5, k, n) for k in range(np_)]
    ref = cpu_prefix(op, dt, ins)
    j = np_ // 2
    di = [to_dev(torch, a) for a in ins]
    do = [torch.zeros_like(t) for t in di]
    do[j - 1] = di[j]  # output j-1 overwrites input j
    _lib.prefix(op, dt, [t.data_ptr() for t in do], [t.data_ptr() for t in di], n,
                own=j if np_ > 8 else -1)
    torch.cuda.synchronize()
    for k in range(np_):
        assert np.array_equal(bits(from_dev(do[k], ref[k])), bits(ref[k])), (np_, k)


@pytest.mark.parametrize("P", [9, 12, 16, 64])
@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("dt,op", [(23, 5), (11, 2), (27, 6), (4, 4)])
def test_fold_runtime_p(torch_cuda, P, order, dt, op):
    torch = torch_cuda
    n = 1001
    ins = [O.fill(dt, 1 if op == 6 else 0, 3, k, n) for k in range(P)]
    ref = plansim.fold_values(op, dt, ins, order)
    di = [to_dev(torch, a) for a in ins]
    out = torch.zeros_like(di[0])
    _lib.fold(op, dt, order, out.data_ptr(), [t.data_ptr() for t in di], n)
    torch.cuda.synchronize()
    assert np.array_equal(bits(from_dev(out, ref)), bits(ref))


@pytest.mark.parametrize("P", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("dt,op", [(23, 5), (24, 4), (11, 2), (27, 6), (26, 5), (3, 3)])
def test_fold_small_inputs(torch_cuda, P, order, dt, op):
    """Folds of inputs of at most 64 KiB each (k_fold_dyn, the latency-bound path of the
    small team calls): every input's element is loaded before the first combine; the
    operation order is the plan's, bit for bit against the plan simulator's fold, ragged
    sizes and an element-misaligned start."""
    torch = torch_cuda
    es = O.lib().oracle_type_size(dt)
    for n in (1, 7, 1000, (1 << 16) // es):
        ins = [O.fill(dt, 1 if op == 6 else 0, 17, k, n) for k in range(P)]
        ref = plansim.fold_values(op, dt, ins, order)
        for off in (0, es if es < 16 else 0):
            di = [to_dev(torch, a, off) for a in ins]
            out = torch.zeros_like(to_dev(torch, ins[0], off))
            _lib.fold(op, dt, order, out.data_ptr() + off, [t.data_ptr() + off for t in di], n)
            torch.cuda.synchronize()
            got = from_dev(out, ref, off) if off else from_dev(out, ref)
            assert np.array_equal(bits(got), bits(ref)), (n, off)


@pytest.mark.parametrize("P", [2, 3, 5, 6, 7, 8])
@pytest.mark.parametrize("dt,op", [(23, 5), (18, 5), (3, 2), (24, 6), (11, 4), (26, 5)])
@pytest.mark.parametrize("layout", ["own", "peers", "peers_es", "mixed"])
@pytest.mark.parametrize("order", [0, 1])
def test_fold_realigned_inputs(torch_cuda, P, dt, op, layout, order):
    """Folds past 64 KiB per input whose inputs sit at other 16-B offsets than the output
    (k_fold_realign), in the ring's LINEAR order and in recdbl_sw's TREE order (the extras
    first, then the pairwise tree): the PE's own source chunk only ("own", the ring at PE
    me with source and target at different offsets), every input at one offset ("peers"
    at +8, "peers_es" at +element size: the p2p transport's in-place reads of the peers'
    sources: unaligned loads for 4- and 8-byte elements, k_fold_outshift realigning the
    output for the others), or each input at its own offset ("mixed"); ragged sizes; bit
    for bit against the plan simulator's fold."""
    torch = torch_cuda
    es = O.lib().oracle_type_size(dt)
    for n in ((1 << 16) // es + 1, (1 << 20) + 3):
        ins = [O.fill(dt, 1 if op == 6 else 0, 11, k, n) for k in range(P)]
        ref = plansim.fold_values(op, dt, ins, order)
        if layout == "own":
            offs = [es] + [0] * (P - 1)
        elif layout == "peers":
            offs = [8 if es <= 8 else 0] * P
        elif layout == "peers_es":
            offs = [es % 16] * P
        else:
            offs = [(es * k) % 16 for k in range(1, P + 1)]
        di = [to_dev(torch, a, off) for a, off in zip(ins, offs)]
        out = torch.zeros_like(to_dev(torch, ins[0]))
        _lib.fold(op, dt, order, out.data_ptr(), [t.data_ptr() + off for t, off in zip(di, offs)], n)
        torch.cuda.synchronize()
        assert np.array_equal(bits(from_dev(out, ref)), bits(ref)), (n, offs)


@pytest.mark.parametrize("form", ["unaligned", "shifted"])
def test_realign_forms_forced(form):
    """Every form of the realigning fold and prefix, bit for bit.  "unaligned": every layout
    with an incongruent input takes the unaligned-load form (fp32/fp64/int32/int64; by
    default only five or more incongruent inputs, or all at one offset); "shifted": the
    register-realigned forms only (DPP per input, outshift for one-offset layouts).  The
    realigned-input tests above rerun in a child process under each setting."""
    import subprocess
    import sys
    here = os.path.abspath(__file__)
    knobs = {"unaligned": ("1", "0"), "shifted": ("9", "1")}[form]
    env = dict(os.environ, SOSX_REALIGN_UNALIGNED=knobs[0], SOSX_FOLD_OUTSHIFT=knobs[1],
               SOSX_PREFIX_OUTSHIFT=knobs[1])
    r = subprocess.run([sys.executable, "-m", "pytest", here, "-q", "-p", "no:cacheprovider", "-k",
                        "test_fold_realigned_inputs or test_prefix_realigned_inputs"],
                       capture_output=True, text=True, timeout=280, env=env,
                       cwd=os.path.dirname(os.path.dirname(here)))
    assert r.returncode == 0, (r.stdout[-2500:], r.stderr[-1500:])
    assert " passed" in r.stdout and "failed" not in r.stdout


def test_fold_selection_exits_cleanly():
    """The float-sum runtime-P fold selection used to abort at interpreter exit (two HIP
    runtimes in one process); the selection must now exit with status 0."""
    import subprocess
    import sys
    here = os.path.abspath(__file__)
    r = subprocess.run([sys.executable, "-m", "pytest", here, "-q", "-p", "no:cacheprovider",
                        "-k", "test_fold_runtime_p and 23-5"], capture_output=True, text=True,
                       timeout=110, cwd=os.path.dirname(os.path.dirname(here)))
    assert r.returncode == 0, (r.stdout[-1500:], r.stderr[-1500:])
    assert "8 passed" in r.stdout


def loopback(torch, alg, op, dt, srcs, dsts_init=None, in_place=False, pad=0):
    P = len(srcs)
    ds = [to_dev(torch, a, pad) for a in srcs]
    if in_place:
        dd = ds
    elif dsts_init is not None:
        dd = [to_dev(torch, a, pad) for a in dsts_init]
    else:
        dd = [torch.zeros_like(t) for t in ds]
    S.loopback_allreduce(alg, op, dt, [t.data_ptr() + pad for t in ds],
                         [t.data_ptr() + pad for t in dd], srcs[0].size)
    torch.cuda.synchronize()
    return [from_dev(dd[p], srcs[p], pad) for p in range(P)]


@pytest.mark.parametrize("exclusive", [False, True])
@pytest.mark.parametrize("P", [1, 2, 3, 5, 8, 12])
@pytest.mark.parametrize("dt", [23, 24, 4, 1, 18, 27, 26, 25])
def test_loopback_scan(torch_cuda, exclusive, P, dt):
    torch = torch_cuda
    alg = _lib.PLAN_EXSCAN if exclusive else _lib.PLAN_INSCAN
    for n in (1, 7, 4096 + 3, (1 << 20) + 1):
        if n > 5000 and dt not in (23, 4):
            continue
        srcs = [src_of(dt, n, p, n) for p in range(P)]
        ref = O.scan(5, dt, srcs, exclusive)
        for in_place, pad in ((False, 0), (True, 0), (False, 4)):
            got = loopback(torch, alg, 5, dt, srcs, in_place=in_place, pad=pad)
            for p in range(P):
                assert np.array_equal(bits(got[p]), bits(ref[p])), (P, n, p, in_place, pad)


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8, 9])
@pytest.mark.parametrize("copy_root", [False, True])
def test_loopback_bcast(torch_cuda, P, copy_root):
    torch = torch_cuda
    rng = np.random.default_rng(P)
    for nbytes, dt, np_t in ((1, 13, np.uint8), (1000, 13, np.uint8), (65536, 15, np.uint32),
                             ((4 << 20) + 8, 16, np.uint64), (200001, 13, np.uint8)):
        n = nbytes // np.dtype(np_t).itemsize
        for root in sorted({0, P - 1, P // 2}):
            srcs = [rng.integers(0, 255, n * np.dtype(np_t).itemsize, dtype=np.uint8).view(np_t)
                    for _ in range(P)]
            init = [np.full(n, 0x5A, np_t) for _ in range(P)]
            ref = O.bcast(srcs, root, copy_root, [a.copy() for a in init])
            got = loopback(torch, _lib.plan_bcast(root, copy_root), 5, dt, srcs, dsts_init=init)
            for p in range(P):
                assert np.array_equal(got[p], ref[p]), (P, nbytes, root, p)


@pytest.mark.parametrize("alg", ["ring", "recdbl_direct", "recdbl", "rechalving"])
def test_loopback_reduce_twelve_pes(torch_cuda, alg):
    """12 PEs: ring / recdbl_direct fold 12 inputs in one runtime-P kernel.  The tree
    schedules equal SOS recdbl_sw bit for bit for commutative element semantics (fp sum)."""
    torch = torch_cuda
    P, dt, op = 12, 23, 5
    for n in (13, 50001):
        srcs = [O.fill(dt, 0, n, p, n) for p in range(P)]
        got = loopback(torch, alg, op, dt, srcs)
        ref = O.ring(op, dt, srcs) if alg == "ring" else O.recdbl(op, dt, srcs)
        for p in range(P):
            assert np.array_equal(bits(got[p]), bits(ref[p])), (alg, n, p)


@pytest.mark.parametrize("case", ["allgather8", "ragged", "incongruent", "incongruent_word", "incongruent_many",
                                  "many", "tiny"])
def test_gather_kernel(torch_cuda, case):
    """sosx_gather (the p2p transport's multi-segment copy, copy.hip k_gather): one tile
    per workgroup over the 16-B bodies on the destination's grid (a source at another 16-B
    offset: unaligned loads at 4-B multiples, realigned in registers otherwise), byte loops
    for the ragged ends; more than 16 segments split into several launches.  Every
    destination byte must equal its source byte, and bytes around the segments stay
    untouched."""
    import ctypes
    torch = torch_cuda
    rng = np.random.default_rng(7)
    if case == "allgather8":
        segs = [(0, 0, 4 << 20)] * 7
    elif case == "ragged":
        segs = [(3, 3, 1000003), (16, 16, 65536 + 5), (1, 1, 17), (8, 8, 4096 * 16 + 1)]
    elif case == "incongruent":
        segs = [(1, 2, 100000), (5, 0, 33), (0, 7, 70000)]
    elif case == "incongruent_word":  # sources at 4 / 8 / 12 B from the destination's grid
        segs = [(4, 0, 1000003), (0, 8, 65536 + 9), (13, 1, 300001), (7, 3, 4096 * 64 + 2), (2, 6, 33)]
    elif case == "many":
        segs = [(int(rng.integers(0, 16)),) * 2 + (int(rng.integers(1, 200000)),) for _ in range(37)]
    elif case == "incongruent_many":  # every src/dst offset pair, bodies realigned in registers
        segs = [(int(rng.integers(0, 16)), int(rng.integers(0, 16)), int(rng.integers(1, 1 << 20)))
                for _ in range(23)]
    else:
        segs = [(0, 0, 1), (15, 15, 15), (4, 9, 0)]
    srcs, dsts, sp, dp, nb = [], [], [], [], []
    for so, do, n in segs:
        s = torch.from_numpy(rng.integers(0, 256, n + 64, dtype=np.uint8)).cuda()
        d = torch.full((n + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        srcs.append((s, so, n))
        dsts.append((d, do, n))
        sp.append(s.data_ptr() + so)
        dp.append(d.data_ptr() + do)
        nb.append(n)
    k = len(segs)
    rc = _lib.lib().sosx_gather(k, (ctypes.c_void_p * k)(*sp), (ctypes.c_void_p * k)(*dp),
                                (ctypes.c_size_t * k)(*nb), None)
    assert rc == 0
    torch.cuda.synchronize()
    for (s, so, n), (d, do, _) in zip(srcs, dsts):
        assert torch.equal(d[do:do + n], s[so:so + n])
        assert bool((d[:do] == 0xA5).all()) and bool((d[do + n:] == 0xA5).all())


def test_gather_dpp_shape_forced():
    """SOSX_GATHER_REALIGN=0 (every incongruent source by the DPP shape, the default only
    for offsets that are not 4-B multiples): the gather cases above rerun in a child."""
    import subprocess
    import sys
    here = os.path.abspath(__file__)
    r = subprocess.run([sys.executable, "-m", "pytest", here, "-q", "-p", "no:cacheprovider", "-k",
                        "test_gather_kernel"], capture_output=True, text=True, timeout=200,
                       env=dict(os.environ, SOSX_GATHER_REALIGN="0"), cwd=os.path.dirname(os.path.dirname(here)))
    assert r.returncode == 0, (r.stdout[-2500:], r.stderr[-1500:])
    assert "7 passed" in r.stdout


def _perspective_inputs(dt, P, n, seed):
    """Inputs whose recdbl_sw value depends on the PE: fp +-0 ties and NaNs with a
    distinct payload per PE (x86 keeps the first NaN operand), next to ordinary values."""
    srcs = [src_of(dt, seed, p, n) for p in range(P)]
    if dt in (23, 24):
        ity = np.uint32 if dt == 23 else np.uint64
        nan0 = ity(0x7FC00000) if dt == 23 else ity(0x7FF8000000000000)
        for p in range(P):
            s = srcs[p]
            s[0] = -0.0 if p % 2 else 0.0
            s.view(ity)[min(1, n - 1)] = nan0 | ity(p + 1)
    return srcs


def _pinned(torch, raw, offset):
    """A pinned host buffer holding `raw` bytes `offset` bytes past a 16-B boundary."""
    buf = torch.zeros(raw.size + 64, dtype=torch.uint8, pin_memory=True)
    base = (-buf.data_ptr()) % 16 + offset
    buf[base:base + raw.size] = torch.from_numpy(raw.copy())
    return buf, buf.data_ptr() + base


# every type/op pair on aligned operands (the 16-B-lane path the small host path takes);
# the misaligned layouts (element lanes, element stores) on a subset of widths
SMALL_CASES = ([(23, 5, "aligned"), (24, 4, "aligned"), (23, 3, "aligned"), (4, 3, "aligned"),
                (27, 6, "aligned"), (25, 5, "aligned"), (1, 6, "aligned")]
               + [(23, 5, "in_misaligned"), (4, 3, "in_misaligned"), (1, 6, "in_misaligned"),
                  (23, 5, "out_misaligned"), (24, 4, "out_misaligned"), (1, 6, "out_misaligned")])


@pytest.mark.parametrize("P", [2, 3, 4, 5, 7, 8, 12, 16])
@pytest.mark.parametrize("dt,op,layout", SMALL_CASES)
def test_small_fold_kernel(torch_cuda, P, dt, op, layout):
    """sosx_small_fold (the small host-resident path's one launch): operands, result and
    completion words all in pinned host memory, every PE's own recdbl_sw value (oracle
    recdbl, per PE: +-0 ties and NaN payloads included).  Aligned operands take the
    16-B-vector lanes; a misaligned operand the element lanes; a misaligned result vector
    loads with element stores.  Exactly the first *nblocks completion words carry the
    call's sequence number."""
    import ctypes
    torch = torch_cuda
    L = _lib.lib()
    p2 = 1 << (P.bit_length() - 1)
    nx = P - p2
    flags = torch.zeros(4096 + 8, dtype=torch.int32, pin_memory=True)
    seq = 0
    for n in (1, 255, 257, 4095, 20001):
        srcs = _perspective_inputs(dt, P, n, seed=n + P)
        ref = O.recdbl(op, dt, srcs)
        es = srcs[0].itemsize
        keep, ptr = [], []
        for p, a in enumerate(srcs):
            b, q = _pinned(torch, np.frombuffer(a.tobytes(), np.uint8),
                           es if (layout == "in_misaligned" and p == P - 1 and es < 16) else 0)
            keep.append(b)
            ptr.append(q)
        ob, optr = _pinned(torch, np.zeros(srcs[0].nbytes, np.uint8),
                           es if (layout == "out_misaligned" and es < 16) else 0)
        for me in sorted({0, P // 2, P - 1}):
            mp = me if me < p2 else me - p2
            leaves = [ptr[y ^ mp] for y in range(p2)]
            extras = [ptr[(y ^ mp) + p2] if (y ^ mp) < nx else None for y in range(p2)]
            seq += 1
            ob.fill_(0xA5)
            nb = ctypes.c_int(-1)
            rc = L.sosx_small_fold(op, dt, ctypes.c_void_p(optr),
                                   (ctypes.c_void_p * p2)(*leaves), (ctypes.c_void_p * p2)(*extras),
                                   p2, ctypes.c_size_t(n), ctypes.c_void_p(flags.data_ptr()),
                                   ctypes.c_uint32(seq), ctypes.byref(nb), None)
            assert rc == 0
            torch.cuda.synchronize()
            assert 1 <= nb.value <= (n + 255) // 256
            assert bool((flags[:nb.value] == seq).all()) and int(flags[nb.value]) != seq, (n, me)
            off = optr - ob.data_ptr()
            got = np.frombuffer(ob[off:off + srcs[0].nbytes].numpy().tobytes(), srcs[0].dtype)
            assert np.array_equal(bits(got), bits(ref[me])), (P, dt, op, n, me, layout)


@pytest.mark.parametrize("P", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("dt,op,layout", SMALL_CASES)
def test_small_ring_kernel(torch_cuda, P, dt, op, layout):
    """sosx_small_ring (the small host-resident path above the crossover): operands,
    result and completion words in pinned host memory; every element equals SOS's ring
    result (oracle ring: chunk c folded from PE c, src/collectives.c:693-727), ragged
    sizes included (n < P leaves chunks empty, chunk starts off the 16-B grid); aligned,
    misaligned-operand and misaligned-result layouts; exactly the first *nblocks
    completion words carry the call's sequence number."""
    import ctypes
    torch = torch_cuda
    L = _lib.lib()
    flags = torch.zeros(4096 + 8, dtype=torch.int32, pin_memory=True)
    seq = 0
    for n in (1, P - 1, 7, 255 * P + 3, 4097, 65536 + 5):
        if n < 1:
            continue
        srcs = _perspective_inputs(dt, P, n, seed=2 * n + P)
        ref = O.ring(op, dt, srcs)
        for p in range(1, P):
            assert np.array_equal(bits(ref[p]), bits(ref[0]))
        es = srcs[0].itemsize
        keep, ptr = [], []
        for p, a in enumerate(srcs):
            b, q = _pinned(torch, np.frombuffer(a.tobytes(), np.uint8),
                           es if (layout == "in_misaligned" and p == 0 and es < 16) else 0)
            keep.append(b)
            ptr.append(q)
        ob, optr = _pinned(torch, np.full(srcs[0].nbytes, 0xA5, np.uint8),
                           es if (layout == "out_misaligned" and es < 16) else 0)
        seq += 1
        nb = ctypes.c_int(-1)
        rc = L.sosx_small_ring(op, dt, ctypes.c_void_p(optr), (ctypes.c_void_p * P)(*ptr), P,
                               ctypes.c_size_t(n), ctypes.c_void_p(flags.data_ptr()),
                               ctypes.c_uint32(seq), ctypes.byref(nb), None)
        assert rc == 0
        torch.cuda.synchronize()
        assert 1 <= nb.value <= (n + 255) // 256 + P
        assert bool((flags[:nb.value] == seq).all()) and int(flags[nb.value]) != seq, n
        off = optr - ob.data_ptr()
        got = np.frombuffer(ob[off:off + srcs[0].nbytes].numpy().tobytes(), srcs[0].dtype)
        assert np.array_equal(bits(got), bits(ref[0])), (P, dt, op, n, layout)


@pytest.mark.parametrize("np_", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("dt,op,layout", SMALL_CASES)
def test_small_linear_kernel(torch_cuda, np_, dt, op, layout):
    """sosx_small_linear (one PE's team scan on the small host-resident path): the
    in-order LINEAR fold of np operands in pinned host memory equals the oracle's
    reduce_local prefix (SOS scan_ring order, running value the left operand)."""
    import ctypes
    torch = torch_cuda
    L = _lib.lib()
    flags = torch.zeros(4096 + 8, dtype=torch.int32, pin_memory=True)
    seq = 0
    for n in (1, 7, 4097, 65536 + 5):
        srcs = _perspective_inputs(dt, np_, n, seed=3 * n + np_)
        ref = cpu_prefix(op, dt, srcs)[-1]
        es = srcs[0].itemsize
        keep, ptr = [], []
        for p, a in enumerate(srcs):
            b, q = _pinned(torch, np.frombuffer(a.tobytes(), np.uint8),
                           es if (layout == "in_misaligned" and p == 0 and es < 16) else 0)
            keep.append(b)
            ptr.append(q)
        ob, optr = _pinned(torch, np.full(srcs[0].nbytes, 0xA5, np.uint8),
                           es if (layout == "out_misaligned" and es < 16) else 0)
        seq += 1
        nb = ctypes.c_int(-1)
        rc = L.sosx_small_linear(op, dt, ctypes.c_void_p(optr), (ctypes.c_void_p * np_)(*ptr), np_,
                                 ctypes.c_size_t(n), ctypes.c_void_p(flags.data_ptr()),
                                 ctypes.c_uint32(seq), ctypes.byref(nb), seq % 2, None)
        assert rc == 0
        torch.cuda.synchronize()
        assert 1 <= nb.value <= (n + 255) // 256
        assert bool((flags[:nb.value] == seq).all()) and int(flags[nb.value]) != seq, n
        off = optr - ob.data_ptr()
        got = np.frombuffer(ob[off:off + srcs[0].nbytes].numpy().tobytes(), srcs[0].dtype)
        assert np.array_equal(bits(got), bits(ref)), (np_, dt, op, n, layout)


@pytest.mark.parametrize("nwords", [1, 7, 8, 9, 63])
@pytest.mark.parametrize("src_off,dst_off", [(0, 0), (4, 0), (0, 8), (1, 3)])
def test_small_stage_kernel(torch_cuda, nwords, src_off, dst_off):
    """sosx_small_stage (the small path's staging of a device operand): the bytes land in
    pinned host memory unchanged, at every size and (mis)alignment, and every post word
    holds its value afterwards -- through the 8-word and the 64-word argument blocks."""
    import ctypes
    torch = torch_cuda
    L = _lib.lib()
    rng = np.random.default_rng(nwords * 31 + src_off * 7 + dst_off)
    words = torch.zeros(64 * 8, dtype=torch.int64, pin_memory=True)   # one per 64-B line
    wptr = [words.data_ptr() + 64 * k for k in range(nwords)]
    call = 0
    for nbytes in (1, 15, 16, 4096 + 3, 65536, (1 << 20) - 5):
        call += 1
        raw = rng.integers(0, 256, nbytes + 32, dtype=np.uint8)
        src = torch.from_numpy(raw).cuda()
        dst = torch.zeros(nbytes + 64, dtype=torch.uint8, pin_memory=True)
        dbase = (-dst.data_ptr()) % 16 + dst_off
        vals = [call * 1000 + k for k in range(nwords)]
        torch.cuda.synchronize()
        rc = L.sosx_small_stage(ctypes.c_void_p(dst.data_ptr() + dbase),
                                ctypes.c_void_p(src.data_ptr() + src_off), ctypes.c_size_t(nbytes),
                                (ctypes.c_void_p * nwords)(*wptr), (ctypes.c_uint64 * nwords)(*vals),
                                nwords, None)
        assert rc == 0
        torch.cuda.synchronize()
        got = dst[dbase:dbase + nbytes].numpy()
        assert np.array_equal(got, raw[src_off:src_off + nbytes]), (nbytes, src_off, dst_off)
        assert int(dst[:dbase].sum()) == 0 and int(dst[dbase + nbytes:].sum()) == 0
        w = words.view(-1, 8)[:, 0].numpy()
        assert list(w[:nwords]) == vals and not w[nwords:].any(), nbytes
