"""GPU parity of the local combine and the fused fold against the CPU oracle.

The oracle (oracle/sos_oracle.c) restates shmem_internal_reduce_local
(src/shmem_internal_op.h:305-339) and the ring / recdbl schedules
(src/collectives.c:647-764, :850-984).  Every (datatype, op) pair SOS accepts is
checked bit for bit, over ragged sizes, misaligned starts and special fp values
(NaN, +-0, +-inf, denormals), plus the Annex G complex-multiply recovery.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# (datatype id, name) for every reducible shm_internal_datatype_t except long double
FP_CLASS = [1, 2, 12, 23, 24]            # char, schar, ptrdiff_t, float, double
CPLX_CLASS = [26, 27]                    # complexf, complexd
INT_CLASS = [3, 4, 5, 6, 8, 9, 10, 11, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22]
OPS_FP = [3, 4, 5, 6]
OPS_CPLX = [5, 6]
OPS_INT = [0, 1, 2, 3, 4, 5, 6]
PAIRS = ([(d, o) for d in FP_CLASS for o in OPS_FP] + [(d, o) for d in CPLX_CLASS for o in OPS_CPLX]
         + [(d, o) for d in INT_CLASS for o in OPS_INT])


def to_dev(torch, arr, offset_bytes=0):
    """Upload the bytes of `arr` into a fresh device buffer at `offset_bytes`."""
    raw = np.frombuffer(arr.tobytes(), dtype=np.uint8)
    buf = torch.zeros(raw.size + offset_bytes + 64, dtype=torch.uint8, device="cuda")
    buf[offset_bytes:offset_bytes + raw.size] = torch.from_numpy(raw.copy()).cuda()
    return buf, buf.data_ptr() + offset_bytes


def from_dev(buf, offset_bytes, like):
    raw = buf.cpu().numpy()[offset_bytes:offset_bytes + like.nbytes]
    return np.frombuffer(raw.tobytes(), dtype=like.dtype).copy()


def special_fp(np_t, n, rng):
    """Random values sprinkled with NaN, +-0, +-inf and denormals."""
    info = np.finfo(np_t)
    base = rng.uniform(-2, 2, n).astype(np_t)
    specials = np.array([np.nan, -np.nan, 0.0, -0.0, np.inf, -np.inf, info.tiny / 4,
                         -info.tiny / 8, info.max, -info.max, 1.0, -1.0], dtype=np_t)
    idx = rng.random(n) < 0.3
    base[idx] = rng.choice(specials, idx.sum())
    return base


def make_inputs(oracle, dt, op, n, rng, special):
    np_t = oracle.np_type(dt)
    if special and dt in (23, 24):
        return special_fp(np_t, n, rng), special_fp(np_t, n, rng)
    if special and dt in (26, 27):
        ft = np.float32 if dt == 26 else np.float64
        def c():
            re, im = special_fp(ft, n, rng), special_fp(ft, n, rng)
            return np.stack([re, im], 1).reshape(-1).view(np_t)
        return c(), c()
    dist = 1 if op == 6 else 0
    seed = int(rng.integers(1 << 62))
    return oracle.fill(dt, dist, seed, 0, n), oracle.fill(dt, dist, seed, 1, n)


def same_bits(a, b):
    return np.array_equal(np.frombuffer(a.tobytes(), np.uint8), np.frombuffer(b.tobytes(), np.uint8))


def same_bits_nan_equiv(a, b):
    """Bitwise equal, except that two NaNs compare equal whatever their payload/sign.

    Used for complex PROD only: which input NaN a NaN product carries depends on the
    operand order gcc's register allocator and libgcc's __mulsc3 chose on x86; every
    non-NaN result (including Annex G recovered infinities) is still bit-exact."""
    ft = np.float32 if a.dtype == np.complex64 else np.float64
    it = np.uint32 if ft == np.float32 else np.uint64
    x, y = a.view(ft), b.view(ft)
    eq = x.view(it) == y.view(it)
    return bool(np.all(eq | (np.isnan(x) & np.isnan(y))))


def check(dt, op, got, ref):
    if dt in (26, 27) and op == 6:
        return same_bits_nan_equiv(got, ref)
    return same_bits(got, ref)


@pytest.mark.parametrize("dt,op", PAIRS)
def test_combine_all_types_ops(torch_cuda, sos, oracle, dt, op):
    torch = torch_cuda
    rng = np.random.default_rng(1000 + 17 * dt + op)
    for n, off in ((1, 0), (7, 0), (4097, 0), (65536 + 3, 0), (1000, 16), (3001, 8)):
        es = oracle.lib().oracle_type_size(dt)
        off = (off // es) * es  # element-aligned offsets, keeps `in` and `inout` congruent
        for special in ((False, True) if dt in (23, 24, 26, 27) else (False,)):
            a, b = make_inputs(oracle, dt, op, n, rng, special)
            ref = a.copy()
            oracle.reduce_local(op, dt, b, ref)
            da, pa = to_dev(torch, a, off)
            db, pb = to_dev(torch, b, off)
            sos.combine(op, dt, pa, pb, n)
            torch.cuda.synchronize()
            got = from_dev(da, off, a)
            assert check(dt, op, got, ref), f"dt={dt} op={op} n={n} off={off} special={special}"


@pytest.mark.parametrize("dt,op", [(23, 5), (24, 6), (11, 2), (4, 4), (27, 6), (13, 3)])
def test_combine_relatively_misaligned(torch_cuda, sos, oracle, dt, op):
    """`in` and `inout` not 16-B congruent: the element-load path."""
    torch = torch_cuda
    rng = np.random.default_rng(7)
    es = oracle.lib().oracle_type_size(dt)
    n = 5000
    a, b = make_inputs(oracle, dt, op, n, rng, False)
    ref = a.copy()
    oracle.reduce_local(op, dt, b, ref)
    da, pa = to_dev(torch, a, 0)
    db, pb = to_dev(torch, b, es if es < 16 else 0)
    sos.combine(op, dt, pa, pb, n)
    torch.cuda.synchronize()
    assert same_bits(from_dev(da, 0, a), ref)


@pytest.mark.parametrize("dt,op", [(18, 5), (3, 2), (23, 5), (4, 4), (24, 6), (11, 2), (26, 5)])
def test_combine_realigned_every_offset(torch_cuda, sos, oracle, dt, op):
    """`in` at every element-aligned 16-B offset relative to `inout` (the realigning
    vector kernel, k_combine3_realign), with `inout` itself on and off a 16-B boundary,
    at sizes from a few elements (head/tail only) to past a million (many tiles); bit for
    bit against the oracle's reduce_local."""
    torch = torch_cuda
    rng = np.random.default_rng(31 + dt)
    es = oracle.lib().oracle_type_size(dt)
    for n in (5, 4097, 65536 + 3, (1 << 20) + 7):
        a, b = make_inputs(oracle, dt, op, n, rng, False)
        ref = a.copy()
        oracle.reduce_local(op, dt, b, ref)
        for a_off in (0, es if es < 16 else 0):
            for d in range(es, 16, es):
                da, pa = to_dev(torch, a, a_off)
                db, pb = to_dev(torch, b, a_off + d)
                sos.combine(op, dt, pa, pb, n)
                torch.cuda.synchronize()
                assert check(dt, op, from_dev(da, a_off, a), ref), f"n={n} a_off={a_off} d={d}"


@pytest.mark.parametrize("mode", ["1", "2"])
def test_combine_realign_shapes_forced(mode):
    """The realigning combine's bench shapes (SOSX_COMBINE_REALIGN: 1 = the next vector by
    DPP, 2 = one unaligned load for 4- and 8-byte elements), bit for bit: the every-offset
    test above reruns in a child process under each."""
    import os
    import subprocess
    import sys
    here = os.path.abspath(__file__)
    r = subprocess.run([sys.executable, "-m", "pytest", here, "-q", "-p", "no:cacheprovider", "-k",
                        "test_combine_realigned_every_offset"], capture_output=True, text=True, timeout=280,
                       env=dict(os.environ, SOSX_COMBINE_REALIGN=mode), cwd=os.path.dirname(os.path.dirname(here)))
    assert r.returncode == 0, (r.stdout[-2500:], r.stderr[-1500:])
    assert "7 passed" in r.stdout


def test_combine3_out_of_place(torch_cuda, sos, oracle):
    torch = torch_cuda
    n = 100003
    a = oracle.fill(23, 0, 5, 0, n)
    b = oracle.fill(23, 0, 5, 1, n)
    ref = a.copy()
    oracle.reduce_local(5, 23, b, ref)
    da, pa = to_dev(torch, a)
    db, pb = to_dev(torch, b)
    dout, po = to_dev(torch, np.zeros_like(a))
    sos.combine3(5, 23, po, pa, pb, n)
    torch.cuda.synchronize()
    assert same_bits(from_dev(dout, 0, a), ref)
    assert same_bits(from_dev(da, 0, a), a)  # inputs untouched


def test_complex_annex_g(torch_cuda, sos, oracle):
    """Both naive parts NaN -> libgcc __mul[sd]c3 recovery (C99 G.5.1)."""
    torch = torch_cuda
    inf, nan = np.inf, np.nan
    pairs = [((inf, 0.0), (0.0, 1.0)), ((inf, inf), (1.0, 0.0)), ((nan, inf), (2.0, 0.0)),
             ((1e300, 1e300), (1e300, -1e300)), ((inf, nan), (nan, 1.0)), ((0.0, 0.0), (inf, nan)),
             ((nan, nan), (1.0, 1.0)), ((-inf, 1.0), (nan, nan)), ((1.0, 2.0), (3.0, -4.0))]
    for dt, ft in ((27, np.float64), (26, np.float32)):
        a = np.array([x for x, _ in pairs], dtype=ft).reshape(-1).view(oracle.np_type(dt))
        b = np.array([y for _, y in pairs], dtype=ft).reshape(-1).view(oracle.np_type(dt))
        ref = a.copy()
        oracle.reduce_local(6, dt, b, ref)
        da, pa = to_dev(torch, a)
        db, pb = to_dev(torch, b)
        sos.combine(6, dt, pa, pb, a.size)
        torch.cuda.synchronize()
        got = from_dev(da, 0, a)
        assert same_bits_nan_equiv(got, ref), (dt, got, ref)
        # the recovered (non-NaN) results must be bit-exact
        ft = np.float32 if dt == 26 else np.float64
        fin = ~np.isnan(ref.view(ft))
        assert np.array_equal(got.view(ft)[fin], ref.view(ft)[fin])


def test_invalid_type_and_op(sos):
    lib = sos.lib()
    assert lib.sosx_combine(5, 0, None, None, 0, None) == -1      # SIGNED_BYTE
    assert lib.sosx_combine(5, 7, None, None, 0, None) == -1      # FORTRAN_INTEGER
    assert lib.sosx_combine(0, 23, None, None, 0, None) == -2     # and on float
    assert lib.sosx_combine(3, 27, None, None, 0, None) == -2     # min on complex
    assert lib.sosx_combine(2, 1, None, None, 0, None) == -2      # xor on char (FP class)


@pytest.mark.parametrize("dt,op", [(23, 5), (24, 6), (11, 2), (10, 3), (4, 4), (27, 6), (26, 5),
                                   (9, 5), (13, 0)])
@pytest.mark.parametrize("P", [2, 3, 5, 8])
def test_fold_matches_oracle_schedules(torch_cuda, sos, oracle, dt, op, P):
    """LINEAR fold == SOS ring fold order; TREE fold == SOS recdbl_sw result."""
    torch = torch_cuda
    n = 3 * 4096 + 5
    dist = 1 if op == 6 else 0
    srcs = [oracle.fill(dt, dist, 99, p, n) for p in range(P)]
    # ring order for a chunk starting at PE c: ((s_c OP s_c+1) OP ...) -> c = 0 here
    lin = srcs[0].copy()
    for p in range(1, P):
        oracle.reduce_local(op, dt, srcs[p], lin)
    tree = oracle.recdbl(op, dt, srcs)[0]
    devs = [to_dev(torch, s) for s in srcs]
    ptrs = [p for _, p in devs]
    for order, ref in ((0, lin), (1, tree)):
        dout, po = to_dev(torch, np.zeros_like(srcs[0]))
        sos.fold(op, dt, order, po, ptrs, n)
        torch.cuda.synchronize()
        assert same_bits(from_dev(dout, 0, srcs[0]), ref), f"order={order}"


def test_fill_matches_oracle(torch_cuda, sos, oracle):
    torch = torch_cuda
    for dt in (23, 24, 26, 27, 4, 11, 13, 9):
        for dist in (0, 1):
            n = 10007
            ref = oracle.fill(dt, dist, 1234, 3, n, 77)
            buf = torch.zeros(ref.nbytes, dtype=torch.uint8, device="cuda")
            sos.fill(dt, dist, 1234, 3, buf.data_ptr(), n, 77)
            torch.cuda.synchronize()
            assert same_bits(from_dev(buf, 0, ref), ref), (dt, dist)


# ---------------------------------------------------------------------------------
# long double: software x87 80-bit arithmetic on the GPU vs the CPU's x87 (oracle)
# ---------------------------------------------------------------------------------
def longdouble_inputs(n, rng):
    ld = np.longdouble
    mant = rng.standard_normal(n).astype(ld) + rng.standard_normal(n).astype(ld) * ld(2.0) ** -40
    a = np.ldexp(mant, rng.integers(-16300, 16300, n))
    small = np.ldexp(mant, rng.integers(-16460, -16370, n))       # denormal range
    pool = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0], dtype=ld)
    pool = np.concatenate([pool, [np.finfo(ld).max, -np.finfo(ld).max, np.finfo(ld).tiny,
                                  np.finfo(ld).tiny / ld(8)]])
    pick = rng.random(n)
    a = np.where(pick < 0.2, small, a)
    sp = rng.random(n) < 0.1
    a[sp] = rng.choice(pool, sp.sum())
    return a.astype(ld)


def ld_equal(got, ref):
    g = got.view(np.uint8).reshape(-1, 16)
    r = ref.view(np.uint8).reshape(-1, 16)
    same = np.all(g == r, axis=1)
    both_nan = np.isnan(got) & np.isnan(ref)
    return same | both_nan


@pytest.mark.parametrize("op", [3, 4, 5, 6])
def test_longdouble_combine_vs_x87(torch_cuda, sos, oracle, op):
    torch = torch_cuda
    rng = np.random.default_rng(80 + op)
    n = 20000
    a = longdouble_inputs(n, rng)
    b = longdouble_inputs(n, rng)
    # cancellation and near-overflow pairs
    b[:500] = -a[:500]
    b[500:1000] = -a[500:1000] * (1 + np.ldexp(np.longdouble(1), -63))
    b[1000:1500] = a[1000:1500]
    ref = a.copy()
    oracle.reduce_local(op, 25, b, ref)
    da, pa = to_dev(torch, a)
    db, pb = to_dev(torch, b)
    sos.combine(op, 25, pa, pb, n)
    torch.cuda.synchronize()
    got = from_dev(da, 0, a)
    ok = ld_equal(got, ref)
    bad = np.nonzero(~ok)[0]
    assert bad.size == 0, [(repr(a[i]), repr(b[i]), repr(got[i]), repr(ref[i])) for i in bad[:5]]


@pytest.mark.parametrize("alg", ["ring", "recdbl"])
def test_longdouble_team_loopback(torch_cuda, sos, oracle, alg):
    from sos_amd import shmem as S
    torch = torch_cuda
    rng = np.random.default_rng(7)
    for P in (2, 3, 5):
        n = 3001
        srcs = [np.ldexp(rng.standard_normal(n).astype(np.longdouble), rng.integers(-30, 30, n))
                for _ in range(P)]
        for op in (5, 6, 4):
            ref = (oracle.ring if alg == "ring" else oracle.recdbl)(op, 25, srcs)
            sb = [to_dev(torch, s)[0] for s in srcs]
            db = [torch.zeros_like(x) for x in sb]
            S.loopback_allreduce(alg, op, 25, [x.data_ptr() for x in sb], [x.data_ptr() for x in db], n)
            torch.cuda.synchronize()
            for p in range(P):
                got = from_dev(db[p], 0, srcs[p])
                assert ld_equal(got, ref[p]).all(), (alg, P, op, p)


@pytest.mark.parametrize("dt,op", [(23, 5), (24, 6), (11, 2), (27, 6), (25, 5)])
def test_combine_host_pipeline(torch_cuda, sos, oracle, dt, op):
    """Host-resident operands through the chunked H2D || combine || D2H pipeline."""
    import ctypes
    rng = np.random.default_rng(dt + op)
    for n, chunk in ((1, 0), (100003, 4096), (3 * 1024 * 1024 + 7, 1 << 20)):
        if dt == 25:
            a = np.ldexp(rng.standard_normal(n).astype(np.longdouble), rng.integers(-9, 9, n))
            b = np.ldexp(rng.standard_normal(n).astype(np.longdouble), rng.integers(-9, 9, n))
        else:
            a, b = make_inputs(oracle, dt, op, n, rng, False)
        ref = a.copy()
        oracle.reduce_local(op, dt, b, ref)
        got = a.copy()
        rc = sos.lib().sosx_combine_host(op, dt, got.ctypes.data_as(ctypes.c_void_p),
                                         b.ctypes.data_as(ctypes.c_void_p), n, chunk)
        assert rc == 0
        assert check(dt, op, got, ref), (dt, op, n, chunk)


def test_combine_host_pipeline_release_and_regrow(torch_cuda, sos, oracle):
    """The host pipeline's HBM slots: grown for a large chunk, reused for a smaller one,
    released (sosx_combine_host_release, as shmem_finalize does) and set up again --
    every call still bit-exact."""
    import ctypes
    L = sos.lib()
    L.sosx_combine_host_release.restype = None
    n = (1 << 21) + 5
    a, b = oracle.fill(24, 0, 31, 0, n), oracle.fill(24, 0, 31, 1, n)
    ref = a.copy()
    oracle.reduce_local(5, 24, b, ref)
    for chunk in (8 << 20, 1 << 20, 0, None, 4 << 20):
        if chunk is None:
            L.sosx_combine_host_release()
            L.sosx_combine_host_release()  # idempotent
            continue
        got = a.copy()
        rc = L.sosx_combine_host(5, 24, got.ctypes.data_as(ctypes.c_void_p),
                                 b.ctypes.data_as(ctypes.c_void_p), n, chunk)
        assert rc == 0
        assert same_bits(got, ref), chunk


def test_combine_past_2_31_elements(torch_cuda, sos, oracle):
    """A local combine of 2^31 + 4101 uint8 elements starting 3 bytes past a 16-B
    boundary (4 GiB of operands): SOS's `int nreduce` stops at 2^31 - 1, this build's
    size_t count does not, and every index stays 64-bit (the vector tiles, the ragged head
    and tail).  Inputs from the device generator and the oracle's (bit-identical) one; the
    expected bytes from the oracle's reduce_local in < 2^31-element slices (an
    elementwise op, so slicing is exact)."""
    torch = torch_cuda
    n, off, dt, op = (1 << 31) + 4101, 3, 18, 5          # uint8 sum (wraps)
    a = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    b = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    sos.fill(dt, 0, 31, 0, a.data_ptr() + off, n)
    sos.fill(dt, 0, 31, 1, b.data_ptr() + off, n)
    torch.cuda.synchronize()
    sos.combine(op, dt, a.data_ptr() + off, b.data_ptr() + off, n)
    torch.cuda.synchronize()
    got = a[off:off + n].cpu().numpy()
    del a, b
    exp = oracle.fill(dt, 0, 31, 0, n)
    step = 1 << 30
    for s in range(0, n, step):
        e = min(n, s + step)
        oracle.reduce_local(op, dt, oracle.fill(dt, 0, 31, 1, e - s, s), exp[s:e])
    assert np.array_equal(got, exp)
    assert not np.array_equal(exp[-4101:], oracle.fill(dt, 0, 31, 0, 4101, n - 4101))  # tail combined
