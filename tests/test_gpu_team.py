"""GPU: the team reduction end to end.

* loopback team: P = 1..8 simulated PEs on one MI355X run the exact per-PE plans of
  the RCCL executor (fused fold kernels, scratch layout, in-place handling) with
  device-to-device copies as the transport; results must equal the oracle's SOS ring /
  recdbl bit for bit.
* public API on one PE: shmem_init + shmem_<T>_<op>_reduce / _to_all on device and
  host buffers, shmemx_reduce_local, and the example programs.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def dev_bytes(torch, arr, pad=0):
    raw = np.frombuffer(arr.tobytes(), np.uint8)
    buf = torch.zeros(raw.size + pad + 64, dtype=torch.uint8, device="cuda")
    buf[pad:pad + raw.size] = torch.from_numpy(raw.copy()).cuda()
    return buf


def host_view(buf, pad, like):
    return np.frombuffer(buf.cpu().numpy()[pad:pad + like.nbytes].tobytes(), dtype=like.dtype)


CASES = [(23, 5, 0), (24, 6, 1), (11, 2, 0), (4, 4, 0), (18, 3, 0), (27, 6, 1), (26, 5, 0),
         (1, 5, 0), (10, 0, 0)]


@pytest.mark.parametrize("alg", ["ring", "recdbl", "rechalving", "recdbl_direct", "recdbl_gather", "auto"])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 8])
def test_loopback_schedules(torch_cuda, sos, oracle, alg, P):
    from sos_amd import shmem as S
    torch = torch_cuda
    for dt, op, dist in CASES:
        if alg in ("rechalving", "recdbl_direct") and (dt, op) in ((4, 4), (18, 3)):
            continue  # min/max ties are perspective dependent: recdbl/ring only
        for n in (1, 37, 4096 * 3 + 5):
            for in_place in (False, True):
                srcs = [oracle.fill(dt, dist, 500 + n, p, n) for p in range(P)]
                bytes_ = n * srcs[0].itemsize
                if alg == "ring" or (alg == "auto" and bytes_ >= 16384):
                    ref = oracle.ring(op, dt, srcs)
                else:
                    ref = oracle.recdbl(op, dt, srcs)
                pad = 16 * (P % 3)  # some PEs' buffers start off 256-B alignment
                sb = [dev_bytes(torch, s, pad) for s in srcs]
                db = sb if in_place else [torch.zeros_like(b) for b in sb]
                S.loopback_allreduce(alg, op, dt, [b.data_ptr() + pad for b in sb],
                                     [b.data_ptr() + pad for b in db], n)
                torch.cuda.synchronize()
                for p in range(P):
                    want = ref[p] if alg in ("ring", "recdbl", "recdbl_gather", "auto") else ref[0]
                    got = host_view(db[p], pad, srcs[p])
                    assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), \
                        (alg, P, dt, op, n, in_place, p)


def test_loopback_large_ring_fp32(torch_cuda, sos, oracle):
    """8 PEs x 4Mi fp32 through the ring plan: bit-exact with SOS ring."""
    from sos_amd import shmem as S
    torch = torch_cuda
    P, n = 8, 4 << 20
    srcs = [oracle.fill(23, 0, 0x5EED, p, n) for p in range(P)]
    ref = oracle.ring(5, 23, srcs)
    sb = [torch.from_numpy(s).cuda() for s in srcs]
    db = [torch.empty_like(b) for b in sb]
    S.loopback_allreduce("ring", 5, 23, [b.data_ptr() for b in sb], [b.data_ptr() for b in db], n)
    torch.cuda.synchronize()
    for p in range(P):
        assert np.array_equal(db[p].cpu().numpy().view(np.uint32), ref[p].view(np.uint32))


@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("spad,dpad", [(4, 0), (0, 8), (12, 4)])
def test_loopback_ring_source_target_misaligned(torch_cuda, sos, oracle, P, spad, dpad):
    """Ring team reductions whose source and target start at different 16-B offsets, with
    chunks past 64 KiB: the fold's own-chunk input is incongruent with the target and its
    scratch slots (k_fold_realign); bit for bit with SOS's ring."""
    from sos_amd import shmem as S
    torch = torch_cuda
    for dt, op in ((23, 5), (11, 2), (3, 4)):
        n = (1 << 20) + 5
        srcs = [oracle.fill(dt, 0, 77 + dt, p, n) for p in range(P)]
        ref = oracle.ring(op, dt, srcs)
        es = srcs[0].itemsize
        sp, dp = (spad // es) * es, (dpad // es) * es
        sb = [dev_bytes(torch, s, sp) for s in srcs]
        db = [torch.zeros(n * es + dp + 64, dtype=torch.uint8, device="cuda") for _ in range(P)]
        S.loopback_allreduce("ring", op, dt, [b.data_ptr() + sp for b in sb], [b.data_ptr() + dp for b in db], n)
        torch.cuda.synchronize()
        for p in range(P):
            got = host_view(db[p], dp, srcs[p])
            assert np.array_equal(got.view(np.uint8), ref[p].view(np.uint8)), (P, dt, op, sp, dp, p)


@pytest.fixture(scope="module")
def shmem1(torch_cuda, sos):
    from sos_amd import shmem as S
    os.environ.pop("WORLD_SIZE", None)
    S.shmem_init()
    assert S.shmem_n_pes() == 1 and S.shmem_my_pe() == 0
    yield S


def test_api_one_pe_device_and_host(torch_cuda, shmem1, oracle):
    S, torch = shmem1, torch_cuda
    team = S.team_world()
    n = 1 << 16
    src = torch.from_numpy(oracle.fill(23, 0, 1, 0, n)).cuda()
    dst = torch.zeros_like(src)
    assert S.shmem_float_sum_reduce(team, dst.data_ptr(), src.data_ptr(), n) == 0
    torch.cuda.synchronize()
    assert torch.equal(dst, src)  # PE_size 1: copy, as SOS (src/collectives.c:664-668)
    h = oracle.fill(11, 0, 2, 0, n)
    out = np.zeros_like(h)
    assert S.shmem_int64_xor_reduce(team, out.ctypes.data, h.ctypes.data, n) == 0
    assert np.array_equal(out, h)
    ld = np.arange(8, dtype=np.longdouble)
    lo = np.zeros_like(ld)
    S.shmem_longdouble_sum_reduce(team, lo.ctypes.data, ld.ctypes.data, 8)  # 1 PE: copy works
    assert np.array_equal(lo, ld)


def test_api_to_all_psync_untouched(torch_cuda, shmem1, oracle):
    S = shmem1
    n = 1000
    src = oracle.fill(24, 0, 3, 0, n)
    dst = np.zeros_like(src)
    psync = np.zeros(35, dtype=np.int64)
    pwrk = np.zeros(n // 2 + 1, dtype=np.float64)
    S.shmem_double_sum_to_all(dst.ctypes.data, src.ctypes.data, n, 0, 0, 1, pwrk.ctypes.data,
                              psync.ctypes.data)
    assert np.array_equal(dst, src) and not psync.any()


def test_reduce_local_extension(torch_cuda, shmem1, oracle):
    S, torch = shmem1, torch_cuda
    n = 12345
    a, b = oracle.fill(24, 1, 4, 0, n), oracle.fill(24, 1, 4, 1, n)
    ref = a.copy()
    oracle.reduce_local(6, 24, b, ref)
    da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    assert S.shmemx_reduce_local(6, 24, n, db.data_ptr(), da.data_ptr()) == 0
    torch.cuda.synchronize()
    assert np.array_equal(da.cpu().numpy().view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("where", ["dev_inout_host_in", "host_inout_dev_in", "host_both"])
def test_reduce_local_mixed_residency(torch_cuda, shmem1, oracle, where):
    """Pageable host operands next to HBM ones: the host side is staged, never dereferenced
    by the kernel, and every path has completed when the call returns (no synchronize)."""
    S, torch = shmem1, torch_cuda
    n = (1 << 18) + 7
    a, b = oracle.fill(23, 0, 9, 0, n), oracle.fill(23, 0, 9, 1, n)
    ref = a.copy()
    oracle.reduce_local(5, 23, b, ref)
    io_h, in_h = a.copy(), b.copy()  # numpy = pageable malloc memory
    io_d, in_d = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    torch.cuda.synchronize()
    if where == "dev_inout_host_in":
        assert S.shmemx_reduce_local(5, 23, n, in_h.ctypes.data, io_d.data_ptr()) == 0
        got = io_d.cpu().numpy()
    elif where == "host_inout_dev_in":
        assert S.shmemx_reduce_local(5, 23, n, in_d.data_ptr(), io_h.ctypes.data) == 0
        got = io_h  # read straight away: the call is synchronous
    else:
        assert S.shmemx_reduce_local(5, 23, n, in_h.ctypes.data, io_h.ctypes.data) == 0
        got = io_h
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(in_h.view(np.uint32), b.view(np.uint32))  # `in` left untouched


@pytest.mark.parametrize("dt,op", [(23, 5), (24, 6), (4, 3), (27, 6), (25, 5), (13, 2)])
def test_reduce_local_small(torch_cuda, shmem1, oracle, dt, op):
    """shmemx_reduce_local on operands of at most 64 KiB (one launch, completion words):
    device / device, host heap / host heap (in place in pinned memory), pageable /
    pageable and heap / pageable (staged), and an in-place call -- each bit for bit the
    oracle's reduce_local, `in` untouched, the result there when the call returns."""
    import ctypes
    S, torch = shmem1, torch_cuda
    es = S.lib().sosx_dtype_size(dt)
    for n in (1, 7, 4097, 65536 // es):
        dist = 1 if op == 6 else 0
        if dt == 25:
            a = np.random.default_rng(n).standard_normal(n).astype(np.longdouble)
            b = np.random.default_rng(n + 1).standard_normal(n).astype(np.longdouble)
        else:
            a, b = oracle.fill(dt, dist, 5, 0, n), oracle.fill(dt, dist, 5, 1, n)
        ref = a.copy()
        oracle.reduce_local(op, dt, b, ref)
        nb = n * es
        ha, hb = S.lib().shmem_malloc(nb), S.lib().shmem_malloc(nb)
        try:
            for where in ("device", "heap", "pageable", "heap_pageable", "inplace_heap"):
                if where == "device":
                    io = torch.from_numpy(a.view(np.uint8).copy()).cuda()
                    ii = torch.from_numpy(b.view(np.uint8).copy()).cuda()
                    torch.cuda.synchronize()
                    assert S.shmemx_reduce_local(op, dt, n, ii.data_ptr(), io.data_ptr()) == 0
                    got = io.cpu().numpy().tobytes()
                    want = ref.tobytes()
                elif where in ("heap", "heap_pageable"):
                    ctypes.memmove(ha, a.ctypes.data, nb)
                    src = b.copy()
                    if where == "heap":
                        ctypes.memmove(hb, b.ctypes.data, nb)
                        src_ptr = hb
                    else:
                        src_ptr = src.ctypes.data
                    assert S.shmemx_reduce_local(op, dt, n, src_ptr, ha) == 0
                    got = ctypes.string_at(ha, nb)
                    want = ref.tobytes()
                    assert src.tobytes() == b.tobytes()
                elif where == "pageable":
                    io, ii = a.copy(), b.copy()
                    assert S.shmemx_reduce_local(op, dt, n, ii.ctypes.data, io.ctypes.data) == 0
                    got, want = io.tobytes(), ref.tobytes()
                    assert ii.tobytes() == b.tobytes()
                else:  # inout == in, both the same host-heap buffer: out = a OP a
                    ctypes.memmove(ha, a.ctypes.data, nb)
                    self_ref = a.copy()
                    oracle.reduce_local(op, dt, a.copy(), self_ref)
                    assert S.shmemx_reduce_local(op, dt, n, ha, ha) == 0
                    got, want = ctypes.string_at(ha, nb), self_ref.tobytes()
                if dt == 25:  # x87 80-bit payload of each 16-B slot (6 padding bytes kept)
                    got = b"".join(got[i:i + 10] for i in range(0, nb, 16))
                    want = b"".join(want[i:i + 10] for i in range(0, nb, 16))
                assert got == want, (dt, op, n, where)
        finally:
            S.lib().shmem_free(hb)
            S.lib().shmem_free(ha)


def _run(cmd, timeout=120, env=None):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e)


def test_examples_one_pe():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples")], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    r = _run([os.path.join(ROOT, "examples", "pi_reduce_amd")])
    assert r.returncode == 0, r.stderr
    # (RCCL may print its version banner on stdout first, depending on NCCL_DEBUG)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("Pi from")]
    assert lines == ["Pi from 10000 points on 1 PEs: 3.171200"], r.stdout
    r = _run([os.path.join(ROOT, "examples", "reduce_types")])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "reduce_types: OK" in r.stdout


def test_error_aborts_like_sos():
    code = ("import ctypes, numpy as np\nfrom sos_amd import shmem as S\nS.shmem_init()\n"
            "a = np.zeros(4, np.int32)\n"
            "S.shmem_int_sum_to_all(a.ctypes.data, a.ctypes.data, 4, 0, 0, 5, None, None)\n")
    r = _run(["python", "-c", code], env={"PYTHONPATH": ROOT})
    assert r.returncode == 1
    assert "Invalid active set" in r.stderr
    # the set {0, 1} on a 1-PE job: SOS's `> num_pes` test admits it (and then waits on the
    # missing PE 1); this build refuses it
    r = _run(["python", "-c", code.replace("4, 0, 0, 5,", "4, 0, 0, 2,")], env={"PYTHONPATH": ROOT})
    assert r.returncode == 1 and "Invalid active set" in r.stderr, r.stderr[-2000:]
    code2 = ("import numpy as np\nfrom sos_amd import shmem as S\nS.shmem_init()\n"
             "a = np.zeros(8, np.int32)\n"
             "S.shmem_int_sum_reduce(S.team_world(), a.ctypes.data + 4, a.ctypes.data, 4)\n")
    r = _run(["python", "-c", code2], env={"PYTHONPATH": ROOT})
    assert r.returncode == 1 and "overlaps" in r.stderr
    # logPE_stride outside [0, 30]: SOS shifts 1 << logPE_stride unchecked (undefined)
    for bad in ("4, 0, 31, 1,", "4, 0, -1, 1,"):
        r = _run(["python", "-c", code.replace("4, 0, 0, 5,", bad)], env={"PYTHONPATH": ROOT})
        assert r.returncode == 1 and "Invalid active set" in r.stderr and "logPE_stride" in r.stderr, \
            r.stderr[-2000:]
    # nreduce * sizeof(T) past SIZE_MAX: refused, not wrapped into a small size
    code3 = ("import numpy as np\nfrom sos_amd import shmem as S\nS.shmem_init()\n"
             "a = np.zeros(8, np.int32)\n"
             "S.shmem_int_sum_reduce(S.team_world(), a.ctypes.data, a.ctypes.data, (1 << 63) + 1)\n")
    r = _run(["python", "-c", code3], env={"PYTHONPATH": ROOT})
    assert r.returncode == 1 and "overflows" in r.stderr, r.stderr[-2000:]


def test_info_and_backtrace_env():
    """SHMEM_INFO prints the package string and the parameter table on PE 0 at init
    (src/init.c:240-255, src/shmem_env.c:177-220); SHMEM_BACKTRACE=execinfo adds the
    failing PE's backtrace to an abort (src/backtrace.c:181-206)."""
    code = ("from sos_amd import shmem as S\nS.shmem_init()\nS.shmem_finalize()\n")
    r = _run(["python", "-c", code], env={"PYTHONPATH": ROOT, "SHMEM_INFO": "1",
                                          "SHMEM_REDUCE_ALGORITHM": "ring"})
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Sandia OpenSHMEM" in r.stdout
    line = next(ln for ln in r.stdout.splitlines() if "SHMEM_REDUCE_ALGORITHM" in ln)
    assert " ring (type: string, default: auto)" in line, line
    assert "Collectives options:" in r.stdout and "SHMEMX_TRANSPORT" in r.stdout
    bad = ("import numpy as np\nfrom sos_amd import shmem as S\nS.shmem_init()\n"
           "a = np.zeros(4, np.int32)\n"
           "S.shmem_int_sum_to_all(a.ctypes.data, a.ctypes.data, 4, 0, 0, 5, None, None)\n")
    r = _run(["python", "-c", bad], env={"PYTHONPATH": ROOT, "SHMEM_BACKTRACE": "execinfo"})
    assert r.returncode == 1 and "Invalid active set" in r.stderr
    assert "backtrace (" in r.stderr and "libsos_amd.so" in r.stderr, r.stderr[-2000:]


def test_init_attr_one_pe():
    """shmemx_get_unique_id + shmemx_init_attr (no TCP bootstrap, no node shared memory):
    a reduction, a team split (agreement path without shm) and finalize."""
    code = ("import numpy as np, ctypes\nfrom sos_amd import shmem as S\n"
            "uid = S.get_unique_id()\nS.init_attr(0, 1, uid)\n"
            "assert S.shmem_n_pes() == 1 and S.shmem_my_pe() == 0\n"
            "a = np.arange(1000, dtype=np.int64); b = np.zeros_like(a)\n"
            "assert S.shmem_int64_xor_reduce(S.team_world(), b.ctypes.data, a.ctypes.data, 1000) == 0\n"
            "assert np.array_equal(a, b)\n"
            "t = ctypes.c_void_p()\n"
            "rc = S.lib().shmem_team_split_strided(ctypes.c_void_p(S.team_world()), 0, 1, 1, None, 0,"
            " ctypes.byref(t))\n"
            "assert rc == 0 and t.value, rc\n"
            "S.lib().shmem_team_destroy(t)\n"
            "S.lib().shmem_finalize()\nprint('init_attr ok')\n")
    r = _run(["python", "-c", code], env={"PYTHONPATH": ROOT})
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "init_attr ok" in r.stdout
