"""Multi-PE correctness run of the public reduction API (one process per PE).

Run under tools/oshrun: every PE calls shmem_<T>_<op>_reduce for every schedule
(auto, ring, recdbl, rechalving, recdbl_direct), several types/ops and sizes, on
device-heap buffers (shmemx_malloc_device), on plain device buffers, on pageable host
buffers and on the host symmetric heap (shmem_malloc), in and out of place, over
SHMEM_TEAM_WORLD and over a split team.  Each PE checks its own result bit for bit
against the CPU oracle (oracle/sos_oracle.c: SOS's ring, src/collectives.c:647-764, or
recdbl_sw, :850-984, as the schedule resolves) over every member's input regenerated on
the CPU (oracle_fill, bit-identical to the device generator) -- no library kernel in
the expected value.  Prints one line per PE, exit 0 = OK.

Test infrastructure: the oracle is the checker only.
"""
import ctypes
import os
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from sos_amd import _lib as L  # noqa: E402
from sos_amd import shmem as S  # noqa: E402
from tests import readback as R  # noqa: E402

CASES = [("float", "sum"), ("double", "prod"), ("int64", "xor"), ("int", "max"), ("complexd", "prod"),
         ("short", "sum"), ("uint8", "min"), ("ulong", "or")]
ALGS = ["auto", "ring", "recdbl", "rechalving", "recdbl_direct", "recdbl_gather"]
SIZES = [1, 37, 5003, 65536, (1 << 20) + 3]  # 65536: equal ring chunks for P | 65536


def expected(dt, opid, dist, seed, members, my_idx, n, alg_resolved, pe_of):
    """This PE's expected target bytes, from the oracle over every member's CPU-generated
    input: the ring for ring plans, this PE's recdbl_sw value otherwise (rechalving and
    recdbl_direct evaluate the same tree; for this data, whose ops commute bitwise, every
    PE's recdbl_sw value is the same)."""
    P = len(members)
    ins = [O.fill(dt, dist, seed, pe_of(i), n) for i in range(P)]
    if P == 1:
        out = ins[0]
    elif alg_resolved == L.ALGS["ring"]:
        out = O.ring(opid, dt, ins)[my_idx]
    else:
        out = O.recdbl(opid, dt, ins)[my_idx]
    return R.as_bytes(out)


def main():
    S.shmem_init()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    torch.cuda.set_device(S.lib().shmemx_get_device())
    world = S.team_world()
    bad = []
    checks = 0
    maxn = max(SIZES)
    hsrc = S.shmemx_malloc_device(maxn * 16)
    hdst = S.shmemx_malloc_device(maxn * 16)
    hh_in = S.lib().shmem_malloc(65536 * 16)      # host symmetric heap (pinned)
    hh_out = S.lib().shmem_malloc(65536 * 16)
    # an even-PE team (split_strided), when there are at least 3 PEs
    even = ctypes.c_void_p(0)
    if P >= 3:
        S.lib().shmem_team_split_strided(world, 0, 2, (P + 1) // 2, None, 0, ctypes.byref(even))
    for alg in ALGS:
        S.shmemx_set_reduce_algorithm(L.ALGS[alg])
        for tname, oname in CASES:
            # the binding's internal type: SOS reduces uint8..64 as INT8..64
            # (bindings/shmem_bind_c.m4:113-116, :136-139, :162-165)
            dt = L.dtype_id({"uint8": "int8", "uint16": "int16", "uint32": "int32",
                             "uint64": "int64"}.get(tname, tname))
            opid = L.op_id(oname)
            es = L.dtype_size(dt)
            dist = L.DIST_PROD if oname == "prod" else L.DIST_UNIFORM
            fn = getattr(S, f"shmem_{tname}_{oname}_reduce")
            for n in SIZES:
                if n > 5003 and (tname, oname) not in (("float", "sum"), ("int64", "xor")):
                    continue
                seed = zlib.crc32(f"{alg}/{tname}/{oname}/{n}".encode())
                resolved = S.lib().sosx_resolve_alg(L.ALGS[alg], n * es, 16384)
                exp = None
                for mode in ("heap", "heap_inplace", "device", "host", "hostheap"):
                    # host operands up to 64Ki elements (the small path's ring sizes) at
                    # P <= 4; at P = 8 on one GPU those calls are staged and slow
                    if mode in ("host", "hostheap") and n > (65536 if P <= 4 else 5003):
                        continue
                    L.fill(dt, dist, seed, me, hsrc, n)
                    torch.cuda.synchronize()
                    if mode == "heap":
                        fn(world, hdst, hsrc, n)
                        out = hdst
                    elif mode == "heap_inplace":
                        fn(world, hsrc, hsrc, n)
                        out = hsrc
                    elif mode == "device":
                        t_in = torch.empty(n * es, dtype=torch.uint8, device="cuda")
                        t_out = torch.empty_like(t_in)
                        L.fill(dt, dist, seed, me, t_in.data_ptr(), n)
                        torch.cuda.synchronize()
                        fn(world, t_out.data_ptr(), t_in.data_ptr(), n)
                        out = t_out.data_ptr()
                    elif mode == "host":
                        h_in = R.device_bytes(hsrc, n * es)
                        h_out = np.zeros_like(h_in)
                        fn(world, h_out.ctypes.data, h_in.ctypes.data, n)
                        out = h_out
                    else:
                        h_in = R.device_bytes(hsrc, n * es)      # (keep the array alive)
                        ctypes.memmove(hh_in, h_in.ctypes.data, n * es)
                        fn(world, hh_out, hh_in, n)
                        out = np.ctypeslib.as_array((ctypes.c_uint8 * (n * es)).from_address(hh_out)).copy()
                    if exp is None:
                        exp = expected(dt, opid, dist, seed, list(range(P)), me, n, resolved, lambda i: i)
                    got = out if isinstance(out, np.ndarray) else R.device_bytes(out, n * es)
                    mm = R.mismatches(exp, got, es)
                    checks += 1
                    if mm:
                        bad.append((alg, tname, oname, n, mode, mm, _where(exp, got, out, n, es)))
                # split team: even PEs reduce among themselves
                if even.value and n <= 5003:
                    L.fill(dt, dist, seed, me, hsrc, n)
                    torch.cuda.synchronize()
                    fn(even.value, hdst, hsrc, n)
                    m = (P + 1) // 2
                    exp = expected(dt, opid, dist, seed, list(range(m)), me // 2, n, resolved,
                                   lambda i: 2 * i)
                    mm = R.mismatches(exp, R.device_bytes(hdst, n * es), es)
                    checks += 1
                    if mm:
                        bad.append((alg, tname, oname, n, "even_team", mm))
                    # the same team on the host symmetric heap (small host-resident path)
                    h_in = R.device_bytes(hsrc, n * es)
                    ctypes.memmove(hh_in, h_in.ctypes.data, n * es)
                    fn(even.value, hh_out, hh_in, n)
                    h_out = np.ctypeslib.as_array((ctypes.c_uint8 * (n * es)).from_address(hh_out))
                    mm = R.mismatches(exp, h_out.copy(), es)
                    checks += 1
                    if mm:
                        bad.append((alg, tname, oname, n, "even_team_hostheap", mm))
    # Per-PE perspective values across real processes: fp min/max/sum with +-0 ties and a
    # NaN whose payload differs per PE, under the schedules that give every PE its own
    # recdbl_sw value (recdbl, recdbl_gather, AUTO below the crossover); the PEs'
    # expected targets genuinely differ (x86 keeps the first NaN operand, the ternary
    # min/max returns the second operand on ties).
    for alg in ("recdbl", "recdbl_gather", "auto"):
        S.shmemx_set_reduce_algorithm(L.ALGS[alg])
        for tname, oname in (("double", "max"), ("float", "min"), ("double", "sum")):
            dt, opid = L.dtype_id(tname), L.op_id(oname)
            es = L.dtype_size(dt)
            fn = getattr(S, f"shmem_{tname}_{oname}_reduce")
            for n in (2, 37, 1001):
                seed = zlib.crc32(f"persp/{alg}/{tname}/{oname}/{n}".encode())
                ins = [_perspective(O.fill(dt, L.DIST_UNIFORM, seed, pe, n), pe) for pe in range(P)]
                exp_np = O.recdbl(opid, dt, ins)[me]
                exp = R.as_bytes(exp_np)
                mine = np.frombuffer(ins[me].tobytes(), np.uint8).copy()
                for mode in ("heap", "hostheap", "host"):
                    if mode == "heap":
                        _hip_copy(hsrc, mine.ctypes.data, n * es)
                        fn(world, hdst, hsrc, n)
                        out = hdst
                    elif mode == "hostheap":
                        ctypes.memmove(hh_in, mine.ctypes.data, n * es)
                        fn(world, hh_out, hh_in, n)
                        out = np.ctypeslib.as_array((ctypes.c_uint8 * (n * es)).from_address(hh_out)).copy()
                    else:
                        h_out = np.zeros_like(mine)
                        fn(world, h_out.ctypes.data, mine.ctypes.data, n)
                        out = h_out
                    got = out if isinstance(out, np.ndarray) else R.device_bytes(out, n * es)
                    mm = R.mismatches(exp, got, es)
                    checks += 1
                    if mm:
                        bad.append(("perspective", alg, tname, oname, n, mode, mm))
    # nreduce = 0: every schedule returns at once and leaves the target alone, on the device
    # and on the host heap (SOS returns before any exchange, src/collectives.c:662, :873)
    sentinel = np.full(64, 0xA5, np.uint8)
    for alg in ALGS:
        S.shmemx_set_reduce_algorithm(L.ALGS[alg])
        _hip_copy(hdst, sentinel.ctypes.data, 64)
        S.shmem_float_sum_reduce(world, hdst, hsrc, 0)
        ctypes.memmove(hh_out, sentinel.ctypes.data, 64)
        S.shmem_double_max_reduce(world, hh_out, hh_in, 0)
        back = np.empty(64, np.uint8)
        _hip_copy(back.ctypes.data, hdst, 64)
        hh = np.ctypeslib.as_array((ctypes.c_uint8 * 64).from_address(hh_out)).copy()
        checks += 2
        if not np.array_equal(back, sentinel):
            bad.append(("nreduce=0", alg, "device"))
        if not np.array_equal(hh, sentinel):
            bad.append(("nreduce=0", alg, "hostheap"))
    S.shmemx_set_reduce_algorithm(L.ALGS["auto"])
    S.shmem_barrier_all()
    S.shmemx_free_device(hdst)
    S.shmemx_free_device(hsrc)
    if even.value:
        S.lib().shmem_team_destroy(even)
    S.lib().shmem_free(hh_out)
    S.lib().shmem_free(hh_in)
    sig = {1: "stream", 0: "host"}.get(L.lib().sosx_p2p_signal_mode(), "none")
    small = L.lib().sosx_small_path_calls()
    small_dev = L.lib().sosx_small_path_device_calls()
    S.shmem_finalize()
    if bad:
        print(f"PE {me}/{P}: {len(bad)} of {checks} checks FAILED: {bad[:6]}", flush=True)
        return 1
    print(f"PE {me}/{P}: {checks} checks OK (p2p signal {sig}, small-path calls {small}, "
          f"device {small_dev})", flush=True)
    return 0


def _perspective(a, pe):
    """Element 0 a signed zero by PE parity, element 1 a NaN with payload pe + 1."""
    a = a.copy()
    ity = np.uint32 if a.dtype == np.float32 else np.uint64
    a[0] = -0.0 if pe % 2 else 0.0
    if a.size > 1:
        a.view(ity)[1] = (ity(0x7FC00000) if ity is np.uint32 else ity(0x7FF8000000000000)) | ity(pe + 1)
    return a


def _where(exp, got, out, n, es):
    """Diagnostics of a mismatch: the differing elements as [first, last) runs (at most 4),
    and, for a device result, the count of a second readback (a different count means the
    bytes changed after the call returned)."""
    again = R.mismatches(exp, R.device_bytes(out, n * es), es) if not isinstance(out, np.ndarray) else None
    return {"recount": again, "runs": R.diff_runs(exp, got, es)}


def _hip_copy(dst, src, nbytes):
    L.check(L.lib().sosx_memcpy(dst, src, nbytes, None), "sosx_memcpy")


if __name__ == "__main__":
    sys.exit(main())
