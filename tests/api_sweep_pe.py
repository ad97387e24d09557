"""One PE of the public-API sweep (run under tools/oshrun by tests/test_gpu_multipe.py).

Every generated typed reduction -- the 154 shmem_<T>_<op>_reduce and the 44
shmem_<T>_<op>_to_all of bindings/shmem_bind_c.m4 (tables in sos_amd/csrc/gen_bindings.py)
-- is called across the real PE processes, at nreduce = 37 on pageable host buffers (SOS
AUTO -> recdbl_sw below 16 KiB) and at nreduce = 5000 on device buffers (ring for types
of >= 4 bytes).  Each PE checks its own target bit for bit against the CPU oracle's SOS
schedule over every PE's regenerated input (oracle.recdbl / oracle.ring, chosen by the
AUTO rule of src/shmem_collectives.h:200-221), and that pSync is left at SHMEM_SYNC_VALUE.
Test infrastructure: the oracle is the checker only.
"""
import ctypes
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sos_amd", "csrc"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gen_bindings as G  # noqa: E402
from oracle import oracle as O  # noqa: E402
from sos_amd import _lib as L  # noqa: E402
from sos_amd import shmem as S  # noqa: E402

ITYPE = {"SHORT": "short", "INT": "int", "LONG": "long", "LONG_LONG": "longlong",
         "UCHAR": "uchar", "USHORT": "ushort", "UINT": "uint", "ULONG": "ulong",
         "ULONG_LONG": "ulonglong", "INT8": "int8", "INT16": "int16", "INT32": "int32",
         "INT64": "int64", "SIZE_T": "size", "CHAR": "char", "SCHAR": "schar",
         "PTRDIFF_T": "ptrdiff", "FLOAT": "float", "DOUBLE": "double",
         "LONG_DOUBLE": "longdouble", "DOUBLE_COMPLEX": "complexd", "FLOAT_COMPLEX": "complexf"}


def make_input(dt, dist, seed, pe, n):
    if dt == 25:  # long double: no counter-hash generator; seeded numpy values, x87 80-bit
        rng = np.random.default_rng(seed * 64 + pe)
        v = (rng.uniform(0.5, 2.0, n) if dist else rng.standard_normal(n)).astype(np.longdouble)
        v.view(np.uint8).reshape(n, 16)[:, 10:] = 0  # x87 padding: defined bytes on every PE
        return v
    return O.fill(dt, dist, seed, pe, n)


def expected(dt, op, dist, seed, P, me, n):
    ins = [make_input(dt, dist, seed, pe, n) for pe in range(P)]
    es = ins[0].itemsize
    if P == 1:
        return ins[me]
    outs = O.ring(op, dt, ins) if n * es >= 16384 else O.recdbl(op, dt, ins)
    return outs[me]


def main():
    S.shmem_init()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    torch.cuda.set_device(S.lib().shmemx_get_device())
    world = S.team_world()
    bad, checks = [], 0
    calls = [("reduce", st, ct, it, op) for (st, ct, it), op in G.REDUCE]
    calls += [("to_all", st, ct, it, op) for (st, ct, it), op in G.TO_ALL]
    psync = np.zeros(35, dtype=np.int64)
    for kind, st, ct, it, op in calls:
        dt = L.dtype_id(ITYPE[it])
        opid = L.op_id(op)
        dist = L.DIST_PROD if op == "prod" else L.DIST_UNIFORM
        name = f"shmem_{st}_{op}_{kind}"
        fn = getattr(S.lib(), name)
        for n in (37, 5000):
            seed = zlib.crc32(f"{name}/{n}".encode())
            src = make_input(dt, dist, seed, me, n)
            ref = expected(dt, opid, dist, seed, P, me, n)
            if n == 37:  # pageable host buffers
                dst = np.zeros_like(src)
                sp, dp = src.ctypes.data, dst.ctypes.data
            else:         # device buffers
                raw = np.frombuffer(src.tobytes(), np.uint8)
                t_src = torch.from_numpy(raw.copy()).cuda()
                t_dst = torch.zeros_like(t_src)
                torch.cuda.synchronize()
                sp, dp = t_src.data_ptr(), t_dst.data_ptr()
            if kind == "reduce":
                fn.restype = ctypes.c_int
                fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
                rc = fn(world, dp, sp, n)
                if rc != 0:
                    bad.append((name, n, "rc", rc))
            else:
                pwrk = np.zeros(max(n // 2 + 1, 1) * src.itemsize, np.uint8)
                fn.restype = None
                fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
                fn(dp, sp, n, 0, 0, P, pwrk.ctypes.data, psync.ctypes.data)
                if psync.any():
                    bad.append((name, n, "pSync not restored"))
            got = dst if n == 37 else np.frombuffer(t_dst.cpu().numpy().tobytes(), src.dtype)
            checks += 1
            if got.tobytes() != ref.tobytes():
                nd = int(np.count_nonzero(np.frombuffer(got.tobytes(), np.uint8)
                                          != np.frombuffer(ref.tobytes(), np.uint8)))
                bad.append((name, n, f"{nd} bytes differ"))
    checks += sweep_scans_bcasts(world, me, P, bad)
    S.shmem_barrier_all()
    S.shmem_finalize()
    if bad:
        print(f"PE {me}/{P}: {len(bad)} of {checks} checks FAILED: {bad[:8]}", flush=True)
        return 1
    print(f"PE {me}/{P}: {checks} checks OK", flush=True)
    return 0


CSIZE = {"float": 4, "double": 8, "long double": 16, "char": 1, "signed char": 1, "short": 2,
         "int": 4, "long": 8, "long long": 8, "unsigned char": 1, "unsigned short": 2,
         "unsigned int": 4, "unsigned long": 8, "unsigned long long": 8, "int8_t": 1,
         "int16_t": 2, "int32_t": 4, "int64_t": 8, "uint8_t": 1, "uint16_t": 2, "uint32_t": 4,
         "uint64_t": 8, "size_t": 8, "ptrdiff_t": 8}


def _buffers(src, n_bytes_on_device):
    """(src_ptr, dst_ptr, read_dst) for host (small) or device (large) operands."""
    if not n_bytes_on_device:
        dst = np.full(src.nbytes, 0x5A, np.uint8)
        return src.ctypes.data, dst.ctypes.data, lambda: dst.tobytes(), (src, dst)
    t_src = torch.from_numpy(np.frombuffer(src.tobytes(), np.uint8).copy()).cuda()
    t_dst = torch.full_like(t_src, 0x5A)
    torch.cuda.synchronize()
    return t_src.data_ptr(), t_dst.data_ptr(), lambda: t_dst.cpu().numpy().tobytes(), (t_src, t_dst)


def sweep_scans_bcasts(world, me, P, bad):
    """The 52 team scans shmemx_<T>_sum_{inscan,exscan} (oracle.scan = SOS scan_ring,
    src/collectives.c:1111-1209) and the 24 typed team broadcasts shmem_<T>_broadcast
    from team PE 1 % P (oracle.bcast, src/collectives.c:429-485)."""
    checks = 0
    for (st, ct, it), kind in G.SCANS:
        dt = L.dtype_id(ITYPE[it])
        name = f"shmemx_{st}_sum_{kind}"
        fn = getattr(S.lib(), name)
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        for n in (37, 5000):
            seed = zlib.crc32(f"{name}/{n}".encode())
            ins = [make_input(dt, 0, seed, pe, n) for pe in range(P)]
            ref = O.scan(5, dt, ins, kind == "exscan",
                         [np.frombuffer(np.full(ins[0].nbytes, 0x5A, np.uint8).tobytes(),
                                        ins[0].dtype).copy() for _ in range(P)])[me]
            sp, dp, read, keep = _buffers(ins[me], n == 5000)
            rc = fn(world, dp, sp, n)
            checks += 1
            if rc != 0 or read() != ref.tobytes():
                bad.append((name, n, "rc" if rc else "bytes differ"))
            del keep
    root = 1 % P
    for st, ct in G.RMA:
        es = CSIZE[ct]
        name = f"shmem_{st}_broadcast"
        fn = getattr(S.lib(), name)
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                       ctypes.c_int]
        for n in (37, 5000):
            seed = zlib.crc32(f"{name}/{n}".encode())
            srcs = [np.random.default_rng(seed * 64 + pe).integers(0, 256, n * es, dtype=np.uint8)
                    for pe in range(P)]
            init = [np.full(n * es, 0x5A, np.uint8) for _ in range(P)]
            ref = O.bcast(srcs, root, True, init)[me]
            sp, dp, read, keep = _buffers(srcs[me], n == 5000)
            rc = fn(world, dp, sp, n, root)
            checks += 1
            if rc != 0 or read() != ref.tobytes():
                bad.append((name, n, "rc" if rc else "bytes differ"))
            del keep
    return checks


if __name__ == "__main__":
    sys.exit(main())
