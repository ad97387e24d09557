"""Python mirror of the shmem.h reduction API (ctypes over libsos_amd.so).

Same names, argument meaning and error behaviour as SOS's C API
(src/collectives_c.c4:221-269): ``shmem_float_sum_reduce(team, dest, source, nreduce)``
returns 0, ``shmem_double_sum_to_all(target, source, nreduce, PE_start, logPE_stride,
PE_size, pWrk, pSync)`` returns None, and invalid arguments abort the process with an
SOS-style message.  Buffers are raw addresses (ints): device pointers (e.g. a torch
tensor's ``data_ptr()``) run in place on the GPU; host addresses are staged.
"""
import ctypes
import re

from . import _lib

_c = ctypes
_RUNTIME = {
    "shmem_init": (None, []),
    "shmem_finalize": (None, []),
    "shmem_my_pe": (_c.c_int, []),
    "shmem_n_pes": (_c.c_int, []),
    "shmem_barrier_all": (None, []),
    "shmem_malloc": (_c.c_void_p, [_c.c_size_t]),
    "shmem_calloc": (_c.c_void_p, [_c.c_size_t, _c.c_size_t]),
    "shmem_free": (None, [_c.c_void_p]),
    "shmem_team_my_pe": (_c.c_int, [_c.c_void_p]),
    "shmem_team_n_pes": (_c.c_int, [_c.c_void_p]),
    "shmem_team_split_strided": (_c.c_int, [_c.c_void_p, _c.c_int, _c.c_int, _c.c_int, _c.c_void_p,
                                            _c.c_long, _c.POINTER(_c.c_void_p)]),
    "shmem_team_destroy": (None, [_c.c_void_p]),
    "shmem_team_split_2d": (_c.c_int, [_c.c_void_p, _c.c_int, _c.c_void_p, _c.c_long,
                                       _c.POINTER(_c.c_void_p), _c.c_void_p, _c.c_long,
                                       _c.POINTER(_c.c_void_p)]),
    "shmem_team_translate_pe": (_c.c_int, [_c.c_void_p, _c.c_int, _c.c_void_p]),
    "shmem_team_get_config": (_c.c_int, [_c.c_void_p, _c.c_long, _c.c_void_p]),
    "shmem_team_sync": (_c.c_int, [_c.c_void_p]),
    "shmemx_get_unique_id": (_c.c_int, [_c.c_void_p, _c.c_size_t]),
    "shmemx_init_attr": (_c.c_int, [_c.c_int, _c.c_int, _c.c_void_p, _c.c_size_t]),
    "shmemx_malloc_device": (_c.c_void_p, [_c.c_size_t]),
    "shmemx_free_device": (None, [_c.c_void_p]),
    "shmemx_set_stream": (None, [_c.c_void_p]),
    "shmemx_get_stream": (_c.c_void_p, []),
    "shmemx_set_reduce_algorithm": (_c.c_int, [_c.c_int]),
    "shmemx_set_transport": (_c.c_int, [_c.c_int]),
    "shmemx_get_device": (_c.c_int, []),
    "shmemx_reduce_local": (_c.c_int, [_c.c_int, _c.c_int, _c.c_size_t, _c.c_void_p, _c.c_void_p]),
    "sosx_loopback_allreduce": (_c.c_int, [_c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                           _c.POINTER(_c.c_void_p), _c.POINTER(_c.c_void_p),
                                           _c.c_size_t, _c.c_void_p]),
    "sosx_plan_encode": (_c.c_longlong, [_c.c_int, _c.c_int, _c.c_int, _c.c_ulonglong,
                                         _c.c_ulonglong, _c.c_uint, _c.c_uint,
                                         _c.POINTER(_c.c_longlong), _c.c_ulonglong]),
    "sosx_resolve_alg": (_c.c_int, [_c.c_int, _c.c_ulonglong, _c.c_ulonglong]),
    "shmem_broadcastmem": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_int]),
    "shmem_broadcast32": (None, [_c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_int, _c.c_int, _c.c_int,
                                 _c.c_int, _c.c_void_p]),
    "shmem_broadcast64": (None, [_c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_int, _c.c_int, _c.c_int,
                                 _c.c_int, _c.c_void_p]),
    "sosx_prof_enable": (None, [_c.c_int]),
    "sosx_prof_get": (None, [_c.POINTER(_c.c_double), _c.POINTER(_c.c_double),
                             _c.POINTER(_c.c_long), _c.POINTER(_c.c_long), _c.POINTER(_c.c_long)]),
}

_REDUCE_RE = re.compile(r"^shmem_(\w+?)_(and|or|xor|min|max|sum|prod)_(reduce|to_all)$")
_SCAN_RE = re.compile(r"^shmemx_(\w+?)_sum_(inscan|exscan)$")
_BCAST_RE = re.compile(r"^shmem_(\w+?)_broadcast$")
_declared = False


def lib():
    global _declared
    L = _lib.lib()
    if not _declared:
        for name, (res, args) in _RUNTIME.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _declared = True
    return L


def team_world():
    return ctypes.c_void_p.in_dll(lib(), "SHMEM_TEAM_WORLD").value


def team_shared():
    return ctypes.c_void_p.in_dll(lib(), "SHMEM_TEAM_SHARED").value


def team_node():
    return ctypes.c_void_p.in_dll(lib(), "SHMEMX_TEAM_NODE").value


def __getattr__(name):
    """shmem_<T>_<op>_reduce / _to_all, shmem_init, ... resolved from the library."""
    L = lib()
    m = _REDUCE_RE.match(name)
    if m:
        fn = getattr(L, name)
        if m.group(3) == "reduce":
            fn.restype = ctypes.c_int
            fn.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_size_t]
        else:
            fn.restype = None
            fn.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                           _c.c_void_p, _c.c_void_p]
        return fn
    if _SCAN_RE.match(name):
        fn = getattr(L, name)
        fn.restype = ctypes.c_int
        fn.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_size_t]
        return fn
    if _BCAST_RE.match(name):
        fn = getattr(L, name)
        fn.restype = ctypes.c_int
        fn.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_int]
        return fn
    if name in _RUNTIME:
        return getattr(L, name)
    raise AttributeError(name)


def init_attr(rank, n_pes, uid):
    buf = ctypes.create_string_buffer(bytes(uid), 128)
    return _lib.check(lib().shmemx_init_attr(rank, n_pes, buf, 128), "shmemx_init_attr")


def get_unique_id():
    buf = ctypes.create_string_buffer(128)
    _lib.check(lib().shmemx_get_unique_id(buf, 128), "shmemx_get_unique_id")
    return buf.raw


def loopback_allreduce(alg, op, dtype, srcs, dsts, count, stream=None):
    P = len(srcs)
    s = (ctypes.c_void_p * P)(*srcs)
    d = (ctypes.c_void_p * P)(*dsts)
    a = _lib.ALGS[alg] if isinstance(alg, str) else int(alg)
    return _lib.check(lib().sosx_loopback_allreduce(a, P, _lib.op_id(op), _lib.dtype_id(dtype), s,
                                                    d, count, stream), "sosx_loopback_allreduce")


def plan(alg, P, me, count, ts, src_mis=0, dst_mis=0):
    """Decode the per-PE plan (see sos_amd/csrc/plan.cpp, sosx_plan_encode)."""
    a = _lib.ALGS[alg] if isinstance(alg, str) else int(alg)
    L = lib()
    n = L.sosx_plan_encode(a, P, me, count, ts, src_mis, dst_mis, None, 0)
    if n < 0:
        raise _lib.SosError(int(n), "sosx_plan_encode")
    buf = (ctypes.c_longlong * n)()
    L.sosx_plan_encode(a, P, me, count, ts, src_mis, dst_mis, buf, n)
    w = list(buf)
    pos = 3
    rounds = []
    for _ in range(w[1]):
        nx, nops = w[pos], w[pos + 1]
        pos += 2
        xfers = []
        for _ in range(nx):
            send, peer, b, off, nbytes = w[pos:pos + 5]
            pos += 5
            xfers.append({"send": send, "peer": peer, "buf": b, "off": off, "bytes": nbytes})
        ops = []
        for _ in range(nops):
            kind, order, ob, ooff, nin, cnt = w[pos:pos + 6]
            pos += 6
            ins = []
            for _ in range(nin):
                ins.append((w[pos], w[pos + 1]))
                pos += 2
            nout = w[pos]
            pos += 1
            outs = []
            for _ in range(nout):
                outs.append((w[pos], w[pos + 1]))
                pos += 2
            ops.append({"kind": kind, "order": order, "out": (ob, ooff), "ins": ins, "count": cnt,
                        "outs": outs})
        rounds.append({"xfers": xfers, "ops": ops})
    return {"alg": w[0], "scratch_bytes": w[2], "rounds": rounds}


def prof_enable(on=True):
    lib().sosx_prof_enable(1 if on else 0)


def prof_get():
    f, x = ctypes.c_double(), ctypes.c_double()
    nf, nx, nc = ctypes.c_long(), ctypes.c_long(), ctypes.c_long()
    lib().sosx_prof_get(ctypes.byref(f), ctypes.byref(x), ctypes.byref(nf), ctypes.byref(nx),
                        ctypes.byref(nc))
    return {"fold_ms": f.value, "xfer_ms": x.value, "nfold": nf.value, "nxfer": nx.value,
            "ncall": nc.value}
