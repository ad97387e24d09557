"""ctypes binding of libsos_amd.so (the MI355X SOS reduction library).

The product path is native: C/C++/HIP in ``sos_amd/csrc`` compiled into
``sos_amd/libsos_amd.so``.  This module only declares the C ABI (include/sosx.h,
include/shmem.h, include/shmemx.h) for Python callers.  There is no Python or CPU
fallback: if the library is missing, :func:`lib` raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsos_amd.so")
# Test hook: SOSX_LIBRARY names another build of the same library to load instead, e.g.
# tests/fakerccl/libsos_amd_fakerccl.so, whose RCCL calls are bound to a file-based
# stand-in so the RCCL executor can run with several PEs on one GPU (tests/test_gpu_fakerccl.py).

# shm_internal_op_t (src/transport_none.h:25-33)
OPS = {"and": 0, "or": 1, "xor": 2, "min": 3, "max": 4, "sum": 5, "prod": 6}

# shm_internal_datatype_t (src/transport.h:19-49)
DTYPES = {
    "signed_byte": 0, "char": 1, "schar": 2, "short": 3, "int": 4, "long": 5,
    "longlong": 6, "fortran_integer": 7, "int8": 8, "int16": 9, "int32": 10,
    "int64": 11, "ptrdiff": 12, "uchar": 13, "ushort": 14, "uint": 15, "ulong": 16,
    "ulonglong": 17, "uint8": 18, "uint16": 19, "uint32": 20, "uint64": 21,
    "size": 22, "float": 23, "double": 24, "longdouble": 25, "complexf": 26,
    "complexd": 27,
}

ORDER_LINEAR, ORDER_TREE = 0, 1
ALGS = {"auto": 0, "recdbl": 1, "ring": 2, "rechalving": 3, "recdbl_direct": 4, "recdbl_gather": 5,
        "inscan": 16, "exscan": 17}
PLAN_INSCAN, PLAN_EXSCAN = 16, 17


def plan_bcast(root, copy_root):
    """Plan id of a broadcast from team index `root` (include/sosx.h SOSX_PLAN_BCAST)."""
    return 32 + 2 * int(root) + (1 if copy_root else 0)
DIST_UNIFORM, DIST_PROD = 0, 1

ERRORS = {
    -1: "invalid data type",
    -2: "unsupported reduction for this data type",
    -3: "invalid argument",
    -4: "HIP runtime error",
    -5: "RCCL error",
    -6: "not supported on the device path",
    -7: "library state error",
}


class SosError(RuntimeError):
    """A non-zero status from the C ABI."""

    def __init__(self, rc, what):
        super().__init__(f"{what}: {ERRORS.get(rc, 'error')} (status {rc})")
        self.rc = rc


_LIB = None

_c = ctypes
_SIGS = {
    "sosx_dtype_size": (_c.c_size_t, [_c.c_int]),
    "sosx_check_op": (_c.c_int, [_c.c_int, _c.c_int]),
    "sosx_combine": (_c.c_int, [_c.c_int, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_void_p]),
    "sosx_combine3": (_c.c_int, [_c.c_int, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                 _c.c_size_t, _c.c_void_p]),
    "sosx_fold": (_c.c_int, [_c.c_int, _c.c_int, _c.c_int, _c.c_void_p,
                             _c.POINTER(_c.c_void_p), _c.c_int, _c.c_size_t, _c.c_void_p]),
    "sosx_prefix": (_c.c_int, [_c.c_int, _c.c_int, _c.POINTER(_c.c_void_p), _c.POINTER(_c.c_void_p),
                               _c.c_int, _c.c_int, _c.c_size_t, _c.c_void_p]),
    "sosx_small_fold": (_c.c_int, [_c.c_int, _c.c_int, _c.c_void_p, _c.POINTER(_c.c_void_p),
                                   _c.POINTER(_c.c_void_p), _c.c_int, _c.c_size_t, _c.c_void_p,
                                   _c.c_uint32, _c.POINTER(_c.c_int), _c.c_void_p]),
    "sosx_small_ring": (_c.c_int, [_c.c_int, _c.c_int, _c.c_void_p, _c.POINTER(_c.c_void_p), _c.c_int,
                                   _c.c_size_t, _c.c_void_p, _c.c_uint32, _c.POINTER(_c.c_int),
                                   _c.c_void_p]),
    "sosx_small_linear": (_c.c_int, [_c.c_int, _c.c_int, _c.c_void_p, _c.POINTER(_c.c_void_p), _c.c_int,
                                     _c.c_size_t, _c.c_void_p, _c.c_uint32, _c.POINTER(_c.c_int),
                                     _c.c_int, _c.c_void_p]),
    "sosx_fill": (_c.c_int, [_c.c_int, _c.c_int, _c.c_uint64, _c.c_int, _c.c_void_p,
                             _c.c_size_t, _c.c_size_t, _c.c_void_p]),
    "sosx_count_mismatch": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_size_t,
                                       _c.POINTER(_c.c_ulonglong), _c.c_void_p]),
    "sosx_memcpy": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_void_p]),
    "sosx_combine_host": (_c.c_int, [_c.c_int, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_size_t,
                                     _c.c_size_t]),
    "sosx_build_info": (_c.c_char_p, []),
    "sosx_small_path_calls": (_c.c_long, []),
    "sosx_small_path_device_calls": (_c.c_long, []),
    "sosx_small_stage": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_void_p, _c.c_void_p,
                                    _c.c_int, _c.c_void_p]),
    "sosx_set_small_device_bytes": (_c.c_size_t, [_c.c_size_t]),
    "sosx_p2p_signal_mode": (_c.c_int, []),
    "sosx_set_p2p_signal_mode": (_c.c_int, [_c.c_int]),
    "sosx_set_rccl_allgather": (_c.c_int, [_c.c_int]),
    "sosx_set_rccl_allreduce": (_c.c_int, [_c.c_int]),
    "sosx_rccl_comm_count": (_c.c_int, []),
    "sosx_release_workspaces": (_c.c_size_t, []),
    "sosx_sys_releases": (_c.c_long, []),
    "sosx_data_segment": (_c.c_size_t, [_c.POINTER(_c.c_void_p)]),
    "sosx_acquire_stats": (None, [_c.POINTER(_c.c_long), _c.POINTER(_c.c_long), _c.POINTER(_c.c_long),
                                  _c.POINTER(_c.c_uint)]),
    "sosx_acquire_kernels": (_c.c_long, []),
    "sosx_acquire_system": (_c.c_int, [_c.c_void_p, _c.c_void_p]),
    "sosx_gather": (_c.c_int, [_c.c_int, _c.POINTER(_c.c_void_p), _c.POINTER(_c.c_void_p),
                               _c.POINTER(_c.c_size_t), _c.c_void_p]),
}


_RUNTIME_LIBS = ("libamdhip64", "libhsa-runtime64", "librccl", "librocm_smi64")


def loaded_runtimes():
    """{runtime library stem: sorted distinct paths mapped into this process}."""
    found = {k: set() for k in _RUNTIME_LIBS}
    with open("/proc/self/maps") as f:
        for line in f:
            path = line.split()[-1]
            base = os.path.basename(path)
            for k in _RUNTIME_LIBS:
                if base.startswith(k + ".so"):
                    found[k].add(path)
    return {k: sorted(v) for k, v in found.items()}


def lib():
    """Load libsos_amd.so (once) and declare its C signatures.

    One HIP runtime per process: torch (when installed) is imported first, so the
    libamdhip64.so.7 / librccl.so.1 it has already mapped satisfy libsos_amd.so's
    DT_NEEDED entries by SONAME.  Loaded the other way round, the loader maps
    /opt/rocm's runtime for libsos_amd.so and torch then maps its own bundled copy
    (it asks for the unversioned names); the two librocm_smi64 copies then free one
    static object twice at exit ("double free or corruption").  A second copy that
    this load maps is refused here rather than left to abort at exit.  (A profiler may
    have preloaded its own HSA runtime before torch; that copy is not ours to refuse.)
    """
    global _LIB
    if _LIB is not None:
        return _LIB
    path = os.environ.get("SOSX_LIBRARY") or LIB_PATH
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback for the SOS reduction path)")
    try:
        import torch  # noqa: F401  (maps torch's HIP runtime before ours is resolved)
    except ImportError:
        pass
    before = loaded_runtimes()
    L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    added = {k: v for k, v in loaded_runtimes().items() if len(v) > max(1, len(before[k]))}
    if added:
        raise ImportError(f"loading {path} mapped a second copy of a ROCm runtime "
                          f"library: {added}")
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    _LIB = L
    return L


def check(rc, what):
    if rc != 0:
        raise SosError(rc, what)
    return rc


def dtype_id(name_or_id):
    return DTYPES[name_or_id] if isinstance(name_or_id, str) else int(name_or_id)


def op_id(name_or_id):
    return OPS[name_or_id] if isinstance(name_or_id, str) else int(name_or_id)


def combine(op, dtype, inout_ptr, in_ptr, count, stream=None):
    """inout = inout OP in on device memory (sosx_combine)."""
    return check(lib().sosx_combine(op_id(op), dtype_id(dtype), inout_ptr, in_ptr, count, stream),
                 "sosx_combine")


def combine3(op, dtype, out_ptr, a_ptr, b_ptr, count, stream=None):
    return check(lib().sosx_combine3(op_id(op), dtype_id(dtype), out_ptr, a_ptr, b_ptr, count,
                                     stream), "sosx_combine3")


def fold(op, dtype, order, out_ptr, in_ptrs, count, stream=None):
    arr = (ctypes.c_void_p * len(in_ptrs))(*in_ptrs)
    return check(lib().sosx_fold(op_id(op), dtype_id(dtype), order, out_ptr, arr, len(in_ptrs),
                                 count, stream), "sosx_fold")


def prefix(op, dtype, out_ptrs, in_ptrs, count, own=-1, stream=None):
    """outs[k] = ins[0] OP ... OP ins[k] on device memory (sosx_prefix)."""
    n = len(in_ptrs)
    outs = (ctypes.c_void_p * n)(*out_ptrs)
    ins = (ctypes.c_void_p * n)(*in_ptrs)
    return check(lib().sosx_prefix(op_id(op), dtype_id(dtype), outs, ins, n, own, count, stream),
                 "sosx_prefix")


def fill(dtype, dist, seed, pe, dst_ptr, count, index0=0, stream=None):
    return check(lib().sosx_fill(dtype_id(dtype), dist, seed, pe, dst_ptr, count, index0, stream),
                 "sosx_fill")


def count_mismatch(a_ptr, b_ptr, count, elem_size, stream=None):
    out = ctypes.c_ulonglong(0)
    check(lib().sosx_count_mismatch(a_ptr, b_ptr, count, elem_size, ctypes.byref(out), stream),
          "sosx_count_mismatch")
    return out.value


def dtype_size(dtype):
    return lib().sosx_dtype_size(dtype_id(dtype))
