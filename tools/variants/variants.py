"""ctypes binding of the BENCH-ONLY kernel-shape library tools/variants/libsos_variants.so
(tools/variants/variants.hip): the combine / fold / prefix shapes the product defaults
were chosen against, fp32 sum.  Used by tools/variants_bench.py, tools/loopback_bench.py
(--fold-ab / --prefix-ab) and the tests that check every shape computes the same bits.
The product library never loads it."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsos_variants.so")
_L = None


def lib():
    global _L
    if _L is None:
        import torch  # noqa: F401  (one HIP runtime per process: torch's, mapped first)
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is not built (make -C sos_amd/csrc)")
        L = ctypes.CDLL(LIB_PATH)
        c = ctypes
        vp, sz, i = c.c_void_p, c.c_size_t, c.c_int
        for k in ("combine", "fold", "prefix"):
            getattr(L, f"sosxv_num_{k}").restype = i
            getattr(L, f"sosxv_{k}_name").restype = c.c_char_p
            getattr(L, f"sosxv_{k}_name").argtypes = [i]
        L.sosxv_combine.argtypes = [i, vp, vp, vp, sz, vp]
        L.sosxv_fold.argtypes = [i, vp, c.POINTER(vp), sz, vp]
        L.sosxv_prefix.argtypes = [i, c.POINTER(vp), c.POINTER(vp), i, sz, vp]
        for f in (L.sosxv_combine, L.sosxv_fold, L.sosxv_prefix):
            f.restype = i
        _L = L
    return _L


def names(kind):
    L = lib()
    return [getattr(L, f"sosxv_{kind}_name")(v).decode()
            for v in range(getattr(L, f"sosxv_num_{kind}")())]


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: status {rc}")


def combine(v, out, a, b, n, stream=None):
    _check(lib().sosxv_combine(v, out, a, b, n, stream), "sosxv_combine")


def fold(v, out, ins, n, stream=None):
    arr = (ctypes.c_void_p * 8)(*ins)
    _check(lib().sosxv_fold(v, out, arr, n, stream), "sosxv_fold")


def prefix(v, outs, ins, n, stream=None):
    k = len(ins)
    o = (ctypes.c_void_p * k)(*outs)
    i = (ctypes.c_void_p * k)(*ins)
    _check(lib().sosxv_prefix(v, o, i, k, n, stream), "sosxv_prefix")
