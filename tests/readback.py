"""Readback for the multi-process GPU checkers (team_check_pe.py, coll_check_pe.py).

A checker compares a PE's result with the CPU oracle's bytes ON THE CPU: the device
result comes back through ONE plain D2H copy into pinned host memory (hipMemcpy from
libamdhip64 itself, no release or fence of the test's own in front of it: what a user's
hipMemcpy or torch .cpu() after the call does), so the suite verifies that the library's
own completion release (sync_system, runtime.h) put the call's stores in HBM.
Host results are compared where they lie.
The expected bytes are never uploaded.  Round 4's checkers uploaded the expected vector
through a pageable torch H2D copy and counted mismatches with a kernel: a path whose
DMA writes and kernel reads were themselves a source of stale bytes under 12-process
queue time-slicing, so a stale read there was indistinguishable
from a wrong result.

Test infrastructure only.
"""
import ctypes

import numpy as np
import torch

from sos_amd import _lib as L

_PINNED = {}
_HIP = None
_D2H = 2  # hipMemcpyDeviceToHost


def _hip_memcpy():
    """hipMemcpy of the HIP runtime libsos_amd.so runs on (dlsym through the library's
    handle searches its dependencies: no second runtime is loaded)."""
    global _HIP
    if _HIP is None:
        f = L.lib().hipMemcpy
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _HIP = f
    return _HIP


def device_bytes(ptr, nbytes):
    """A host copy (numpy uint8) of `nbytes` of device memory at `ptr`."""
    if nbytes == 0:
        return np.empty(0, np.uint8)
    t = _PINNED.get(nbytes)
    if t is None:
        if len(_PINNED) > 8:
            _PINNED.clear()
        t = _PINNED[nbytes] = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    rc = _hip_memcpy()(t.data_ptr(), ptr, nbytes, _D2H)
    assert rc == 0, f"hipMemcpy D2H failed ({rc})"
    return t.numpy().copy()


def as_bytes(a):
    return np.frombuffer(np.ascontiguousarray(a).tobytes(), np.uint8)


def mismatches(exp, got, es):
    """Elements (es bytes each) whose bytes differ; exp/got: arrays of any dtype."""
    e, g = as_bytes(exp), as_bytes(got)
    assert e.size == g.size, (e.size, g.size)
    if es == 0 or e.size == 0:
        return 0
    return int(np.count_nonzero((e.reshape(-1, es) != g.reshape(-1, es)).any(axis=1)))


def diff_runs(exp, got, es, k=4):
    """The differing elements as [first, last) runs (at most k) and the run count."""
    e, g = as_bytes(exp).reshape(-1, es), as_bytes(got).reshape(-1, es)
    diff = np.nonzero((e != g).any(axis=1))[0]
    if diff.size == 0:
        return []
    cuts = np.nonzero(np.diff(diff) != 1)[0]
    starts = np.concatenate(([diff[0]], diff[cuts + 1]))
    ends = np.concatenate((diff[cuts], [diff[-1]])) + 1
    return [(int(a), int(b)) for a, b in zip(starts[:k], ends[:k])] + [f"{starts.size} runs"]
