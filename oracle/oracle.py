"""ctypes wrapper of the CPU oracle (oracle/sos_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker (or the timed CPU baseline), never by the
product package sos_amd/.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libsos_oracle.so")

# numpy view of each shm_internal_datatype_t's C type (x86-64 LP64; `char` is signed).
NP_TYPES = {
    1: np.int8, 2: np.int8, 3: np.int16, 4: np.int32, 5: np.int64, 6: np.int64,
    8: np.int8, 9: np.int16, 10: np.int32, 11: np.int64, 12: np.int64, 13: np.uint8,
    14: np.uint16, 15: np.uint32, 16: np.uint64, 17: np.uint64, 18: np.uint8,
    19: np.uint16, 20: np.uint32, 21: np.uint64, 22: np.uint64, 23: np.float32,
    24: np.float64, 25: np.longdouble, 26: np.complex64, 27: np.complex128,
}

_L = None


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            import subprocess
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.oracle_reduce_local.argtypes = [i, i, i, vp, vp]
        L.oracle_reduce_local.restype = i
        L.oracle_type_size.argtypes = [i]
        L.oracle_type_size.restype = sz
        L.oracle_ring.argtypes = [i, sz, i, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.oracle_ring.restype = i
        L.oracle_recdbl.argtypes = [i, sz, i, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.oracle_recdbl.restype = i
        L.oracle_scan.argtypes = [i, sz, i, i, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.oracle_scan.restype = i
        L.oracle_bcast.argtypes = [i, sz, i, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.oracle_bcast.restype = i
        L.oracle_fill.argtypes = [i, i, ctypes.c_uint64, i, vp, sz, sz]
        L.oracle_fill.restype = i
        L.oracle_time_reduce_local.argtypes = [i, i, i, vp, vp, i]
        L.oracle_time_reduce_local.restype = ctypes.c_double
        L.oracle_pe_header_bytes.argtypes = [i]
        L.oracle_pe_header_bytes.restype = sz
        L.oracle_pe_barrier.argtypes = [vp, i, ctypes.c_long]
        L.oracle_pe_barrier.restype = None
        L.oracle_pe_ring.argtypes = [vp, sz, i, i, sz, i, i, vp]
        L.oracle_pe_ring.restype = i
        L.oracle_pe_ring_time.argtypes = [vp, sz, i, i, sz, i, i, vp, i,
                                          ctypes.POINTER(ctypes.c_long)]
        L.oracle_pe_ring_time.restype = ctypes.c_double
        L.oracle_pe_recdbl.argtypes = [vp, sz, i, i, sz, i, i, vp]
        L.oracle_pe_recdbl.restype = i
        L.oracle_pe_time.argtypes = [i, vp, sz, i, i, sz, i, i, vp, i,
                                     ctypes.POINTER(ctypes.c_long)]
        L.oracle_pe_time.restype = ctypes.c_double
        _L = L
    return _L


def np_type(dt):
    return NP_TYPES[dt]


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def reduce_local(op, dt, inp, inout):
    """inout = inout OP inp, in place (shmem_internal_reduce_local)."""
    assert inp.shape == inout.shape
    rc = lib().oracle_reduce_local(op, dt, inout.size, _ptr(inp), _ptr(inout))
    if rc:
        raise ValueError(f"oracle_reduce_local rc={rc}")
    return inout


def fill(dt, dist, seed, pe, count, index0=0):
    a = np.empty(count, dtype=np_type(dt))
    rc = lib().oracle_fill(dt, dist, seed, pe, _ptr(a), count, index0)
    if rc:
        raise ValueError(f"oracle_fill rc={rc}")
    return a


def _team(fn, op, dt, srcs, dsts):
    P = len(srcs)
    s = (ctypes.c_void_p * P)(*[a.ctypes.data for a in srcs])
    d = (ctypes.c_void_p * P)(*[a.ctypes.data for a in dsts])
    rc = fn(P, srcs[0].size, op, dt, s, d)
    if rc:
        raise ValueError(f"oracle team rc={rc}")
    return dsts


def ring(op, dt, srcs, dsts=None):
    """SOS ring all-reduce (src/collectives.c:647-764) over P simulated PEs."""
    if dsts is None:
        dsts = [np.zeros_like(a) for a in srcs]
    return _team(lib().oracle_ring, op, dt, srcs, dsts)


def recdbl(op, dt, srcs, dsts=None):
    """SOS recursive doubling (src/collectives.c:850-984) over P simulated PEs."""
    if dsts is None:
        dsts = [np.zeros_like(a) for a in srcs]
    return _team(lib().oracle_recdbl, op, dt, srcs, dsts)


def scan(op, dt, srcs, exclusive, dsts=None):
    """SOS team prefix scan (src/collectives.c:1111-1209) over P simulated PEs."""
    if dsts is None:
        dsts = [np.zeros_like(a) for a in srcs]
    P = len(srcs)
    s = (ctypes.c_void_p * P)(*[a.ctypes.data for a in srcs])
    d = (ctypes.c_void_p * P)(*[a.ctypes.data for a in dsts])
    rc = lib().oracle_scan(P, srcs[0].size, op, dt, 1 if exclusive else 0, s, d)
    if rc:
        raise ValueError(f"oracle_scan rc={rc}")
    return dsts


def bcast(srcs, root, copy_root, dsts):
    """SOS broadcast (src/collectives.c:429-485) over P simulated PEs, in place on dsts."""
    P = len(srcs)
    s = (ctypes.c_void_p * P)(*[a.ctypes.data for a in srcs])
    d = (ctypes.c_void_p * P)(*[a.ctypes.data for a in dsts])
    rc = lib().oracle_bcast(P, srcs[0].nbytes, root, 1 if copy_root else 0, s, d)
    if rc:
        raise ValueError(f"oracle_bcast rc={rc}")
    return dsts


def time_reduce_local(op, dt, inp, inout, reps):
    return lib().oracle_time_reduce_local(op, dt, inout.size, _ptr(inp), _ptr(inout), reps)


class PeRing:
    """One PE of SOS's ring (alg "ring", oracle_pe_ring: the N > 1 CPU baseline) or
    recdbl_sw (alg "recdbl", oracle_pe_recdbl: the small-message latency comparison) run
    by a real process.  Every PE process maps the same shared segment `path` (PE 0
    creates it before the others open it; the caller provides that ordering) holding
    every PE's pSync words and target; the source stays private to the process."""

    ALGS = {"ring": 0, "recdbl": 1}

    def __init__(self, path, P, me, count, dt, create, alg="ring"):
        import mmap
        self.P, self.me, self.count, self.dt = P, me, count, dt
        self.alg = self.ALGS[alg]
        ts = lib().oracle_type_size(dt)
        self.stride = (count * ts + 4095) & ~4095
        self.hdr = lib().oracle_pe_header_bytes(P)
        size = self.hdr + P * self.stride
        fd = os.open(path, os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0), 0o600)
        try:
            if create:
                # reserve the pages now: a tmpfs that runs out later raises SIGBUS on touch
                os.posix_fallocate(fd, 0, size)
            self.mm = mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        self._anchor = ctypes.c_char.from_buffer(self.mm)
        self.base = ctypes.addressof(self._anchor)
        self.epoch = ctypes.c_long(0)

    def target(self):
        """This PE's target as a numpy view (valid while the segment is mapped)."""
        a = np.frombuffer(self.mm, dtype=np.uint8, count=self.count * lib().oracle_type_size(self.dt),
                          offset=self.hdr + self.me * self.stride)
        return a.view(NP_TYPES[self.dt])

    def barrier(self):
        self.epoch.value += 1
        lib().oracle_pe_barrier(self.base, self.P, self.epoch.value)

    def run(self, op, src):
        fn = lib().oracle_pe_recdbl if self.alg == 1 else lib().oracle_pe_ring
        rc = fn(self.base, self.stride, self.P, self.me, self.count, op, self.dt, _ptr(src))
        if rc:
            raise ValueError(f"oracle_pe_{'recdbl' if self.alg else 'ring'} rc={rc}")

    def time(self, op, src, reps):
        t = lib().oracle_pe_time(self.alg, self.base, self.stride, self.P, self.me, self.count,
                                 op, self.dt, _ptr(src), reps, ctypes.byref(self.epoch))
        if t < 0:
            raise ValueError("oracle_pe_time failed")
        return t

    def close(self):
        del self._anchor
        self.mm.close()
