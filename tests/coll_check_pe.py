"""Multi-PE correctness run of the public scan and broadcast API (one process per PE).

Run under tools/oshrun: every PE calls shmemx_<T>_sum_{inscan,exscan},
shmem_<T>_broadcast, shmem_broadcastmem and the active-set shmem_broadcast32/64 on
device-heap buffers (shmemx_malloc_device), plain device buffers and host buffers, in
and out of place, over SHMEM_TEAM_WORLD and over an even-PE split team.  Scan results
are checked bit for bit against the CPU oracle's SOS scan_ring (oracle.scan,
src/collectives.c:1111-1209) over every member's input regenerated on the CPU;
broadcast results against the root's regenerated input, with the root's target
checked for SOS's copy / no-copy rule (src/collectives_c.c4:342-429).
Prints one line per PE, exit 0 = OK.

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

SCAN_TYPES = ["float", "double", "int", "char", "long", "complexd", "uint8"]
BCAST_TYPES = ["int", "double", "uint8", "longdouble", "size"]
SIZES = [1, 37, 5003, (1 << 20) + 3]
SENTINEL = 0x6B


def gen(dt, seed, pe, n, es):
    b = torch.empty(max(n * es, 1), dtype=torch.uint8, device="cuda")
    if n:
        L.fill(dt, L.DIST_UNIFORM, seed, pe, b.data_ptr(), n)
    return b


def upload(dst_ptr, t):
    torch.cuda.synchronize()
    L.check(L.lib().sosx_memcpy(dst_ptr, t.data_ptr(), t.numel(), None), "sosx_memcpy")


class Buffers:
    """Source/target pairs in the four residency modes."""

    def __init__(self, hsrc, hdst, nbytes, hh=None):
        self.hsrc, self.hdst, self.nbytes = hsrc, hdst, nbytes
        self.hh = hh  # (src, dst) in the host symmetric heap (shmem_malloc)

    def run(self, mode, src_dev, init_dst, call):
        """Place src (device tensor) and the target's initial bytes, call(dst, src),
        return the target's bytes as a host (numpy) copy, read back by tests/readback.py."""
        nb = self.nbytes
        if mode in ("heap", "heap_inplace"):
            upload(self.hsrc, src_dev[:nb])
            if mode == "heap":
                upload(self.hdst, init_dst[:nb])
                call(self.hdst, self.hsrc)
                return R.device_bytes(self.hdst, nb)
            call(self.hsrc, self.hsrc)
            return R.device_bytes(self.hsrc, nb)
        if mode == "hostheap":
            hs, hd = self.hh
            a_in = src_dev[:nb].cpu().numpy()      # kept alive across the memmoves
            a_init = init_dst[:nb].cpu().numpy()
            ctypes.memmove(hs, a_in.ctypes.data, nb)
            ctypes.memmove(hd, a_init.ctypes.data, nb)
            call(hd, hs)
            return np.ctypeslib.as_array((ctypes.c_uint8 * nb).from_address(hd)).copy()
        if mode == "device":
            s = src_dev[:nb].clone()
            d = init_dst[:nb].clone()
            torch.cuda.synchronize()
            call(d.data_ptr(), s.data_ptr())
            return R.device_bytes(d.data_ptr(), nb)
        h_in = src_dev[:nb].cpu().numpy().copy()
        h_out = init_dst[:nb].cpu().numpy().copy()
        call(h_out.ctypes.data, h_in.ctypes.data)
        return h_out


def main():
    S.shmem_init()
    me, P = S.shmem_my_pe(), S.shmem_n_pes()
    torch.cuda.set_device(S.lib().shmemx_get_device())
    world = S.team_world()
    bad, checks = [], 0
    maxb = max(SIZES) * 16
    hsrc = S.shmemx_malloc_device(maxb)
    hdst = S.shmemx_malloc_device(maxb)
    psync = S.shmem_malloc(8 * 4)
    ctypes.memset(psync, 0, 8 * 4)
    hh = (S.shmem_malloc(5003 * 16), S.shmem_malloc(5003 * 16))   # host symmetric heap
    S.shmem_barrier_all()
    even = ctypes.c_void_p(0)
    if P >= 3:
        S.lib().shmem_team_split_strided(world, 0, 2, (P + 1) // 2, None, 0, ctypes.byref(even))
    teams = [("world", world, list(range(P)))]
    if even.value:
        teams.append(("even", even.value, list(range(0, P, 2))))

    def check(ok, what):
        nonlocal checks
        checks += 1
        if not ok:
            bad.append(what)

    for tname, team, members in teams:
        if me not in members:
            continue
        idx = members.index(me)
        m = len(members)
        # ---- scans ------------------------------------------------------------------
        for ty in SCAN_TYPES:
            dt = L.dtype_id({"uint8": "int8"}.get(ty, ty))  # SOS binds uint8 to INT8
            es = L.dtype_size(dt)
            for n in SIZES:
                if n > 5003 and ty not in ("float", "int"):
                    continue
                for kind in ("inscan", "exscan"):
                    fn = getattr(S, f"shmemx_{ty}_sum_{kind}")
                    seed = zlib.crc32(f"{tname}/{ty}/{n}/{kind}".encode())
                    mine = gen(dt, seed, members[idx], n, es)
                    cpu_ins = [O.fill(dt, L.DIST_UNIFORM, seed, members[i], n) for i in range(m)]
                    ref = O.scan(L.op_id("sum"), dt, cpu_ins, kind == "exscan")[idx]
                    exp = R.as_bytes(ref)
                    zero = torch.zeros_like(mine)
                    for mode in ("heap", "heap_inplace", "device", "host", "hostheap"):
                        if mode in ("host", "hostheap") and n > 5003:
                            continue
                        got = Buffers(hsrc, hdst, n * es, hh).run(
                            mode, mine, zero, lambda d, s: fn(team, d, s, n))
                        mm = R.mismatches(exp, got, es)
                        check(mm == 0, (tname, kind, ty, n, mode, mm))
        # ---- typed / mem broadcasts -----------------------------------------------------
        for ty in BCAST_TYPES + ["mem"]:
            es = 1 if ty == "mem" else L.dtype_size(L.dtype_id(ty))
            fn = S.shmem_broadcastmem if ty == "mem" else getattr(S, f"shmem_{ty}_broadcast")
            for n in SIZES:
                if n > 5003 and ty not in ("int", "mem"):
                    continue
                for root in sorted({0, m - 1, m // 2}):
                    seed = zlib.crc32(f"{tname}/b/{ty}/{n}/{root}".encode())
                    src = gen(L.DTYPES["uchar"], seed, members[idx], n * es, 1)
                    rsrc = O.fill(L.DTYPES["uchar"], L.DIST_UNIFORM, seed, members[root], n * es)
                    init = torch.full_like(src, SENTINEL)
                    for mode in ("heap", "heap_inplace", "device", "host", "hostheap"):
                        if mode in ("host", "hostheap") and n > 5003:
                            continue
                        got = Buffers(hsrc, hdst, n * es, hh).run(
                            mode, src, init, lambda d, s: fn(team, d, s, n, root))
                        # every PE ends with the root's data (the root copies too)
                        mm = R.mismatches(rsrc, got, 1)
                        check(mm == 0, (tname, "bcast", ty, n, root, mode, mm))
    # ---- active-set broadcast32/64: the root's target is left untouched -------------------
    for bits_, fn in ((32, S.shmem_broadcast32), (64, S.shmem_broadcast64)):
        es = bits_ // 8
        for n in (1, 1001, 300001):
            for root in sorted({0, P - 1}):
                seed = zlib.crc32(f"as/{bits_}/{n}/{root}".encode())
                src = gen(L.DTYPES["uchar"], seed, me, n * es, 1)
                rsrc = O.fill(L.DTYPES["uchar"], L.DIST_UNIFORM, seed, root, n * es)
                init = torch.full_like(src, SENTINEL)
                for mode in ("heap", "device", "host", "hostheap"):
                    if mode in ("host", "hostheap") and n > 5003:
                        continue
                    got = Buffers(hsrc, hdst, n * es, hh).run(
                        mode, src, init, lambda d, s: fn(d, s, n, root, 0, 0, P, psync))
                    exp = np.full(n * es, SENTINEL, np.uint8) if me == root else rsrc
                    mm = R.mismatches(exp, got, 1)
                    check(mm == 0, ("active_set", bits_, n, root, mode, mm))
    S.shmem_barrier_all()
    S.shmemx_free_device(hdst)
    S.shmemx_free_device(hsrc)
    S.shmem_free(psync)
    S.shmem_free(hh[1])
    S.shmem_free(hh[0])
    if even.value:
        S.lib().shmem_team_destroy(even)
    sig = {1: "stream", 0: "host"}.get(L.lib().sosx_p2p_signal_mode(), "none")
    small_dev = L.lib().sosx_small_path_device_calls()
    S.shmem_finalize()
    if bad:
        print(f"PE {me}/{P}: {len(bad)} of {checks} checks FAILED: {bad[:6]}", flush=True)
        return 1
    print(f"PE {me}/{P}: {checks} checks OK (p2p signal {sig}, small-path device calls {small_dev})",
          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
