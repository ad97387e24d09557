"""Probe: are a kernel's writes visible to a DMA read on ANOTHER stream right after the
kernel's stream was synchronised?  (the 12-PE wrong results.)

Per iteration: fill `a` and `b` with fresh seeds and combine a = a + b (sosx_combine,
nontemporal stores) on a non-blocking stream; then either hipStreamSynchronize(stream)
("stream-sync", what the library did before round 5) or record + synchronise an event
with a system-scope release ("sys-event", what it does now); then copy `a` to pageable
host memory with ONE hipMemcpy on the null stream (a DMA read) and compare it with the
CPU oracle.  A mismatch whose elements equal a's PREVIOUS contents means the combine's
writes were still in an XCD's L2 when the host was told the stream was done.

Run one process, or several at once under tools/oshrun (no shmem calls: each process
is independent; several processes time-slice the GPU's queues as the 12-PE tests do).
Diagnostic code: the oracle is the checker only.

Usage: python tools/visibility_probe.py [--iters 400] [--n 1048579] [--mode stream-sync|sys-event]
"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from sos_amd import _lib as L  # noqa: E402

HIP = ctypes.CDLL("libamdhip64.so.7")
HIP_EVENT_RELEASE_TO_SYSTEM = 0x80000000
HIP_EVENT_DISABLE_TIMING = 0x2


class IpcHandle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]   # hipIpcMemHandle_t, passed by value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--n", type=int, default=(1 << 20) + 3)
    ap.add_argument("--mode", default="stream-sync", choices=("stream-sync", "sys-event"))
    ap.add_argument("--exported", action="store_true",
                    help="`a` lives in a hipMalloc region exported with hipIpcGetMemHandle (as the "
                         "device symmetric heap), not in torch's allocator")
    ap.add_argument("--churn", action="store_true",
                    help="hipFree + hipMalloc of a 60 MiB buffer before every combine (the "
                         "exchange scratch's grow)")
    ap.add_argument("--peer-read", action="store_true",
                    help="with --shared: the combine's second operand is the NEXT process's "
                         "region (constant data it wrote before the loop), read in place")
    ap.add_argument("--shared", action="store_true",
                    help="with --exported: every process maps every other process's region "
                         "(hipIpcOpenMemHandle through files in /dev/shm), as the p2p heap is")
    a = ap.parse_args()
    me = int(os.environ.get("SHMEM_PE", "0"))
    torch.cuda.set_device(0)
    n = a.n
    dt, op = L.dtype_id("float"), L.op_id("sum")
    stream = torch.cuda.Stream()
    S = stream.cuda_stream
    ev = ctypes.c_void_p()
    assert HIP.hipEventCreateWithFlags(ctypes.byref(ev),
                                       HIP_EVENT_RELEASE_TO_SYSTEM | HIP_EVENT_DISABLE_TIMING) == 0
    if a.exported:
        region = ctypes.c_void_p()
        assert HIP.hipMalloc(ctypes.byref(region), ctypes.c_size_t(256 << 20)) == 0
        handle = IpcHandle()
        assert HIP.hipIpcGetMemHandle(ctypes.byref(handle), region) == 0
        a_ptr = region.value + (64 << 20)
        if a.shared:
            import time
            npes = int(os.environ["SHMEM_NPES"])
            tag = os.environ.get("VIS_TAG", "vis")
            path = f"/dev/shm/{tag}_{{}}"
            # constant data for the peers' in-place reads, written before the handle is shown
            L.fill(dt, 0, 0xBEEF, me, region.value + (128 << 20), n, 0, S)
            assert HIP.hipDeviceSynchronize() == 0
            with open(path.format(me) + ".tmp", "wb") as f:
                f.write(bytes(handle))
            os.rename(path.format(me) + ".tmp", path.format(me))
            peers = []
            for q in range(npes):
                if q == me:
                    continue
                t0 = time.time()
                while not os.path.exists(path.format(q)):
                    assert time.time() - t0 < 60
                    time.sleep(0.01)
                hq = IpcHandle.from_buffer_copy(open(path.format(q), "rb").read())
                pq = ctypes.c_void_p()
                assert HIP.hipIpcOpenMemHandle(ctypes.byref(pq), hq, ctypes.c_uint(1)) == 0
                peers.append((q, pq))
    else:
        ta = torch.empty(n * 4, dtype=torch.uint8, device="cuda")
        a_ptr = ta.data_ptr()
    churn = ctypes.c_void_p()
    b_src = None
    if a.peer_read:
        q, pq = next(x for x in peers if x[0] == (me + 1) % npes)
        b_src = (pq.value + (128 << 20), O.fill(dt, 0, 0xBEEF, q, n))
    tb = torch.empty(n * 4, dtype=torch.uint8, device="cuda")
    host = np.empty(n, np.float32)
    before = np.zeros(n, np.float32)
    bad = []
    for it in range(a.iters):
        seed = 0x700000 + 1000 * me + it
        if a.churn:
            if churn.value:
                assert HIP.hipStreamSynchronize(ctypes.c_void_p(S)) == 0
                assert HIP.hipFree(churn) == 0
            assert HIP.hipMalloc(ctypes.byref(churn), ctypes.c_size_t(60 << 20)) == 0
        L.fill(dt, 0, seed, 0, a_ptr, n, 0, S)
        if b_src is None:
            L.fill(dt, 0, seed, 1, tb.data_ptr(), n, 0, S)
            L.combine(op, dt, a_ptr, tb.data_ptr(), n, S)
        else:
            L.combine(op, dt, a_ptr, b_src[0], n, S)
        if a.mode == "stream-sync":
            assert HIP.hipStreamSynchronize(ctypes.c_void_p(S)) == 0
        else:
            assert HIP.hipEventRecord(ev, ctypes.c_void_p(S)) == 0
            assert HIP.hipEventSynchronize(ev) == 0
        L.check(L.lib().sosx_memcpy(host.ctypes.data, a_ptr, n * 4, None), "sosx_memcpy")
        exp = O.fill(dt, 0, seed, 0, n)
        O.reduce_local(op, dt, O.fill(dt, 0, seed, 1, n) if b_src is None else b_src[1], exp)
        diff = np.nonzero(host.view(np.uint32) != exp.view(np.uint32))[0]
        if diff.size:
            stale = int(np.count_nonzero(host[diff].view(np.uint32) == before[diff].view(np.uint32)))
            bad.append({"iter": it, "mismatches": int(diff.size), "equal_to_previous": stale})
        before = exp
        if me == 0 and it % 100 == 0:
            print(f"[visibility_probe] {a.mode} iteration {it}/{a.iters}", file=sys.stderr, flush=True)
    verdict = f"{len(bad)} of {a.iters} DMA reads stale" if bad else f"0 of {a.iters} DMA reads stale"
    opts = ",".join(k for k in ("exported", "shared", "peer_read", "churn") if getattr(a, k)) or "plain"
    print(f"PE {me}: {a.mode} ({opts}): {verdict} {bad[:4]}", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
