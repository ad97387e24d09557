"""Diagnostic: the copy pattern of striped_host_ring with raw HIP copies (ctypes on the
runtime torch loaded), P = 8 ring chunks: per stripe either P 1-D hipMemcpyAsync calls
(one per chunk slice) or ONE hipMemcpy2DAsync over the P slices (pitch = chunk length),
three device slots, H2D || add || D2H.  Compared with the serial H2D + add + D2H."""
import ctypes
import sys
import time

import torch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 512 << 20   # bytes
P = 8
torch.cuda.set_device(0)
hip = ctypes.CDLL("libamdhip64.so.7")  # already mapped by torch: same runtime
H2D, D2H = 1, 2
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                               ctypes.c_void_p]
hip.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                 ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
h_in = torch.ones(N // 4, dtype=torch.float32, pin_memory=True)
h_out = torch.empty(N // 4, dtype=torch.float32, pin_memory=True)
main = torch.cuda.current_stream()
s_h2d, s_d2h = torch.cuda.Stream(), torch.cuda.Stream()
q = N // P  # bytes per ring chunk


def serial():
    d = h_in.to("cuda", non_blocking=True)
    d += 1
    h_out.copy_(d, non_blocking=True)
    torch.cuda.synchronize()


def striped(K, two_d):
    L = q // K  # bytes per slice
    slots = [torch.empty(P * L // 4, dtype=torch.float32, device="cuda") for _ in range(3)]
    ev = [[torch.cuda.Event() for _ in range(3)] for _ in range(3)]  # [slot][h2d, x, d2h]
    for sl in range(3):
        ev[sl][2].record(s_d2h)

    def copy(dst, src, k, kind, stream, to_dev):
        if two_d:
            if to_dev:
                rc = hip.hipMemcpy2DAsync(dst, L, src + k * L, q, L, P, kind, stream)
            else:
                rc = hip.hipMemcpy2DAsync(dst + k * L, q, src, L, L, P, kind, stream)
            assert rc == 0, rc
        else:
            for c in range(P):
                if to_dev:
                    rc = hip.hipMemcpyAsync(dst + c * L, src + c * q + k * L, L, kind, stream)
                else:
                    rc = hip.hipMemcpyAsync(dst + c * q + k * L, src + c * L, L, kind, stream)
                assert rc == 0, rc

    def h2d(k):
        sl = k % 3
        s_h2d.wait_event(ev[sl][2])
        copy(slots[sl].data_ptr(), h_in.data_ptr(), k, H2D, s_h2d.cuda_stream, True)
        ev[sl][0].record(s_h2d)

    h2d(0)
    h2d(1)
    for k in range(K):
        if k + 2 < K:
            h2d(k + 2)
        sl = k % 3
        main.wait_event(ev[sl][0])
        slots[sl] += 1
        ev[sl][1].record(main)
        s_d2h.wait_event(ev[sl][1])
        copy(h_out.data_ptr(), slots[sl].data_ptr(), k, D2H, s_d2h.cuda_stream, False)
        ev[sl][2].record(s_d2h)
    torch.cuda.synchronize()


def timed(fn, reps=5):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


print(f"serial: {timed(serial) * 1e3:.3f} ms for {N >> 20} MiB", flush=True)
for K in (4, 8, 16):
    for two_d in (False, True):
        t = timed(lambda: striped(K, two_d))
        ok = torch.equal(h_out, h_in + 1)
        print(f"K={K:2d} {'2-D' if two_d else '1-D'} copies: {t * 1e3:.3f} ms"
              f" {'ok' if ok else 'MISMATCH'}", flush=True)
