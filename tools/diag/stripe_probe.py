"""Diagnostic: the stream/event pattern of striped_host_ring, in one process, on torch.

A host buffer of N bytes (pinned) goes H2D -> (on-device add) -> D2H in K stripes through
three device slots: H2D(k+2) on one copy stream || compute(k) on the main stream ||
D2H(k-1) on another copy stream.  Prints ms per pass against the serial schedule.
"""
import sys
import time

import torch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
torch.cuda.set_device(0)
h_in = torch.ones(N // 4, dtype=torch.float32, pin_memory=True)
h_out = torch.empty(N // 4, dtype=torch.float32, pin_memory=True)
main = torch.cuda.current_stream()
s_h2d, s_d2h = torch.cuda.Stream(), torch.cuda.Stream()


def serial():
    d = h_in.to("cuda", non_blocking=True)
    d += 1
    h_out.copy_(d, non_blocking=True)
    torch.cuda.synchronize()


def striped(K, pieces=1, fresh=False):
    m = N // 4 // K
    slots = [torch.empty(m, dtype=torch.float32, device="cuda") for _ in range(3)]
    ne = K + 3 if fresh else 3  # fresh: one event per stripe (none re-recorded in flight)
    ev_h2d = [torch.cuda.Event() for _ in range(ne)]
    ev_x = [torch.cuda.Event() for _ in range(ne)]
    ev_d2h = [torch.cuda.Event() for _ in range(ne)]
    for e in ev_d2h:
        e.record(s_d2h)

    def ix(k):
        return k if fresh else k % 3

    def h2d(k):
        sl = k % 3
        s_h2d.wait_event(ev_d2h[ix(k - 3) if k >= 3 else ix(k)])
        with torch.cuda.stream(s_h2d):
            w = m // pieces
            for j in range(pieces):
                slots[sl][j * w:(j + 1) * w].copy_(h_in[k * m + j * w:k * m + (j + 1) * w],
                                                   non_blocking=True)
        ev_h2d[ix(k)].record(s_h2d)

    h2d(0)
    h2d(1)
    for k in range(K):
        if k + 2 < K:
            h2d(k + 2)
        sl = k % 3
        main.wait_event(ev_h2d[ix(k)])
        slots[sl] += 1
        ev_x[ix(k)].record(main)
        s_d2h.wait_event(ev_x[ix(k)])
        with torch.cuda.stream(s_d2h):
            w = m // pieces
            for j in range(pieces):
                h_out[k * m + j * w:k * m + (j + 1) * w].copy_(slots[sl][j * w:(j + 1) * w],
                                                               non_blocking=True)
        ev_d2h[ix(k)].record(s_d2h)
    torch.cuda.synchronize()


def timed(fn, reps=10):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


print(f"serial: {timed(serial) * 1e3:.3f} ms for {N >> 20} MiB", flush=True)
for K in (4, 8, 16, 32, 64):
    for fresh in (False, True):
        print(f"striped K={K} fresh_events={fresh}: "
              f"{timed(lambda: striped(K, 8, fresh)) * 1e3:.3f} ms", flush=True)
ok = torch.equal(h_out, h_in + 1)
print("result ok" if ok else "RESULT MISMATCH", flush=True)
