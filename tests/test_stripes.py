"""CPU: the stripe decomposition of host-resident ring reductions is bit-exact.

striped_host_ring (sos_amd/csrc/collectives.cpp) runs SOS's ring over "stripes": stripe k
takes the k-th slice [k*L, k*L + L_k) of EVERY ring chunk (src/collectives.c:697-709),
and the n mod P extra elements of chunks c < r form a last stripe of r elements.  Each
stripe runs as an ordinary ring over its own elements.  Here the oracle checks the claim
behind it: scattering the stripes' ring results back gives, bit for bit, the ring over
the whole vector on every PE -- fp sum/prod and complex prod included, where any other
regrouping would change the bits.
"""
import numpy as np
import pytest

from oracle import oracle as O


def ring_chunk(n, P, c):
    q, r = divmod(n, P)
    cnt = q + (c < r)
    return cnt, (c * cnt if c < r else c * cnt + r)


def striped_ring(op, dt, srcs, L):
    P, n = len(srcs), srcs[0].size
    q, r = divmod(n, P)
    outs = [np.zeros_like(a) for a in srcs]
    disp = [ring_chunk(n, P, c)[1] for c in range(P)]
    stripes = [(k * L, min(L, q - k * L), P) for k in range((q + L - 1) // L)]
    if r:
        stripes.append((q, 1, r))
    for first, ln, npieces in stripes:
        idx = np.concatenate([np.arange(disp[c] + first, disp[c] + first + ln)
                              for c in range(npieces)])
        res = O.ring(op, dt, [np.ascontiguousarray(a[idx]) for a in srcs])
        for p in range(P):
            outs[p][idx] = res[p]
    return outs


@pytest.mark.parametrize("dt,op", [(23, 5), (24, 6), (27, 6), (26, 5), (4, 4), (11, 2)])
@pytest.mark.parametrize("P", [2, 3, 5, 8])
@pytest.mark.parametrize("n,L", [(1000, 37), (4099, 100), (8 * 300 + 7, 300), (65536 + 5, 4096)])
def test_stripes_equal_full_ring(dt, op, P, n, L):
    dist = 1 if op == 6 else 0
    srcs = [O.fill(dt, dist, n + P, p, n) for p in range(P)]
    full = O.ring(op, dt, srcs)
    got = striped_ring(op, dt, srcs, L)
    for p in range(P):
        assert got[p].tobytes() == full[p].tobytes(), (p, n, L)


def test_whole_vector_regrouping_would_differ():
    """Control: splitting the vector into contiguous halves (the naive pipeline) does
    change fp sum bits, so the stripe shape above is what keeps the ring's order."""
    P, n = 8, 1 << 14
    srcs = [O.fill(23, 0, 3, p, n) for p in range(P)]
    full = O.ring(5, 23, srcs)
    halves = [O.ring(5, 23, [np.ascontiguousarray(a[s]) for a in srcs])
              for s in (slice(0, n // 2), slice(n // 2, n))]
    naive = np.concatenate([halves[0][0], halves[1][0]])
    assert naive.tobytes() != full[0].tobytes()
