"""GPU: every kernel shape of the bench-only variant library (tools/variants/) computes
the same fp32 sum bits as the CPU oracle's reduce_local -- the combine shapes, the
8-input LINEAR fold shapes and the prefix shapes the product defaults were chosen
against.  Ragged heads and tails included, so the shapes' A/B
numbers compare like with like."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "variants"))

FLOAT, SUM = 23, 5


@pytest.fixture(scope="module")
def V(torch_cuda):
    import variants
    return variants


def _dev(torch, a, off):
    t = torch.zeros(a.nbytes + 64, dtype=torch.uint8, device="cuda")
    t[off:off + a.nbytes].copy_(torch.from_numpy(a.view(np.uint8)))
    return t, t.data_ptr() + off


def _host(t, off, like):
    return t[off:off + like.nbytes].cpu().numpy().view(like.dtype)


def test_every_combine_shape_bit_exact(torch_cuda, V, oracle):
    torch = torch_cuda
    n = (1 << 22) + 4099
    a, b = oracle.fill(FLOAT, 0, 77, 0, n), oracle.fill(FLOAT, 0, 77, 1, n)
    ref = a.copy()
    oracle.reduce_local(SUM, FLOAT, b, ref)
    for v, name in enumerate(V.names("combine")):
        for off in (0, 4):
            da, pa = _dev(torch, a, off)
            db, pb = _dev(torch, b, off)
            V.combine(v, pa, pa, pb, n)
            torch.cuda.synchronize()
            assert np.array_equal(_host(da, off, a).view(np.uint32), ref.view(np.uint32)), (name, off)


def test_every_fold_shape_bit_exact(torch_cuda, V, oracle):
    torch = torch_cuda
    n = (1 << 20) + 1029
    ins = [oracle.fill(FLOAT, 0, 91, k, n) for k in range(8)]
    ref = ins[0].copy()
    for k in range(1, 8):                    # the ring's LINEAR order: acc = acc OP in[k]
        oracle.reduce_local(SUM, FLOAT, ins[k], ref)
    for v, name in enumerate(V.names("fold")):
        for off in (0, 8):
            di = [_dev(torch, x, off) for x in ins]
            do, po = _dev(torch, np.zeros_like(ref), off)
            V.fold(v, po, [p for _, p in di], n)
            torch.cuda.synchronize()
            assert np.array_equal(_host(do, off, ref).view(np.uint32), ref.view(np.uint32)), (name, off)


@pytest.mark.parametrize("np_", [2, 5, 8])
def test_every_prefix_shape_bit_exact(torch_cuda, V, oracle, np_):
    torch = torch_cuda
    n = (1 << 18) + 1029
    ins = [oracle.fill(FLOAT, 0, 55, k, n) for k in range(np_)]
    refs, acc = [], ins[0].copy()
    refs.append(acc.copy())
    for k in range(1, np_):                  # running prefix is the left operand
        oracle.reduce_local(SUM, FLOAT, ins[k], acc)
        refs.append(acc.copy())
    for v, name in enumerate(V.names("prefix")):
        di = [_dev(torch, x, 4) for x in ins]
        do = [_dev(torch, np.zeros_like(x), 4) for x in ins]
        V.prefix(v, [p for _, p in do], [p for _, p in di], n)
        torch.cuda.synchronize()
        for k in range(np_):
            got = _host(do[k][0], 4, refs[k])
            assert np.array_equal(got.view(np.uint32), refs[k].view(np.uint32)), (name, k)
