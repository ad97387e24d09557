"""GPU: the combine on every pair of special fp values, bit for bit against the oracle
(x86 gcc -O2, SOS's reduce_local, src/shmem_internal_op.h:23-43).

Specials: quiet NaNs of both signs with and without payloads, a signalling-pattern NaN,
+-0, +-inf, 1, -2.5, a denormal and the largest finite value -- every ordered pair, so
the ternary min/max tie rules (second operand on ties, not fmin/fmax), x86's
first-operand NaN rule for sum/prod and the default NaN of an invalid operation are all
exercised.  Complex sum: bit-exact.  Complex prod: bit-exact wherever the x86 result is
not a NaN; where it is, the device result is a NaN too (payload and sign follow the
device).  (Was tools/nan_probe.py, a printing probe, through
round 2.)
"""
import numpy as np
import pytest

from oracle import oracle as O
from sos_amd import _lib as L

pytestmark = pytest.mark.gpu


def specials(ft):
    it = np.uint32 if ft == np.float32 else np.uint64
    bits = [0x7FC00000, 0xFFC00000, 0x7FC00123, 0x7F800001, 0xFF800123] if ft == np.float32 else \
        [0x7FF8000000000000, 0xFFF8000000000000, 0x7FF8000000000123, 0x7FF0000000000001,
         0xFFF0000000000123]
    nans = list(np.array(bits, dtype=it).view(ft))
    vals = [0.0, -0.0, np.inf, -np.inf, 1.0, -2.5, np.finfo(ft).tiny / 4, np.finfo(ft).max]
    return np.array(nans + [ft(v) for v in vals], dtype=ft)


def run(torch, dt, op, a, b):
    ref = a.copy()
    O.reduce_local(op, dt, b, ref)
    da = torch.from_numpy(a.view(np.uint8).copy()).cuda()
    db = torch.from_numpy(b.view(np.uint8).copy()).cuda()
    L.combine(op, dt, da.data_ptr(), db.data_ptr(), a.size)
    torch.cuda.synchronize()
    return da.cpu().numpy().view(a.dtype), ref


FTYPES = [(np.float32, 23, 26), (np.float64, 24, 27)]


@pytest.mark.parametrize("ft,dt,cdt", FTYPES)
@pytest.mark.parametrize("op", [3, 4, 5, 6])
def test_real_specials_bit_exact(torch_cuda, ft, dt, cdt, op):
    s = specials(ft)
    A, B = np.meshgrid(s, s, indexing="ij")
    a, b = A.reshape(-1).copy(), B.reshape(-1).copy()
    ib = np.uint32 if ft == np.float32 else np.uint64
    got, ref = run(torch_cuda, dt, op, a, b)
    bad = np.nonzero(got.view(ib) != ref.view(ib))[0]
    assert bad.size == 0, [(hex(a.view(ib)[k]), hex(b.view(ib)[k]), hex(got.view(ib)[k]),
                            hex(ref.view(ib)[k])) for k in bad[:6]]


@pytest.mark.parametrize("ft,dt,cdt", FTYPES)
@pytest.mark.parametrize("op", [5, 6])
def test_complex_specials(torch_cuda, ft, dt, cdt, op):
    s = specials(ft)
    sc = s[[0, 1, 2, 5, 6, 7, 9, 10]]
    grid = np.array(np.meshgrid(sc, sc, sc, sc, indexing="ij")).reshape(4, -1).T.copy()
    ca = grid[:, :2].copy().reshape(-1).view(O.np_type(cdt))
    cb = grid[:, 2:].copy().reshape(-1).view(O.np_type(cdt))
    ib = np.uint32 if ft == np.float32 else np.uint64
    got, ref = run(torch_cuda, cdt, op, ca, cb)
    gb, rb = got.view(ib).reshape(-1, 2), ref.view(ib).reshape(-1, 2)
    gf, rf = got.view(ft).reshape(-1, 2), ref.view(ft).reshape(-1, 2)
    if op == 5:
        bad = np.nonzero((gb != rb).any(1))[0]
    else:
        ref_nan = np.isnan(rf).any(1)
        bad = np.nonzero(((gb != rb).any(1) & ~ref_nan) | (ref_nan & ~np.isnan(gf).any(1)))[0]
    assert bad.size == 0, [(gb[k].tolist(), rb[k].tolist()) for k in bad[:6]]
