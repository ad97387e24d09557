"""GPU parity at BASELINE.json's full sizes, bit for bit against
the CPU oracle (oracle/sos_oracle.c: shmem_internal_reduce_local,
src/shmem_internal_op.h:305-339, and the ring schedule, src/collectives.c:647-764).

  headline   float sum combine, nreduce = 128Mi
  config #2  double sum (shmem_double_sum_to_all's local combine), nreduce = 16Mi
  config #3  int64 and / or / xor, nreduce = 128Mi
  config #4  float sum over 8 PEs, nreduce = 64Mi (single-GPU loopback team: the same
             per-PE ring plan and fold kernels the RCCL executor runs)
  config #5  int / double / complexd x min / max / prod (complexd: prod, sum) at the
             sweep's largest size, nreduce = 256Mi, and through the team schedules at
             P = 2 / 4 / 8 for nreduce = 1Ki, 64Ki, 4Mi

Inputs are the SURVEY 8(d) synthetic streams, generated on the GPU (sosx_fill) and on the
host (oracle fill) -- test_fill_matches_oracle pins that the two are identical.
The fp tolerance of these configs is 0 ulp: the combine is element-wise with the same
operand order as the reference, so results are bit-identical.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED
Mi = 1 << 20


def dev_fill(torch, sos, dt, dist, pe, n):
    es = sos.dtype_size(dt)
    t = torch.empty(n * es, dtype=torch.uint8, device="cuda")
    sos.fill(dt, dist, SEED, pe, t.data_ptr(), n)
    return t


def combine_vs_oracle(torch, sos, oracle, dt, op, n):
    dist = 1 if op == 6 else 0
    da = dev_fill(torch, sos, dt, dist, 0, n)
    db = dev_fill(torch, sos, dt, dist, 1, n)
    sos.combine(op, dt, da.data_ptr(), db.data_ptr(), n)
    ref = oracle.fill(dt, dist, SEED, 0, n)
    oracle.reduce_local(op, dt, oracle.fill(dt, dist, SEED, 1, n), ref)
    torch.cuda.synchronize()
    got = da.cpu().numpy()
    del da, db
    bad = np.count_nonzero(got != np.frombuffer(ref.tobytes(), np.uint8))
    assert bad == 0, f"dt={dt} op={op} n={n}: {bad} bytes differ"


def test_headline_float_sum_128mi(torch_cuda, sos, oracle):
    combine_vs_oracle(torch_cuda, sos, oracle, 23, 5, 128 * Mi)


def test_config2_double_sum_16mi(torch_cuda, sos, oracle):
    combine_vs_oracle(torch_cuda, sos, oracle, 24, 5, 16 * Mi)


@pytest.mark.parametrize("op", [0, 1, 2])
def test_config3_int64_bitwise_128mi(torch_cuda, sos, oracle, op):
    combine_vs_oracle(torch_cuda, sos, oracle, 11, op, 128 * Mi)


@pytest.mark.parametrize("dt,op", [(4, 3), (4, 4), (4, 6), (24, 3), (24, 4), (24, 6),
                                   (27, 6), (27, 5)])
def test_config5_sweep_top_256mi(torch_cuda, sos, oracle, dt, op):
    combine_vs_oracle(torch_cuda, sos, oracle, dt, op, 256 * Mi)


def test_config4_float_sum_8pes_64mi(torch_cuda, sos, oracle):
    """8 PEs x 64Mi fp32 through the ring plan (SOS AUTO at this size), loopback on one GPU."""
    from sos_amd import shmem as S
    torch = torch_cuda
    P, n, dt, op = 8, 64 * Mi, 23, 5
    src = [dev_fill(torch, sos, dt, 0, p, n) for p in range(P)]
    dst = [torch.empty_like(t) for t in src]
    S.loopback_allreduce("ring", op, dt, [t.data_ptr() for t in src], [t.data_ptr() for t in dst],
                         n)
    torch.cuda.synchronize()
    del src
    ref = oracle.ring(op, dt, [oracle.fill(dt, 0, SEED, p, n) for p in range(P)])
    for p in range(P):
        got = dst[p].cpu().numpy()
        assert np.array_equal(got, np.frombuffer(ref[p].tobytes(), np.uint8)), p


@pytest.mark.parametrize("P,n", [(2, 1024), (2, 65536), (2, 4 * Mi), (4, 1024), (4, 65536), (4, 4 * Mi),
                                 (8, 1024), (8, 65536), (8, 4 * Mi)])
@pytest.mark.parametrize("dt,op", [(4, 3), (4, 4), (4, 6), (24, 3), (24, 4), (24, 6), (27, 6), (27, 5)])
def test_config5_sweep_team(torch_cuda, sos, oracle, P, n, dt, op):
    """Config #5 at P = 2/4/8: int / double / complexd x min / max / prod
    (complexd: prod, sum) through the schedule SOS AUTO picks at that size -- recdbl_sw
    below the 16 KiB crossover, the ring above it -- every PE bit for bit against the
    oracle's schedule over the CPU-regenerated inputs (loopback team on one GPU: the same
    per-PE plans and kernels the transports run)."""
    from sos_amd import shmem as S
    torch = torch_cuda
    dist = 1 if op == 6 else 0
    es = sos.dtype_size(dt)
    alg = "recdbl" if n * es < 16384 else "ring"
    src = [dev_fill(torch, sos, dt, dist, p, n) for p in range(P)]
    dst = [torch.empty_like(t) for t in src]
    S.loopback_allreduce(alg, op, dt, [t.data_ptr() for t in src], [t.data_ptr() for t in dst], n)
    torch.cuda.synchronize()
    del src
    ins = [oracle.fill(dt, dist, SEED, p, n) for p in range(P)]
    ref = oracle.ring(op, dt, ins) if alg == "ring" else oracle.recdbl(op, dt, ins)
    for p in range(P):
        got = dst[p].cpu().numpy()
        assert np.array_equal(got, np.frombuffer(ref[p].tobytes(), np.uint8)), (alg, p)
