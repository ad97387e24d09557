// fold.hip -- the fused P-way fold used by the team schedules (sosx_fold).
//
// A team reduction over P resident input vectors (own source + P-1 received partner
// chunks) is evaluated in ONE pass: (P+1)*n*s HBM bytes instead of 3*(P-1)*n*s for
// P-1 pairwise reduce_local calls.  Two element orders are available, each
// bit-identical to one SOS schedule:
//   LINEAR: acc = in[0]; acc = acc OP in[k]  -- the ring reduce-scatter fold
//           (src/collectives.c:693-727: partial = partial OP own source);
//   TREE  : the recdbl_sw butterfly (src/collectives.c:905-963).
// P <= 8 (one PE per GPU on one node) is a template parameter; 9..64 run a runtime-P
// element loop.
#include "fold_kernels.h"

namespace sos {

// Runtime P, element loads: teams of 9..64 PEs (several PEs per GPU or more than one
// node), and every fold whose inputs are small (latency-bound: one element per lane) or
// not 16-B congruent.  The TREE order walks the recdbl_sw leaves left to right with a
// binary-counter stack (merge equal-height neighbours: w[k] = w[k] OP w[k+d]), so no
// P-sized array; for P <= 8 it is fold_elem's tree, operation for operation (the extras
// first, then distance 1, 2, 4 pairs with the lower subtree the left operand).
template <class T, class OP, int ORDER>
__global__ __launch_bounds__(kThreads) void k_fold_dyn(T *out, FoldPtrs ins, int np,
                                                         size_t n)
{
    const size_t stride = (size_t)gridDim.x * kThreads;
    int p2 = 1;
    while (p2 * 2 <= np) p2 *= 2;
    if (np <= 8) {
        // one PE's node (the latency-bound small folds): every input's element is loaded
        // before the first combine, so the P loads are in flight together instead of one
        // round trip per input (fold_runtime_np_elem: the same operation order)
        FoldRealignArgs a;
#pragma unroll
        for (int k = 0; k < 8; ++k) a.p[k] = ins.p[k];
        a.np = np;
        for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
            out[i] = fold_runtime_np_elem<T, OP, ORDER>(a, i);
        return;
    }
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
        if constexpr (ORDER == SOSX_ORDER_LINEAR) {
            T acc = ((const T *)ins.p[0])[i];
            for (int k = 1; k < np; ++k) acc = OP::f(acc, ((const T *)ins.p[k])[i]);
            out[i] = acc;
        } else {
            T val[8];
            int height[8];
            int top = 0;
            for (int k = 0; k < p2; ++k) {
                T leaf = ((const T *)ins.p[k])[i];
                if (k < np - p2) leaf = OP::f(leaf, ((const T *)ins.p[k + p2])[i]);
                val[top] = leaf;
                height[top] = 0;
                ++top;
                while (top >= 2 && height[top - 1] == height[top - 2]) {
                    val[top - 2] = OP::f(val[top - 2], val[top - 1]);
                    height[top - 2]++;
                    --top;
                }
            }
            out[i] = val[0];
        }
    }
}

// ---------------------------------------------------------------------------------
// Fused prefix (the team scan's local step): outs[k] = ins[0] OP ... OP ins[k].
// P inputs, P outputs, one pass: 2*P*n*s HBM bytes.  P <= 8 (vector kernels and the
// element loop alike): every input of an element is loaded before the first store, so
// any output may alias any input.  Larger P: the one input that may alias an output
// (`own`, the PE's own source chunk under an in-place scan) is loaded before any store.
// ---------------------------------------------------------------------------------
template <class T, class OP>
__device__ __forceinline__ void prefix_elem_dyn(const PrefixPtrs &p, int np, int own, size_t i)
{
    if (np <= 8) {
        T v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = k < np ? ((const T *)p.in[k])[i] : T();
        T acc = v[0];
        ((T *)p.out[0])[i] = acc;
#pragma unroll
        for (int k = 1; k < 8; ++k)
            if (k < np) {
                acc = OP::f(acc, v[k]);
                ((T *)p.out[k])[i] = acc;
            }
        return;
    }
    const T ov = own >= 0 ? ((const T *)p.in[own])[i] : T();
    T acc = own == 0 ? ov : ((const T *)p.in[0])[i];
    ((T *)p.out[0])[i] = acc;
    for (int k = 1; k < np; ++k) {
        acc = OP::f(acc, k == own ? ov : ((const T *)p.in[k])[i]);
        ((T *)p.out[k])[i] = acc;
    }
}

// Runtime P (any P <= 64, or 16-B incongruent operands): element loads.
template <class T, class OP>
__global__ __launch_bounds__(kThreads) void k_prefix_dyn(PrefixPtrs p, int np, int own, size_t n)
{
    const size_t stride = (size_t)gridDim.x * kThreads;
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
        prefix_elem_dyn<T, OP>(p, np, own, i);
}

}  // namespace sos

using namespace sos;

namespace {

// Inputs of at most this many bytes each are folded one element per lane: the grid then
// has n/256 workgroups instead of n/(256*U*V), so a small fold whose inputs sit behind
// xGMI (the p2p transport's folds read peers in place) has many workgroups' loads in
// flight at once instead of one workgroup's; latency, not bandwidth, bounds these calls.
constexpr size_t kSpreadBytes = 64 * 1024;

// Occupancy cap of the multi-stream streaming kernels (round 5): a
// fold or prefix reads/writes `streams` concurrent HBM streams, and with every CU full
// (8 workgroups) the chip holds ~2048 tiles x streams open DRAM rows at once.  Reserving
// unused dynamic LDS caps the workgroups per CU (160 KiB / bytes): fewer rows open, better
// row-buffer locality.  Interleaved A/Bs over 9 random buffer layouts, twice
// (profiles/r5_multistream_ab.json): the 8-input fold (9 streams) 6.10-6.14 -> 6.29-6.35
// TB/s at 3 per CU; the 8-input prefix (16 streams) 5.75-5.87 -> 5.96-6.07 at 2 per CU;
// the 4- and 2-input prefixes (8, 4 streams) +2.5 / +1.7 % at 3 per CU.  The 3-stream
// combine loses with any cap (6.61 -> 6.31 TB/s at 3 per CU), so it has none, and neither
// do the folds of 2-4 inputs (U > 1 vectors per lane; unmeasured with a cap).
inline unsigned occupancy_lds(int streams)
{
    if (streams >= 12) return 64u << 10;  // 2 workgroups per CU
    if (streams >= 4) return 48u << 10;   // 3 per CU
    return 0;
}

template <class T, class OP, int ORDER>
int launch_fold_dyn(T *out, const FoldPtrs &ins, int np, size_t n, hipStream_t st)
{
    size_t blocks = (n + kThreads - 1) / kThreads;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL((k_fold_dyn<T, OP, ORDER>), dim3((unsigned)blocks), dim3(kThreads), 0, st, out, ins,
                       np, n);
    return hip_ok(hipGetLastError());
}

// Some inputs at another 16-B offset than the output (all element-aligned), either
// order: 16-B vectors, the incongruent inputs realigned in registers (fold_kernels.h).
template <class T, class OP, int ORDER>
int launch_fold_realign(T *out, const FoldPtrs &ins, int np, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), 1);
    FoldRealignArgs a;
    memset(&a, 0, sizeof(a));
    a.np = np;
    for (int k = 0; k < np; ++k) {
        a.p[k] = ins.p[k];
        a.d[k] = (unsigned)((uintptr_t)((const T *)ins.p[k] + g.head) & 15);
    }
    hipLaunchKernelGGL((k_fold_realign<T, OP, ORDER>), dim3(grid_for(g, kNoCap)), dim3(kThreads),
                       np >= 5 ? occupancy_lds(np + 1) : 0u, st, out, a, g);
    return hip_ok(hipGetLastError());
}

template <class T, class OP, int NP, int ORDER>
int launch_fold_np(T *out, const FoldPtrs &ins, size_t n, hipStream_t st)
{
    uintptr_t o = (uintptr_t)out;
    bool congruent = (o % sizeof(T)) == 0 && sizeof(T) <= 16;
    bool elem_aligned = congruent;
    for (int k = 0; k < NP; ++k) {
        congruent &= (((uintptr_t)ins.p[k] ^ o) & 15) == 0;
        elem_aligned &= ((uintptr_t)ins.p[k] % sizeof(T)) == 0;
    }
    // both orders: the LINEAR one is the ring's fold (SOS AUTO past the crossover,
    // src/shmem_collectives.h:192-199), the TREE one recdbl_sw's (AUTO below a raised
    // SHMEM_COLL_SIZE_CROSSOVER, or SHMEM_REDUCE_ALGORITHM=recdbl/linear/tree)
    if (!congruent && elem_aligned && n * sizeof(T) > kSpreadBytes)
        return launch_fold_realign<T, OP, ORDER>(out, ins, NP, n, st);
    if (!congruent || n * sizeof(T) <= kSpreadBytes) return launch_fold_dyn<T, OP, ORDER>(out, ins, NP, n, st);
    constexpr int U = NP <= 2 ? 4 : (NP <= 4 ? 2 : 1);
    Geom g = make_geom(o, n, sizeof(T), U);
    hipLaunchKernelGGL((k_fold<T, OP, NP, ORDER, U>), dim3(grid_for(g, kNoCap)), dim3(kThreads),
                       U == 1 ? occupancy_lds(NP + 1) : 0u, st, out, ins, g);
    return hip_ok(hipGetLastError());
}

template <class T, class OP, int ORDER>
int launch_fold(T *out, const FoldPtrs &ins, int nin, size_t n, hipStream_t st)
{
    switch (nin) {
        case 2: return launch_fold_np<T, OP, 2, ORDER>(out, ins, n, st);
        case 3: return launch_fold_np<T, OP, 3, ORDER>(out, ins, n, st);
        case 4: return launch_fold_np<T, OP, 4, ORDER>(out, ins, n, st);
        case 5: return launch_fold_np<T, OP, 5, ORDER>(out, ins, n, st);
        case 6: return launch_fold_np<T, OP, 6, ORDER>(out, ins, n, st);
        case 7: return launch_fold_np<T, OP, 7, ORDER>(out, ins, n, st);
        case 8: return launch_fold_np<T, OP, 8, ORDER>(out, ins, n, st);
        default: return launch_fold_dyn<T, OP, ORDER>(out, ins, nin, n, st);
    }
}

struct FoldFn {
    template <class T, class OP>
    static int run(int order, void *out, const FoldPtrs *ins, int nin, size_t n, hipStream_t st)
    {
        if (order == SOSX_ORDER_TREE) return launch_fold<T, OP, SOSX_ORDER_TREE>((T *)out, *ins, nin, n, st);
        return launch_fold<T, OP, SOSX_ORDER_LINEAR>((T *)out, *ins, nin, n, st);
    }
};

template <class T, class OP, int NP>
int launch_prefix_np(const PrefixPtrs &p, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)p.out[0], n, sizeof(T), kPrefixU);
    hipLaunchKernelGGL((k_prefix<T, OP, NP, kPrefixU, true>), dim3(grid_for(g, kNoCap)),
                       dim3(kThreads), occupancy_lds(2 * NP), st, p, g);
    return hip_ok(hipGetLastError());
}

struct PrefixFn {
    template <class T, class OP>
    static int run(const PrefixPtrs *p, int np, int own, size_t n, hipStream_t st)
    {
        const uintptr_t o = (uintptr_t)p->out[0];
        bool congruent = (o % sizeof(T)) == 0 && sizeof(T) <= 16;
        for (int k = 0; k < np; ++k)
            congruent &= (((uintptr_t)p->in[k] ^ o) & 15) == 0 && (((uintptr_t)p->out[k] ^ o) & 15) == 0;
        // the vector kernels serve the team scans, which are sums (shmemx_<T>_sum_inscan /
        // _exscan); other ops take the element loop (sosx_prefix accepts them all)
        if constexpr (std::is_same<OP, OpSum>::value) {
            if (!congruent && np <= 8 && sizeof(T) <= 16 && (o % sizeof(T)) == 0) {
                // outputs congruent, some inputs at other 16-B offsets (element-aligned):
                // 16-B vectors, the inputs realigned in registers
                bool outs_ok = true;
                for (int k = 0; k < np; ++k)
                    outs_ok &= (((uintptr_t)p->out[k] ^ o) & 15) == 0 && ((uintptr_t)p->in[k] % sizeof(T)) == 0;
                if (outs_ok) {
                    Geom g = make_geom(o, n, sizeof(T), 1);
                    PrefixRealignArgs a;
                    memset(&a, 0, sizeof(a));
                    a.np = np;
                    for (int k = 0; k < np; ++k) {
                        a.in[k] = p->in[k];
                        a.out[k] = p->out[k];
                        a.d[k] = (unsigned)((uintptr_t)((const T *)p->in[k] + g.head) & 15);
                    }
                    hipLaunchKernelGGL((k_prefix_realign<T, OP>), dim3(grid_for(g, kNoCap)), dim3(kThreads),
                                       occupancy_lds(2 * np), st, a, g);
                    return hip_ok(hipGetLastError());
                }
            }
            if (congruent) {
                switch (np) {
                    case 1: return launch_prefix_np<T, OP, 1>(*p, n, st);
                    case 2: return launch_prefix_np<T, OP, 2>(*p, n, st);
                    case 3: return launch_prefix_np<T, OP, 3>(*p, n, st);
                    case 4: return launch_prefix_np<T, OP, 4>(*p, n, st);
                    case 5: return launch_prefix_np<T, OP, 5>(*p, n, st);
                    case 6: return launch_prefix_np<T, OP, 6>(*p, n, st);
                    case 7: return launch_prefix_np<T, OP, 7>(*p, n, st);
                    case 8: return launch_prefix_np<T, OP, 8>(*p, n, st);
                    default: break;
                }
            }
        }
        size_t blocks = (n + kThreads - 1) / kThreads;
        if (blocks > 8192) blocks = 8192;
        hipLaunchKernelGGL((k_prefix_dyn<T, OP>), dim3((unsigned)blocks), dim3(kThreads), 0, st, *p,
                           np, own, n);
        return hip_ok(hipGetLastError());
    }
};

}  // namespace

extern "C" {

// outs[k] = ins[0] OP ins[1] OP ... OP ins[k] (left operand the running prefix), k < np,
// np <= 64.  `own` (or -1) names the one input that may alias an output when np > 8.
int sosx_prefix(int op, int dtype, void *const *outs, const void *const *ins, int np, int own,
                size_t count, void *stream)
{
    if (np < 1 || np > kMaxPrefix || own >= np) return SOSX_ERR_ARG;
    int rc = sos_check_op(op, dtype);
    if (rc) return rc;
    if (count == 0) return SOSX_OK;
    if (!outs || !ins) return SOSX_ERR_ARG;
    PrefixPtrs pp;
    memset(&pp, 0, sizeof(pp));
    for (int k = 0; k < np; ++k) {
        if (!outs[k] || !ins[k]) return SOSX_ERR_ARG;
        pp.in[k] = ins[k];
        pp.out[k] = outs[k];
    }
    return dispatch<PrefixFn>(op, dtype, &pp, np, own, count, as_stream(stream));
}

int sosx_fold(int op, int dtype, int order, void *out, const void *const *ins, int nin,
              size_t count, void *stream)
{
    if (nin < 1 || nin > SOSX_MAX_FOLD || (order != SOSX_ORDER_LINEAR && order != SOSX_ORDER_TREE))
        return SOSX_ERR_ARG;
    int rc = sos_check_op(op, dtype);
    if (rc) return rc;
    if (count == 0) return SOSX_OK;
    if (!out) return SOSX_ERR_ARG;
    for (int k = 0; k < nin; ++k)
        if (!ins[k]) return SOSX_ERR_ARG;
    const size_t bytes = count * sos_dtype_info(dtype).size;
    if (nin == 1) {
        if (out == ins[0]) return SOSX_OK;
        return hip_ok(hipMemcpyAsync(out, ins[0], bytes, hipMemcpyDeviceToDevice, as_stream(stream)));
    }
    FoldPtrs fp;
    memset(&fp, 0, sizeof(fp));
    for (int k = 0; k < nin; ++k) fp.p[k] = ins[k];
    return dispatch<FoldFn>(op, dtype, order, out, &fp, nin, count, as_stream(stream));
}

}  // extern "C"
