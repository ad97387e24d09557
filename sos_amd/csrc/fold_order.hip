// fold_order.hip -- the fused P-way fold's launchers and kernels for ONE element order,
// compiled twice (Makefile: -DSOSX_FOLD_ORDER=0 -> fold_linear.o, =1 -> fold_tree.o) so
// the two halves of the (type, op, P) instantiations build in parallel.  sosx_fold
// (fold.hip) picks the order:
//   LINEAR: acc = in[0]; acc = acc OP in[k]  -- the ring reduce-scatter fold
//           (src/collectives.c:693-727: partial = partial OP own source);
//   TREE  : the recdbl_sw butterfly (src/collectives.c:905-963).
// P <= 8 (one PE per GPU on one node) is a template parameter; 9..64 run a runtime-P
// element loop.
#include "fold_kernels.h"

#ifndef SOSX_FOLD_ORDER
#error "build with -DSOSX_FOLD_ORDER=0 (LINEAR) or 1 (TREE)"
#endif

namespace sos {

// Runtime P, element loads: teams of 9..64 PEs (several PEs per GPU or more than one
// node), and every fold whose inputs are small (latency-bound: one element per lane) or
// not 16-B congruent.  The TREE order walks the recdbl_sw leaves left to right with a
// binary-counter stack (merge equal-height neighbours: w[k] = w[k] OP w[k+d]), so no
// P-sized array; for P <= 8 it is fold_elem's tree, operation for operation (the extras
// first, then distance 1, 2, 4 pairs with the lower subtree the left operand).
template <class T, class OP, int ORDER>
__global__ __launch_bounds__(kThreads) void k_fold_dyn(T *out, FoldPtrs ins, int np,
                                                         size_t n, int acquire)
{
    if (acquire) wg_acquire();  // a small grid reading a peer's bytes (carry_acquire)
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

}  // namespace sos

using namespace sos;

namespace {

// Inputs of at most this many bytes each are folded one element per lane: the grid then
// has n/256 workgroups instead of n/(256*U*V), so a small fold whose inputs sit behind
// xGMI (the p2p transport's folds read peers in place) has many workgroups' loads in
// flight at once instead of one workgroup's; latency, not bandwidth, bounds these calls.
constexpr size_t kSpreadBytes = 64 * 1024;

// Bench switch for the one-offset case (every input at the same 16-B offset d != 0; every
// choice is bit-exact, only speed differs).  Unset: the unaligned-load form for 4- and
// 8-byte elements, k_fold_outshift for the others; =1 k_fold_outshift for every type, =2
// the same under the multi-stream occupancy cap, =0 k_fold_realign_np (DPP or UL by the
// incongruent count).  P x 16Mi fp32 at +4 / +8 (profiles/r6_outshift_ab.txt): the UL
// form 6.52-6.63 / 6.50-6.57 / 6.13-6.28 / 6.06-6.10 TB/s at P = 2 / 3 / 4 / 8 against
// outshift's 6.34-6.41 / 6.37-6.41 / 6.11-6.21 / 5.88-6.08.  Round 5 (r5_fold_outshift.txt):
// outshift 5.79-6.17 beat the cap (5.21-5.59) and the two-load realign (4.16-4.44).
inline int outshift_mode()
{
    static const int m = [] {
        const char *e = getenv("SOSX_FOLD_OUTSHIFT");
        return e && *e ? atoi(e) : -1;
    }();
    return m;
}

template <class T, class OP, int ORDER>
int launch_fold_dyn(T *out, const FoldPtrs &ins, int np, size_t n, hipStream_t st)
{
    size_t blocks = (n + kThreads - 1) / kThreads;
    if (blocks > 8192) blocks = 8192;
    const int acq = carry_acquire(st, (unsigned)blocks);
    if (acq < 0) return SOSX_ERR_HIP;
    hipLaunchKernelGGL((k_fold_dyn<T, OP, ORDER>), dim3((unsigned)blocks), dim3(kThreads), 0, st, out, ins,
                       np, n, acq);
    return hip_ok(hipGetLastError());
}

// Some inputs at another 16-B offset than the output (all element-aligned), either
// order: 16-B vectors (fold_kernels.h), loaded unaligned (4- and 8-byte elements, every
// input at one offset or at least realign_unaligned_min() inputs incongruent) or
// realigned in registers (the output when every input sits at one offset, else each
// incongruent input).  No occupancy cap (the shapes lost with it: r5_fold_outshift.txt).
template <class T, class OP, int NP, int ORDER>
int launch_fold_realign(T *out, const FoldPtrs &ins, size_t n, hipStream_t st)
{
    constexpr int np = NP;
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), 1);
    FoldRealignArgs a;
    memset(&a, 0, sizeof(a));
    a.np = np;
    bool same = true;  // every input at one offset: realign the output instead
    int m = 0;         // incongruent inputs
    for (int k = 0; k < np; ++k) {
        a.p[k] = ins.p[k];
        a.d[k] = (unsigned)((uintptr_t)((const T *)ins.p[k] + g.head) & 15);
        same &= a.d[k] == a.d[0];
        m += a.d[k] != 0;
    }
    const unsigned lds = np >= 5 ? occupancy_lds(np + 1) : 0u;  // the bench A/B only
    g.acquire = carry_acquire(st, grid_for(g, kNoCap));
    if (g.acquire < 0) return SOSX_ERR_HIP;
    constexpr bool kUL = sizeof(T) == 4 || sizeof(T) == 8;
    const bool one_offset = same && a.d[0] != 0;
    const int om = outshift_mode();
    if (one_offset && (om > 0 || (om < 0 && !kUL)))
        hipLaunchKernelGGL((k_fold_outshift<T, OP, NP, ORDER>), dim3(grid_for(g, kNoCap)), dim3(kThreads),
                           om == 2 ? lds : 0u, st, out, a, g);
    else if (kUL && (m >= realign_unaligned_min() || (one_offset && om < 0)))
        hipLaunchKernelGGL((k_fold_realign_np<T, OP, NP, ORDER, kUL>),
                           dim3(grid_for(g, kNoCap)), dim3(kThreads), 0u, st, out, a, g);
    else
        hipLaunchKernelGGL((k_fold_realign_np<T, OP, NP, ORDER>), dim3(grid_for(g, kNoCap)), dim3(kThreads), 0u,
                           st, out, a, g);
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
    // (16-B elements that are element-aligned are always congruent: no realigning kernels)
    if constexpr (sizeof(T) < 16)
        if (!congruent && elem_aligned && n * sizeof(T) > kSpreadBytes)
            return launch_fold_realign<T, OP, NP, ORDER>(out, ins, n, st);
    if (!congruent || n * sizeof(T) <= kSpreadBytes) return launch_fold_dyn<T, OP, ORDER>(out, ins, NP, n, st);
    constexpr int U = NP <= 2 ? 4 : (NP <= 4 ? 2 : 1);
    Geom g = make_geom(o, n, sizeof(T), U);
    g.acquire = carry_acquire(st, grid_for(g, kNoCap));
    if (g.acquire < 0) return SOSX_ERR_HIP;
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

struct FoldOrderFn {
    template <class T, class OP>
    static int run(void *out, const FoldPtrs *ins, int nin, size_t n, hipStream_t st)
    {
        return launch_fold<T, OP, SOSX_FOLD_ORDER>((T *)out, *ins, nin, n, st);
    }
};

}  // namespace

namespace sos {

#if SOSX_FOLD_ORDER == SOSX_ORDER_TREE
int fold_tree(int op, int dtype, void *out, const FoldPtrs *ins, int nin, size_t n, hipStream_t st)
#else
int fold_linear(int op, int dtype, void *out, const FoldPtrs *ins, int nin, size_t n, hipStream_t st)
#endif
{
    return dispatch<FoldOrderFn>(op, dtype, out, ins, nin, n, st);
}

}  // namespace sos
