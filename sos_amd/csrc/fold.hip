// fold.hip -- the fused P-way fold used by the team schedules (sosx_fold) and the fused
// prefix of the team scans (sosx_prefix).
//
// A team reduction over P resident input vectors (own source + P-1 received partner
// chunks) is evaluated in ONE pass: (P+1)*n*s HBM bytes instead of 3*(P-1)*n*s for
// P-1 pairwise reduce_local calls.  The fold's kernels and launchers live in
// fold_order.hip, built once per element order (LINEAR: the ring; TREE: recdbl_sw).
#include "fold_kernels.h"

namespace sos {

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
__global__ __launch_bounds__(kThreads) void k_prefix_dyn(PrefixPtrs p, int np, int own, size_t n, int acquire)
{
    if (acquire) wg_acquire();  // a small grid reading a peer's bytes (carry_acquire)
    const size_t stride = (size_t)gridDim.x * kThreads;
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
        prefix_elem_dyn<T, OP>(p, np, own, i);
}

}  // namespace sos

using namespace sos;

namespace {

// Bench switch for the one-offset case (all bit-exact): unset, the unaligned-load form
// for 4- and 8-byte elements at P = 1 and P >= 5, k_prefix_outshift otherwise; =1
// k_prefix_outshift always, =0 k_prefix_realign_np (DPP or UL by the incongruent count).
// P x 16Mi fp32 at +4 / +8 (profiles/r6_outshift_ab.txt): UL 6.14-6.24 / 5.75-5.81 TB/s at
// P = 1 / 8 against outshift's 5.82-5.99 / 5.37-5.40; at P = 2 / 3 the two tie, at P = 4
// outshift leads (5.94-6.01 against 5.79-5.85).  Neither prefix shape takes the occupancy
// cap: it measured neutral (k_prefix_realign_np: -1..+0 %).
inline int prefix_outshift_mode()
{
    static const int m = [] {
        const char *e = getenv("SOSX_PREFIX_OUTSHIFT");
        return e && *e ? atoi(e) : -1;
    }();
    return m;
}

template <class T, class OP, int NP>
int launch_prefix_np(const PrefixPtrs &p, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)p.out[0], n, sizeof(T), kPrefixU);
    g.acquire = carry_acquire(st, grid_for(g, kNoCap));
    if (g.acquire < 0) return SOSX_ERR_HIP;
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
                    bool same = true;
                    int m = 0;  // incongruent inputs
                    for (int k = 0; k < np; ++k) {
                        same &= a.d[k] == a.d[0];
                        m += a.d[k] != 0;
                    }
                    constexpr bool kUL = sizeof(T) == 4 || sizeof(T) == 8;
                    const bool one_offset = same && a.d[0] != 0;
                    const int om = prefix_outshift_mode();
                    const bool ul_one = kUL && (np == 1 || np >= 5);  // the one-offset auto choice
                    const bool outshift = one_offset && (om > 0 || (om < 0 && !ul_one));
                    const bool ul = kUL && !outshift && (m >= realign_unaligned_min() || (one_offset && om < 0));
                    g.acquire = carry_acquire(st, grid_for(g, kNoCap));
                    if (g.acquire < 0) return SOSX_ERR_HIP;
                    switch (np) {
#define SOSX_PREFIX_RA(P)                                                                                  \
    case P:                                                                                                \
        if (outshift)                                                                                      \
            hipLaunchKernelGGL((k_prefix_outshift<T, OP, P>), dim3(grid_for(g, kNoCap)), dim3(kThreads), 0u, \
                               st, a, g);                                                                  \
        else if (ul)                                                                                       \
            hipLaunchKernelGGL((k_prefix_realign_np<T, OP, P, kUL>), dim3(grid_for(g, kNoCap)), dim3(kThreads), \
                               0u, st, a, g);                                                              \
        else                                                                                               \
            hipLaunchKernelGGL((k_prefix_realign_np<T, OP, P>), dim3(grid_for(g, kNoCap)), dim3(kThreads), \
                               0u, st, a, g);                                                              \
        break;
                        SOSX_PREFIX_RA(1) SOSX_PREFIX_RA(2) SOSX_PREFIX_RA(3) SOSX_PREFIX_RA(4)
                        SOSX_PREFIX_RA(5) SOSX_PREFIX_RA(6) SOSX_PREFIX_RA(7) SOSX_PREFIX_RA(8)
#undef SOSX_PREFIX_RA
                    }
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
        const int acq = carry_acquire(st, (unsigned)blocks);
        if (acq < 0) return SOSX_ERR_HIP;
        hipLaunchKernelGGL((k_prefix_dyn<T, OP>), dim3((unsigned)blocks), dim3(kThreads), 0, st, *p,
                           np, own, n, acq);
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
        if (carry_acquire(as_stream(stream), 0, false) < 0) return SOSX_ERR_HIP;  // a library copy
        return hip_ok(hipMemcpyAsync(out, ins[0], bytes, hipMemcpyDeviceToDevice, as_stream(stream)));
    }
    FoldPtrs fp;
    memset(&fp, 0, sizeof(fp));
    for (int k = 0; k < nin; ++k) fp.p[k] = ins[k];
    return order == SOSX_ORDER_TREE ? fold_tree(op, dtype, out, &fp, nin, count, as_stream(stream))
                                    : fold_linear(op, dtype, out, &fp, nin, count, as_stream(stream));
}

}  // extern "C"
