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
#include "elementwise.h"

namespace sos {

// ---------------------------------------------------------------------------------
// Fused P-way fold, P = NP known at compile time (one PE per GPU: P <= 8).
// ---------------------------------------------------------------------------------
struct FoldPtrs {
    const void *p[SOSX_MAX_FOLD];
};

// recdbl_sw tree, evaluated from the perspective of the lowest PE of every subtree:
// extras first (v[k] = v[k] OP v[k+pow2], src/collectives.c:920-926), then distance
// 1, 2, 4, ... pairs (src/collectives.c:932-963).  Own value is always the left
// operand, which makes the result bit-identical to recdbl_sw for commutative
// element semantics (all integer ops, fp sum/prod without NaN payload choices).
template <int NP> struct Pow2Floor {
    static constexpr int v = NP >= 8 ? 8 : NP >= 4 ? 4 : NP >= 2 ? 2 : 1;
};

template <class T, class OP, int NP, int ORDER>
__device__ __forceinline__ T fold_elem(const T (&v)[NP])
{
    if constexpr (ORDER == SOSX_ORDER_LINEAR) {
        T acc = v[0];
#pragma unroll
        for (int k = 1; k < NP; ++k) acc = OP::f(acc, v[k]);
        return acc;
    } else {
        constexpr int P2 = Pow2Floor<NP>::v;
        T w[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) w[k] = v[k];
#pragma unroll
        for (int k = 0; k < NP - P2; ++k) w[k] = OP::f(w[k], w[k + P2]);
#pragma unroll
        for (int d = 1; d < P2; d <<= 1)
#pragma unroll
            for (int k = 0; k < P2; k += 2 * d) w[k] = OP::f(w[k], w[k + d]);
        return w[0];
    }
}

template <class T, class OP, int NP, int ORDER>
__device__ __forceinline__ u32x4 fold_pack(const u32x4 (&x)[NP])
{
    Pack<T> p[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) p[k] = __builtin_bit_cast(Pack<T>, x[k]);
    Pack<T> r;
#pragma unroll
    for (int j = 0; j < Pack<T>::N; ++j) {
        T v[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) v[k] = p[k].e[j];
        r.e[j] = fold_elem<T, OP, NP, ORDER>(v);
    }
    return __builtin_bit_cast(u32x4, r);
}

template <class T, class OP, int NP, int ORDER, int U>
__global__ __launch_bounds__(kThreads) void k_fold(T *out, FoldPtrs ins, Geom g)
{
    constexpr int V = Pack<T>::N;
    u32x4 *O = reinterpret_cast<u32x4 *>(out + g.head);
    for (size_t t = blockIdx.x; t < g.tiles; t += gridDim.x) {
        const size_t base = t * (size_t)(kThreads * U) + threadIdx.x;
        u32x4 x[U][NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const u32x4 *I = reinterpret_cast<const u32x4 *>((const T *)ins.p[k] + g.head);
#pragma unroll
            for (int u = 0; u < U; ++u) x[u][k] = ldv<true>(I + base + u * kThreads);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) stv<true>(O + base + u * kThreads, fold_pack<T, OP, NP, ORDER>(x[u]));
    }
    if (g.has_rem && blockIdx.x == gridDim.x - 1) {
        auto one = [&](size_t i) {
            T v[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) v[k] = ((const T *)ins.p[k])[i];
            out[i] = fold_elem<T, OP, NP, ORDER>(v);
        };
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) one(i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * U * V) + threadIdx.x; i < g.n;
             i += kThreads)
            one(i);
    }
}

// Tuning variants of k_fold (bench A/B, sosx_set_fold_variant): each workgroup takes S
// consecutive tiles (longer contiguous runs per input stream), optionally loading tile
// j+1 before storing tile j (PF), optionally with an XCD-contiguous tile order
// (workgroup w runs on XCD w % 8).  Same element order as k_fold.
template <class T, class OP, int NP, int ORDER, int S, bool PF, bool XCD>
__global__ __launch_bounds__(kThreads) void k_fold_st(T *out, FoldPtrs ins, Geom g, size_t groups)
{
    constexpr int V = Pack<T>::N;
    u32x4 *O = reinterpret_cast<u32x4 *>(out + g.head);
    size_t grp = blockIdx.x;
    if (XCD && groups % 8 == 0 && grp < groups) grp = (grp % 8) * (groups / 8) + grp / 8;
    if (grp < groups) {
        const size_t t0 = grp * S;
        const size_t t1 = t0 + S < g.tiles ? t0 + S : g.tiles;
        u32x4 x[NP];
        auto load = [&](size_t t, u32x4 (&d)[NP]) {
            const size_t i = t * (size_t)kThreads + threadIdx.x;
#pragma unroll
            for (int k = 0; k < NP; ++k)
                d[k] = ldv<true>(reinterpret_cast<const u32x4 *>((const T *)ins.p[k] + g.head) + i);
        };
        if (PF) {
            load(t0, x);
            for (size_t t = t0; t < t1; ++t) {
                u32x4 y[NP];
                if (t + 1 < t1) load(t + 1, y);
                stv<true>(O + t * (size_t)kThreads + threadIdx.x, fold_pack<T, OP, NP, ORDER>(x));
#pragma unroll
                for (int k = 0; k < NP; ++k) x[k] = y[k];
            }
        } else {
            for (size_t t = t0; t < t1; ++t) {
                load(t, x);
                stv<true>(O + t * (size_t)kThreads + threadIdx.x, fold_pack<T, OP, NP, ORDER>(x));
            }
        }
    }
    if (g.has_rem && blockIdx.x == gridDim.x - 1) {
        auto one = [&](size_t i) {
            T v[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) v[k] = ((const T *)ins.p[k])[i];
            out[i] = fold_elem<T, OP, NP, ORDER>(v);
        };
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) one(i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            one(i);
    }
}

template <class T, class OP, int NP, int ORDER>
__global__ __launch_bounds__(kThreads) void k_fold_scalar(T *out, FoldPtrs ins,
                                                            size_t n)
{
    const size_t stride = (size_t)gridDim.x * kThreads;
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
        T v[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) v[k] = ((const T *)ins.p[k])[i];
        out[i] = fold_elem<T, OP, NP, ORDER>(v);
    }
}

// Runtime P (9..64 PEs per team: several PEs per GPU or more than one node): element
// loads; the TREE order walks the recdbl_sw leaves left to right with a binary-counter
// stack (merge equal-height neighbours: w[k] = w[k] OP w[k+d]), so no P-sized array.
template <class T, class OP, int ORDER>
__global__ __launch_bounds__(kThreads) void k_fold_dyn(T *out, FoldPtrs ins, int np,
                                                         size_t n)
{
    const size_t stride = (size_t)gridDim.x * kThreads;
    int p2 = 1;
    while (p2 * 2 <= np) p2 *= 2;
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
// P inputs, P outputs, one pass: 2*P*n*s HBM bytes.  NP <= 8: every input of a vector
// is loaded before the first store (any output may alias any input).  Larger P: a
// runtime loop; the one input that may alias an output (`own`, the PE's own source
// chunk under an in-place scan) is loaded before any store.
// ---------------------------------------------------------------------------------
constexpr int kMaxPrefix = 64;

struct PrefixPtrs {
    const void *in[kMaxPrefix];
    void *out[kMaxPrefix];
};

// 16-B vectors per lane per tile.  U = 2/4/8 and plain loads/stores measured slower over
// random buffer layouts (profiles/r2_prefix_variants*.txt); they stay as
// bench variants (sosx_set_prefix_variant).
constexpr int kPrefixU = 1;

// NT: nontemporal loads/stores (the default); the plain variant is a bench A/B only.
template <class T, class OP, int NP, int U, bool NT = true>
__global__ __launch_bounds__(kThreads) void k_prefix(PrefixPtrs p, Geom g)
{
    constexpr int V = Pack<T>::N;
    for (size_t t = blockIdx.x; t < g.tiles; t += gridDim.x) {
        const size_t base = t * (size_t)(kThreads * U) + threadIdx.x;
        u32x4 x[U][NP];
#pragma unroll
        for (int k = 0; k < NP; ++k)
#pragma unroll
            for (int u = 0; u < U; ++u)
                x[u][k] = ldv<NT>(reinterpret_cast<const u32x4 *>((const T *)p.in[k] + g.head) + base + u * kThreads);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + u * kThreads;
            u32x4 acc = x[u][0];
            stv<NT>(reinterpret_cast<u32x4 *>((T *)p.out[0] + g.head) + i, acc);
#pragma unroll
            for (int k = 1; k < NP; ++k) {
                acc = apply<T, OP>(acc, x[u][k]);
                stv<NT>(reinterpret_cast<u32x4 *>((T *)p.out[k] + g.head) + i, acc);
            }
        }
    }
    if (g.has_rem && blockIdx.x == gridDim.x - 1) {
        auto one = [&](size_t i) {
            T v[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) v[k] = ((const T *)p.in[k])[i];
            T acc = v[0];
            ((T *)p.out[0])[i] = acc;
#pragma unroll
            for (int k = 1; k < NP; ++k) {
                acc = OP::f(acc, v[k]);
                ((T *)p.out[k])[i] = acc;
            }
        };
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) one(i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * U * V) + threadIdx.x; i < g.n; i += kThreads)
            one(i);
    }
}

template <class T, class OP>
__device__ __forceinline__ void prefix_elem_dyn(const PrefixPtrs &p, int np, int own, size_t i)
{
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

int g_fold_variant = 0;  // tuning experiments on the 8-input fp32 sum fold (bench A/B)
int g_prefix_variant = 0;  // same for the fp32 sum prefix, 2..8 inputs

template <class T, class OP, int NP, int ORDER, int U>
int launch_fold_u(T *out, const FoldPtrs &ins, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), U);
    hipLaunchKernelGGL((k_fold<T, OP, NP, ORDER, U>), dim3(grid_for(g, kNoCap)), dim3(kThreads),
                       0, st, out, ins, g);
    return hip_ok(hipGetLastError());
}

template <class T, class OP, int NP, int ORDER, int S, bool PF, bool XCD>
int launch_fold_st(T *out, const FoldPtrs &ins, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), 1);
    const size_t groups = (g.tiles + S - 1) / S;
    unsigned blocks = (unsigned)(groups + (g.has_rem ? 1 : 0));
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL((k_fold_st<T, OP, NP, ORDER, S, PF, XCD>), dim3(blocks), dim3(kThreads), 0, st,
                       out, ins, g, groups);
    return hip_ok(hipGetLastError());
}

template <class T, class OP, int NP, int ORDER>
int launch_fold_np(T *out, const FoldPtrs &ins, size_t n, hipStream_t st)
{
    uintptr_t o = (uintptr_t)out;
    bool congruent = (o % sizeof(T)) == 0 && sizeof(T) <= 16;
    for (int k = 0; k < NP; ++k) congruent &= (((uintptr_t)ins.p[k] ^ o) & 15) == 0;
    if (!congruent) {
        size_t blocks = (n + kThreads - 1) / kThreads;
        if (blocks > 8192) blocks = 8192;
        hipLaunchKernelGGL((k_fold_scalar<T, OP, NP, ORDER>), dim3((unsigned)blocks),
                           dim3(kThreads), 0, st, out, ins, n);
        return hip_ok(hipGetLastError());
    }
    if constexpr (std::is_same<T, float>::value && std::is_same<OP, OpSum>::value && NP == 8 &&
                  ORDER == SOSX_ORDER_LINEAR) {
        if (g_fold_variant == 1) return launch_fold_u<T, OP, NP, ORDER, 2>(out, ins, n, st);
        if (g_fold_variant == 2) return launch_fold_u<T, OP, NP, ORDER, 4>(out, ins, n, st);
        if (g_fold_variant == 3) return launch_fold_st<T, OP, NP, ORDER, 4, false, false>(out, ins, n, st);
        if (g_fold_variant == 4) return launch_fold_st<T, OP, NP, ORDER, 16, false, false>(out, ins, n, st);
        if (g_fold_variant == 5) return launch_fold_st<T, OP, NP, ORDER, 1, false, true>(out, ins, n, st);
        if (g_fold_variant == 6) return launch_fold_st<T, OP, NP, ORDER, 4, true, false>(out, ins, n, st);
        if (g_fold_variant == 7) return launch_fold_st<T, OP, NP, ORDER, 16, true, true>(out, ins, n, st);
    }
    constexpr int U = NP <= 2 ? 4 : (NP <= 4 ? 2 : 1);
    Geom g = make_geom(o, n, sizeof(T), U);
    hipLaunchKernelGGL((k_fold<T, OP, NP, ORDER, U>), dim3(grid_for(g, kNoCap)), dim3(kThreads),
                       0, st, out, ins, g);
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
        default: {
            size_t blocks = (n + kThreads - 1) / kThreads;
            if (blocks > 8192) blocks = 8192;
            hipLaunchKernelGGL((k_fold_dyn<T, OP, ORDER>), dim3((unsigned)blocks), dim3(kThreads), 0,
                               st, out, ins, nin, n);
            return hip_ok(hipGetLastError());
        }
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

template <class T, class OP, int NP, int U, bool NT>
int launch_prefix_u(const PrefixPtrs &p, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)p.out[0], n, sizeof(T), U);
    hipLaunchKernelGGL((k_prefix<T, OP, NP, U, NT>), dim3(grid_for(g, kNoCap)), dim3(kThreads), 0, st, p, g);
    return hip_ok(hipGetLastError());
}

template <class T, class OP, int NP>
int launch_prefix_np(const PrefixPtrs &p, size_t n, hipStream_t st)
{
    if constexpr (std::is_same<T, float>::value && std::is_same<OP, OpSum>::value && NP >= 2) {
        if (g_prefix_variant == 1) return launch_prefix_u<T, OP, NP, 2, true>(p, n, st);
        if (g_prefix_variant == 2) return launch_prefix_u<T, OP, NP, 4, true>(p, n, st);
        if (g_prefix_variant == 3) return launch_prefix_u<T, OP, NP, 1, false>(p, n, st);
        if (g_prefix_variant == 4) return launch_prefix_u<T, OP, NP, 2, false>(p, n, st);
        if (g_prefix_variant == 5) return launch_prefix_u<T, OP, NP, 8, true>(p, n, st);
    }
    return launch_prefix_u<T, OP, NP, kPrefixU, true>(p, n, st);
}

struct PrefixFn {
    template <class T, class OP>
    static int run(const PrefixPtrs *p, int np, int own, size_t n, hipStream_t st)
    {
        const uintptr_t o = (uintptr_t)p->out[0];
        bool congruent = (o % sizeof(T)) == 0 && sizeof(T) <= 16;
        for (int k = 0; k < np; ++k)
            congruent &= (((uintptr_t)p->in[k] ^ o) & 15) == 0 && (((uintptr_t)p->out[k] ^ o) & 15) == 0;
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

// Tuning knob (bench A/B only) for the 8-input fp32 sum LINEAR fold: 0 = default,
// 1 = U=2, 2 = U=4, 3/4 = 4/16 consecutive tiles per workgroup, 5 = XCD-contiguous
// tile order, 6 = 4 tiles with the next tile's loads issued before the store,
// 7 = 16 tiles prefetched, XCD-contiguous.  Returns the previous value.
int sosx_set_fold_variant(int v)
{
    const int prev = g_fold_variant;
    if (v >= 0 && v <= 7) g_fold_variant = v;
    return prev;
}

// Same for the 8-input fp32 sum prefix: 0 = default (U=1, nontemporal), 1 = U=2,
// 2 = U=4, 3 = U=1 plain loads/stores, 4 = U=2 plain, 5 = U=8.  Returns the previous value.
int sosx_set_prefix_variant(int v)
{
    const int prev = g_prefix_variant;
    if (v >= 0 && v <= 5) g_prefix_variant = v;
    return prev;
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
