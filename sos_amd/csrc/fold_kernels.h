// fold_kernels.h -- the fused P-way fold (k_fold) and the fused prefix (k_prefix), the
// team schedules' local steps, shared by the product library (fold.hip) and the
// bench-only variant library (tools/variants/variants.hip).
#pragma once
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

// ---------------------------------------------------------------------------------
// The P-way fold (2 <= P <= 8, at run time) when some inputs are NOT 16-B congruent with
// the output: a team reduction whose source and target sit at different 16-B offsets
// (the PE's own source chunk, or the peers' sources read in place, against exchange
// scratch congruent with the target).  16-B vectors throughout: an input at byte offset
// d[k] != 0 is read as the two aligned vectors its bytes straddle and funnel-shifted
// into place (realign16; see k_combine3_realign for why the extra bytes are safe to
// load).  LINEAR: acc = in[0] OP in[1] OP ... (the ring); TREE: the recdbl_sw tree of
// fold_elem (the extras folded into the first P - p2 leaves, then distance 1, 2, 4 pairs,
// the lower subtree the left operand) -- with P at run time on compile-time indices, so
// one kernel per (type, op, order) serves every P.
// ---------------------------------------------------------------------------------
struct FoldRealignArgs {
    const void *p[8];
    unsigned d[8];
    int np;
};

template <class T, class OP, int ORDER>
__device__ __forceinline__ u32x4 fold_runtime_np(u32x4 (&x)[8], int np)
{
    if constexpr (ORDER == SOSX_ORDER_LINEAR) {
        u32x4 acc = x[0];
#pragma unroll
        for (int k = 1; k < 8; ++k)
            if (k < np) acc = apply<T, OP>(acc, x[k]);
        return acc;
    } else {
        const int p2 = np >= 8 ? 8 : np >= 4 ? 4 : 2;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < np - p2) x[k] = apply<T, OP>(x[k], x[k + p2]);
#pragma unroll
        for (int d = 1; d < 8; d <<= 1)
#pragma unroll
            for (int k = 0; k < 8; k += 2 * d)
                if (d < p2 && k < p2) x[k] = apply<T, OP>(x[k], x[k + d]);
        return x[0];
    }
}

template <class T, class OP, int ORDER>
__device__ __forceinline__ T fold_runtime_np_elem(const FoldRealignArgs &a, size_t i)
{
    T v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = k < a.np ? ((const T *)a.p[k])[i] : T();
    // (LINEAR: v[0] OP v[1] OP ...; TREE: fold_elem's recdbl_sw tree, 2 <= np <= 8)
    if constexpr (ORDER == SOSX_ORDER_LINEAR) {
        T acc = v[0];
        for (int k = 1; k < a.np; ++k) acc = OP::f(acc, v[k]);
        return acc;
    } else {
        const int p2 = a.np >= 8 ? 8 : a.np >= 4 ? 4 : 2;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < a.np - p2) v[k] = OP::f(v[k], v[k + p2]);
#pragma unroll
        for (int d = 1; d < 8; d <<= 1)
#pragma unroll
            for (int k = 0; k < 8; k += 2 * d)
                if (d < p2 && k < p2) v[k] = OP::f(v[k], v[k + d]);
        return v[0];
    }
}

template <class T, class OP, int ORDER = SOSX_ORDER_LINEAR>
__global__ __launch_bounds__(kThreads) void k_fold_realign(T *out, FoldRealignArgs a, Geom g)
{
    constexpr int V = Pack<T>::N;
    const size_t nblk = gridDim.x;
    const int np = a.np;
    u32x4 *O = reinterpret_cast<u32x4 *>(out + g.head);
    for (size_t t = blockIdx.x; t < g.tiles; t += nblk) {
        const size_t i = t * (size_t)kThreads + threadIdx.x;
        u32x4 x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k < np) {
                const unsigned d = a.d[k];
                const u32x4 *I = reinterpret_cast<const u32x4 *>(
                    reinterpret_cast<const char *>((const T *)a.p[k] + g.head) - d);
                const u32x4 lo = ldv<true>(I + i);
                x[k] = d ? realign16(lo, ldv<true>(I + i + 1), d) : lo;
            }
        }
        stv<true>(O + i, fold_runtime_np<T, OP, ORDER>(x, np));
    }
    if (g.has_rem && blockIdx.x == nblk - 1) {
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) out[i] = fold_runtime_np_elem<T, OP, ORDER>(a, i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            out[i] = fold_runtime_np_elem<T, OP, ORDER>(a, i);
    }
}

constexpr int kMaxPrefix = 64;

struct PrefixPtrs {
    const void *in[kMaxPrefix];
    void *out[kMaxPrefix];
};

// 16-B vectors per lane per tile.  U = 2/4/8 and plain loads/stores measured slower over
// random buffer layouts (profiles/r2_prefix_variants*.txt); they are kept in
// the bench-only variant library (tools/variants/).
constexpr int kPrefixU = 1;

// NT: nontemporal loads/stores (the default); plain loads/stores are a bench A/B only.
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

// The team scan's prefix (1 <= P <= 8, at run time) when some INPUTS sit at another 16-B
// offset than the outputs (a scan whose source and target are at different offsets: the
// PE's own source chunk against target-congruent scratch); the outputs are congruent.
// Inputs realigned as in k_fold_realign; every input vector of a tile is loaded before
// the first store, as in k_prefix (an output may alias an input: the aliased pair is
// congruent, so it is never read past its own vector).
struct PrefixRealignArgs {
    const void *in[8];
    void *out[8];
    unsigned d[8];
    int np;
};

template <class T, class OP>
__global__ __launch_bounds__(kThreads) void k_prefix_realign(PrefixRealignArgs a, Geom g)
{
    constexpr int V = Pack<T>::N;
    const size_t nblk = gridDim.x;
    const int np = a.np;
    for (size_t t = blockIdx.x; t < g.tiles; t += nblk) {
        const size_t i = t * (size_t)kThreads + threadIdx.x;
        u32x4 x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k < np) {
                const unsigned d = a.d[k];
                const u32x4 *I = reinterpret_cast<const u32x4 *>(
                    reinterpret_cast<const char *>((const T *)a.in[k] + g.head) - d);
                const u32x4 lo = ldv<true>(I + i);
                x[k] = d ? realign16(lo, ldv<true>(I + i + 1), d) : lo;
            }
        }
        u32x4 acc = x[0];
        stv<true>(reinterpret_cast<u32x4 *>((T *)a.out[0] + g.head) + i, acc);
#pragma unroll
        for (int k = 1; k < 8; ++k) {
            if (k < np) {
                acc = apply<T, OP>(acc, x[k]);
                stv<true>(reinterpret_cast<u32x4 *>((T *)a.out[k] + g.head) + i, acc);
            }
        }
    }
    if (g.has_rem && blockIdx.x == nblk - 1) {
        auto one = [&](size_t i) {
            T v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = k < np ? ((const T *)a.in[k])[i] : T();
            T acc = v[0];
            ((T *)a.out[0])[i] = acc;
#pragma unroll
            for (int k = 1; k < 8; ++k) {
                if (k < np) {
                    acc = OP::f(acc, v[k]);
                    ((T *)a.out[k])[i] = acc;
                }
            }
        };
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) one(i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            one(i);
    }
}

}  // namespace sos
