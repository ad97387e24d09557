// combine_kernels.h -- the local combine kernel (out = a OP b, out may alias a), shared by
// the product library (combine.hip) and the bench-only variant library
// (tools/variants/variants.hip).
#pragma once
#include "elementwise.h"

namespace sos {

// ---------------------------------------------------------------------------------
// out = a OP b (out may alias a): the local combine.
// ---------------------------------------------------------------------------------
template <class T, class OP, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(kThreads) void k_combine3(T *out, const T *a,
                                                         const T *b, Geom g)
{
    constexpr int V = Pack<T>::N;
    const u32x4 *A = reinterpret_cast<const u32x4 *>(a + g.head);
    const u32x4 *B = reinterpret_cast<const u32x4 *>(b + g.head);
    u32x4 *O = reinterpret_cast<u32x4 *>(out + g.head);
    for (size_t t = blockIdx.x; t < g.tiles; t += gridDim.x) {
        const size_t base = t * (size_t)(kThreads * U) + threadIdx.x;
        u32x4 ra[U], rb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ra[u] = ldv<NTL>(A + base + u * kThreads);
            rb[u] = ldv<NTL>(B + base + u * kThreads);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) stv<NTS>(O + base + u * kThreads, apply<T, OP>(ra[u], rb[u]));
    }
    if (g.has_rem && blockIdx.x == gridDim.x - 1) {
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) out[i] = OP::f(a[i], b[i]);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * U * V) + threadIdx.x; i < g.n;
             i += kThreads)
            out[i] = OP::f(a[i], b[i]);
    }
}

// ---------------------------------------------------------------------------------
// out = a OP b with `b` NOT 16-B congruent with out/a (a caller's sub-array, SOS's
// reduce_local takes any element alignment): out and a stream as in k_combine3; each
// lane loads the two 16-B-aligned vectors of b that its 16 bytes straddle and funnel-
// shifts them into place (v_alignbyte), so every HBM access stays a 16-B vector instead
// of one element per lane.  `d` = the byte offset of b's vector j within b's aligned
// vector j (1..15, a multiple of the element alignment).  A 16-B-aligned load that holds
// at least one byte of b cannot cross a page boundary, and every load here does, so
// reading the bytes shifted out is safe.  Same element operations as k_combine3.
// ---------------------------------------------------------------------------------
// MODE 0: the two aligned loads per lane; 1: the next vector from the next lane (DPP,
// lane 63 loads its own); 2: one unaligned 16-B load (4- and 8-byte elements).
template <class T, class OP, int MODE = 0>
__global__ __launch_bounds__(kThreads) void k_combine3_realign(T *out, const T *a, const T *b,
                                                                 Geom g, unsigned d)
{
    constexpr int V = Pack<T>::N;
    const size_t nblk = gridDim.x;
    const u32x4 *A = reinterpret_cast<const u32x4 *>(a + g.head);
    const u32x4 *B = reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>(b + g.head) - d);
    u32x4 *O = reinterpret_cast<u32x4 *>(out + g.head);
    for (size_t t = blockIdx.x; t < g.tiles; t += nblk) {
        const size_t i = t * (size_t)kThreads + threadIdx.x;
        const u32x4 ra = ldv<true>(A + i);
        if constexpr (MODE == 2) {
            stv<true>(O + i, apply<T, OP>(ra, ldv_unaligned(reinterpret_cast<const char *>(B + i) + d)));
        } else if constexpr (MODE == 1) {
            const bool last_lane = (threadIdx.x & 63) == 63;
            const u32x4 lo = ldv<true>(B + i);
            u32x4 hi = next_lane16(lo);
            if (last_lane) hi = ldv<true>(B + i + 1);
            stv<true>(O + i, apply<T, OP>(ra, realign16(lo, hi, d)));
        } else {
            const u32x4 lo = ldv<true>(B + i), hi = ldv<true>(B + i + 1);
            stv<true>(O + i, apply<T, OP>(ra, realign16(lo, hi, d)));
        }
    }
    if (g.has_rem && blockIdx.x == nblk - 1) {
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) out[i] = OP::f(a[i], b[i]);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            out[i] = OP::f(a[i], b[i]);
    }
}

}  // namespace sos
