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

}  // namespace sos
