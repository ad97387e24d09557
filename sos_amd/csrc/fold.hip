// fold.hip -- the fused P-way fold used by the team schedules (sosx_fold).
//
// A team reduction over P resident input vectors (own source + P-1 received partner
// chunks) is evaluated in ONE pass: (P+1)*n*s HBM bytes instead of 3*(P-1)*n*s for
// P-1 pairwise reduce_local calls.  Two element orders are available, each
// bit-identical to one SOS schedule:
//   LINEAR: acc = in[0]; acc = acc OP in[k]  -- the ring reduce-scatter fold
//           (src/collectives.c:693-727: partial = partial OP own source);
//   TREE  : the recdbl_sw butterfly (src/collectives.c:905-963).
// P <= 8 (one PE per GPU on one node) and is a template parameter.
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
__global__ __launch_bounds__(kThreads) void k_fold(T *__restrict__ out, FoldPtrs ins, Geom g)
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

template <class T, class OP, int NP, int ORDER>
__global__ __launch_bounds__(kThreads) void k_fold_scalar(T *__restrict__ out, FoldPtrs ins,
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

}  // namespace sos

using namespace sos;

namespace {

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
        default: return SOSX_ERR_ARG;
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

}  // namespace

extern "C" {

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
