// combine.hip -- the local combine inout = inout OP in (sosx_combine / sosx_combine3),
// the device replacement for shmem_internal_reduce_local (src/shmem_internal_op.h:305-339).
//
// A 3-stream elementwise pass (read in, read inout, write inout; 1 op per element) is
// HBM-bandwidth bound.  The kernel (combine_kernels.h) is built for the HBM roofline:
//   * 16-byte (dwordx4) nontemporal loads/stores per lane, U vectors per lane per
//     operand (default U=1), all 2U loads of a tile issued before the first combine;
//   * 256-thread workgroups, one 4 KiB-per-operand tile per workgroup, >> 256
//     workgroups per launch (a 128Mi fp32 combine is 131072 workgroups), the ragged
//     head/tail handled by one extra workgroup so the hot tiles carry no bounds checks;
//   * `in` at another 16-B offset than inout: the same vectors, each lane funnel-shifting
//     the two aligned vectors of `in` its bytes straddle (k_combine3_realign); only
//     operands that are not element-aligned, or inout/out incongruent, take element loads.
// The shapes this default won against (U, plain loads/stores, persistent grids, LDS-DMA
// partner tiles, buffer loads, 512/1024-thread workgroups, XCD-contiguous tile order;
// DESIGN.md section 4) live in the bench-only library tools/variants/.
#include "combine_kernels.h"

namespace sos {

// Operands not element-aligned, or out and a not 16-B congruent: element loads.
template <class T, class OP>
__global__ __launch_bounds__(kThreads) void k_combine3_scalar(T *out, const T *a,
                                                                const T *b, size_t n)
{
    const size_t stride = (size_t)gridDim.x * kThreads;
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
        out[i] = OP::f(a[i], b[i]);
}

}  // namespace sos

using namespace sos;

namespace {

template <class T, class OP, int U, bool NTL, bool NTS>
int launch_combine3_vec(T *out, const T *a, const T *b, size_t n, hipStream_t st, size_t cap)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), U);
    unsigned grid = grid_for(g, cap);
    hipLaunchKernelGGL((k_combine3<T, OP, U, NTL, NTS>), dim3(grid), dim3(kThreads), 0, st, out,
                       a, b, g);
    return hip_ok(hipGetLastError());
}

// Bench switch SOSX_COMBINE_REALIGN (k_combine3_realign's MODE): 0 two aligned loads per
// lane, 1 DPP, 2 unaligned loads (4- and 8-byte elements; others take 0).
inline int combine_realign_mode()
{
    static const int m = [] {
        const char *e = getenv("SOSX_COMBINE_REALIGN");
        return e && *e ? atoi(e) : 0;
    }();
    return m;
}

template <class T, class OP>
int launch_combine3(T *out, const T *a, const T *b, size_t n, hipStream_t st)
{
    if (n == 0) return SOSX_OK;
    const uintptr_t o = (uintptr_t)out, pa = (uintptr_t)a, pb = (uintptr_t)b;
    const bool congruent = ((o ^ pa) & 15) == 0 && ((o ^ pb) & 15) == 0 && (o % sizeof(T)) == 0;
    // `in` at another 16-B offset than inout (element-aligned): the realigning kernel,
    // 6.41-6.63 TB/s at 512 MiB per operand against 2.68-5.13 for element loads
    // (profiles/r4_misaligned_combine.txt)
    if (!congruent && sizeof(T) <= 16 && ((o ^ pa) & 15) == 0 && (o % sizeof(T)) == 0 &&
        (pb % sizeof(T)) == 0) {
        Geom g = make_geom(o, n, sizeof(T), 1);
        const unsigned d = (unsigned)((uintptr_t)(b + g.head) & 15);
        constexpr bool kUL = sizeof(T) == 4 || sizeof(T) == 8;
        const int mode = combine_realign_mode();
        if (mode == 2 && kUL)
            hipLaunchKernelGGL((k_combine3_realign<T, OP, kUL ? 2 : 0>), dim3(grid_for(g, kNoCap)), dim3(kThreads),
                               0, st, out, a, b, g, d);
        else if (mode == 1)
            hipLaunchKernelGGL((k_combine3_realign<T, OP, 1>), dim3(grid_for(g, kNoCap)), dim3(kThreads), 0, st,
                               out, a, b, g, d);
        else
            hipLaunchKernelGGL((k_combine3_realign<T, OP>), dim3(grid_for(g, kNoCap)), dim3(kThreads), 0,
                               st, out, a, b, g, d);
        return hip_ok(hipGetLastError());
    }
    if (!congruent || sizeof(T) > 16) {
        size_t blocks = (n + kThreads - 1) / kThreads;
        if (blocks > 8192) blocks = 8192;
        hipLaunchKernelGGL((k_combine3_scalar<T, OP>), dim3((unsigned)blocks), dim3(kThreads), 0,
                           st, out, a, b, n);
        return hip_ok(hipGetLastError());
    }
    // Default: U=1 (one 16-B vector per lane per operand, 4 KiB tiles), nontemporal loads
    // and stores: nt is worth +16% over plain loads/stores, U=1 ~2% over U=4 in two
    // independent A/B runs on the 128Mi fp32 sum (profiles/r1_combine_variants*.txt).
    return launch_combine3_vec<T, OP, 1, true, true>(out, a, b, n, st, kNoCap);
}

struct Combine3Fn {
    template <class T, class OP>
    static int run(void *out, const void *a, const void *b, size_t n, hipStream_t st)
    {
        return launch_combine3<T, OP>((T *)out, (const T *)a, (const T *)b, n, st);
    }
};

}  // namespace

extern "C" {

size_t sosx_dtype_size(int dtype) { return sos_dtype_info(dtype).size; }

int sosx_check_op(int op, int dtype) { return sos_check_op(op, dtype); }

int sosx_combine3(int op, int dtype, void *out, const void *a, const void *b, size_t count,
                  void *stream)
{
    if (count == 0) return sos_check_op(op, dtype);
    if (!out || !a || !b) return SOSX_ERR_ARG;
    return dispatch<Combine3Fn>(op, dtype, out, a, b, count, as_stream(stream));
}

int sosx_combine(int op, int dtype, void *inout, const void *in, size_t count, void *stream)
{
    return sosx_combine3(op, dtype, inout, inout, in, count, stream);
}

const char *sosx_build_info(void)
{
    return "sos_amd: gfx950 HIP kernels (combine/fold/fill), hipcc " __clang_version__;
}

}  // extern "C"
