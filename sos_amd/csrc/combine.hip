// combine.hip -- the local combine inout = inout OP in (sosx_combine / sosx_combine3),
// the device replacement for shmem_internal_reduce_local (src/shmem_internal_op.h:305-339).
//
// A 3-stream elementwise pass (read in, read inout, write inout; 1 op per element) is
// HBM-bandwidth bound.  The kernel is built for the HBM roofline:
//   * 16-byte (dwordx4) nontemporal loads/stores per lane, U vectors per lane per
//     operand (default U=1), all 2U loads of a tile issued before the first combine;
//   * 256-thread workgroups, one 4 KiB-per-operand tile per workgroup, >> 256
//     workgroups per launch (a 128Mi fp32 combine is 131072 workgroups), the ragged
//     head/tail handled by one extra workgroup so the hot tiles carry no bounds checks;
//   * relative 16-B misalignment of the operands falls back to element loads.
// Tuning variants (bench.py --variants) are compiled for the fp32 sum only.
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

// Buffer-descriptor variant: raw_buffer_load/store_b128 with explicit cache-policy
// bits (gfx950 aux: sc0 = 1, nt = 2, sc1 = 16), one wave-uniform descriptor per tile.
// Tuning variants only (bench --variants).
template <class T, class OP, int U, int AUXL, int AUXS>
__global__ __launch_bounds__(kThreads) void k_combine3_buf(T *out, const T *a,
                                                             const T *b, Geom g)
{
    constexpr int V = Pack<T>::N;
    constexpr int kTileBytes = kThreads * U * 16;
    for (size_t t = blockIdx.x; t < g.tiles; t += gridDim.x) {
        const size_t tb = t * (size_t)kTileBytes;
        auto rA = __builtin_amdgcn_make_buffer_rsrc((void *)((const char *)(a + g.head) + tb), 0,
                                                    kTileBytes, 0x00020000);
        auto rB = __builtin_amdgcn_make_buffer_rsrc((void *)((const char *)(b + g.head) + tb), 0,
                                                    kTileBytes, 0x00020000);
        auto rO = __builtin_amdgcn_make_buffer_rsrc((void *)((char *)(out + g.head) + tb), 0,
                                                    kTileBytes, 0x00020000);
        u32x4 ra[U], rb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int off = (int)(threadIdx.x + u * kThreads) * 16;
            ra[u] = __builtin_amdgcn_raw_buffer_load_b128(rA, off, 0, AUXL);
            rb[u] = __builtin_amdgcn_raw_buffer_load_b128(rB, off, 0, AUXL);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(apply<T, OP>(ra[u], rb[u]), rO,
                                                   (int)(threadIdx.x + u * kThreads) * 16, 0, AUXS);
    }
    if (g.has_rem && blockIdx.x == gridDim.x - 1) {
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) out[i] = OP::f(a[i], b[i]);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * U * V) + threadIdx.x; i < g.n;
             i += kThreads)
            out[i] = OP::f(a[i], b[i]);
    }
}

// LDS-staged partner tile: the partner vector `b` is brought into LDS by LDS-DMA
// (global_load_lds_dwordx4) while `a` streams into registers.  Kept as a measured
// alternative (bench --variants); for a pure 3-stream combine the LDS round trip
// buys nothing over register staging (MI355X guide, "glds vs register staging").
template <class T, class OP, int U>
__global__ __launch_bounds__(kThreads) void k_combine3_lds(T *out, const T *a,
                                                             const T *b, Geom g)
{
    constexpr int V = Pack<T>::N;
    __shared__ __attribute__((aligned(16))) u32x4 tile[kThreads * U];
    const u32x4 *A = reinterpret_cast<const u32x4 *>(a + g.head);
    const u32x4 *B = reinterpret_cast<const u32x4 *>(b + g.head);
    u32x4 *O = reinterpret_cast<u32x4 *>(out + g.head);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (size_t t = blockIdx.x; t < g.tiles; t += gridDim.x) {
        const size_t base = t * (size_t)(kThreads * U) + threadIdx.x;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // LDS destination = wave-uniform base + lane*16 (lane-linear image).
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(B + base + u * kThreads),
                (__attribute__((address_space(3))) void *)(&tile[u * kThreads + wave * 64]), 16,
                0, 0);
        }
        u32x4 ra[U];
#pragma unroll
        for (int u = 0; u < U; ++u) ra[u] = A[base + u * kThreads];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < U; ++u)
            O[base + u * kThreads] = apply<T, OP>(ra[u], tile[u * kThreads + wave * 64 + lane]);
        __builtin_amdgcn_s_barrier();
    }
    if (g.has_rem && blockIdx.x == gridDim.x - 1) {
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) out[i] = OP::f(a[i], b[i]);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * U * V) + threadIdx.x; i < g.n;
             i += kThreads)
            out[i] = OP::f(a[i], b[i]);
    }
}

// Shape experiments (bench --variants): TPB threads per workgroup (tile = TPB 16-B
// vectors per operand) and, with XCD = 1, an XCD-contiguous tile order: the dispatcher
// deals consecutive workgroups round-robin to the 8 XCDs, so workgroup w runs on XCD
// w % 8; tile = (w % 8) * per_xcd + w / 8 gives each XCD one contiguous stretch of the
// vectors instead of every 8th tile.
template <class T, class OP, int TPB, int XCD>
__global__ __launch_bounds__(TPB) void k_combine3_x(T *out, const T *a, const T *b, Geom g,
                                                   unsigned nvec_tiles)
{
    constexpr int V = Pack<T>::N;
    const u32x4 *A = reinterpret_cast<const u32x4 *>(a + g.head);
    const u32x4 *B = reinterpret_cast<const u32x4 *>(b + g.head);
    u32x4 *O = reinterpret_cast<u32x4 *>(out + g.head);
    const unsigned w = blockIdx.x;
    if (w < nvec_tiles) {
        size_t t = w;
        if constexpr (XCD) {
            const unsigned per = nvec_tiles / 8;   // host guarantees nvec_tiles % 8 == 0
            t = (size_t)(w % 8) * per + w / 8;
        }
        const size_t i = t * TPB + threadIdx.x;
        u32x4 ra = ldv<true>(A + i), rb = ldv<true>(B + i);
        stv<true>(O + i, apply<T, OP>(ra, rb));
    } else if (g.has_rem && threadIdx.x < kThreads) {
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) out[i] = OP::f(a[i], b[i]);
        for (size_t i = g.head + (size_t)nvec_tiles * TPB * V + threadIdx.x; i < g.n; i += kThreads)
            out[i] = OP::f(a[i], b[i]);
    }
}

// Relative misalignment between the operands (not 16-B congruent): element loads.
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

int g_variant = 0;

struct VariantDesc {
    const char *name;
};
const VariantDesc kVariants[] = {
    {"u1_nt"},             // 0: default: U=1, nontemporal loads+stores, one tile/workgroup
    {"u4_nt"},             // 1: U=4 (round-1 default until the A/B in profiles/r1_combine_variants*)
    {"u2_nt"},             // 2
    {"u8_nt"},             // 3
    {"u4_ntload"},         // 4: nontemporal loads, plain stores
    {"u4_plain"},          // 5: plain loads/stores
    {"u1_plain"},          // 6
    {"u4_nt_persist4096"}, // 7: grid-stride over 4096 workgroups
    {"u2_nt_persist2048"}, // 8
    {"u4_lds_dma"},        // 9: partner tile via global_load_lds (LDS-DMA)
    {"buf_u4_nt"},         // 10: buffer loads/stores, aux nt
    {"buf_u4_plainld_ntst"},  // 11
    {"buf_u4_sc1nt"},      // 12: aux sc1|nt both ways
    {"buf_u2_nt"},         // 13
    {"buf_u1_nt"},         // 14
    {"x256_xcd"},          // 15: 256 threads, XCD-contiguous tiles
    {"x512"},              // 16: 512 threads per workgroup (8 KiB tiles)
    {"x1024"},             // 17: 1024 threads per workgroup
    {"x512_xcd"},          // 18
    {"x256"},              // 19: the k_combine3_x control (same shape as u1_nt)
};
constexpr int kNumVariants = (int)(sizeof(kVariants) / sizeof(kVariants[0]));

template <class T, class OP, int U, bool NTL, bool NTS>
int launch_combine3_vec(T *out, const T *a, const T *b, size_t n, hipStream_t st, size_t cap)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), U);
    unsigned grid = grid_for(g, cap);
    hipLaunchKernelGGL((k_combine3<T, OP, U, NTL, NTS>), dim3(grid), dim3(kThreads), 0, st, out,
                       a, b, g);
    return hip_ok(hipGetLastError());
}

template <class T, class OP, int TPB, int XCD>
int launch_x(T *out, const T *a, const T *b, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), 1);
    const size_t V = 16 / sizeof(T);
    size_t tiles = (n - g.head) / V / TPB;
    if (XCD) tiles -= tiles % 8;
    g.tiles = tiles;
    g.has_rem = (g.head > 0) || (tiles * TPB * V != n - g.head);
    const unsigned grid = (unsigned)(tiles + (g.has_rem ? 1 : 0));
    if (grid == 0) return SOSX_OK;
    hipLaunchKernelGGL((k_combine3_x<T, OP, TPB, XCD>), dim3(grid), dim3(TPB), 0, st, out, a, b, g,
                       (unsigned)tiles);
    return hip_ok(hipGetLastError());
}

template <class T, class OP>
int launch_combine3(T *out, const T *a, const T *b, size_t n, hipStream_t st)
{
    if (n == 0) return SOSX_OK;
    const uintptr_t o = (uintptr_t)out, pa = (uintptr_t)a, pb = (uintptr_t)b;
    const bool congruent = ((o ^ pa) & 15) == 0 && ((o ^ pb) & 15) == 0 && (o % sizeof(T)) == 0;
    if (!congruent || sizeof(T) > 16) {
        size_t blocks = (n + kThreads - 1) / kThreads;
        if (blocks > 8192) blocks = 8192;
        hipLaunchKernelGGL((k_combine3_scalar<T, OP>), dim3((unsigned)blocks), dim3(kThreads), 0,
                           st, out, a, b, n);
        return hip_ok(hipGetLastError());
    }
    if constexpr (std::is_same<T, float>::value && std::is_same<OP, OpSum>::value) {
        switch (g_variant) {
            case 1: return launch_combine3_vec<T, OP, 4, true, true>(out, a, b, n, st, kNoCap);
            case 2: return launch_combine3_vec<T, OP, 2, true, true>(out, a, b, n, st, kNoCap);
            case 3: return launch_combine3_vec<T, OP, 8, true, true>(out, a, b, n, st, kNoCap);
            case 4: return launch_combine3_vec<T, OP, 4, true, false>(out, a, b, n, st, kNoCap);
            case 5: return launch_combine3_vec<T, OP, 4, false, false>(out, a, b, n, st, kNoCap);
            case 6: return launch_combine3_vec<T, OP, 1, false, false>(out, a, b, n, st, kNoCap);
            case 7: return launch_combine3_vec<T, OP, 4, true, true>(out, a, b, n, st, 4096);
            case 8: return launch_combine3_vec<T, OP, 2, true, true>(out, a, b, n, st, 2048);
            case 9: {
                Geom g = make_geom(o, n, sizeof(T), 4);
                hipLaunchKernelGGL((k_combine3_lds<T, OP, 4>), dim3(grid_for(g, kNoCap)),
                                   dim3(kThreads), 0, st, out, a, b, g);
                return hip_ok(hipGetLastError());
            }
            case 10: case 11: case 12: case 13: case 14: {
                const int U = g_variant == 13 ? 2 : g_variant == 14 ? 1 : 4;
                Geom g = make_geom(o, n, sizeof(T), U);
                dim3 gr(grid_for(g, kNoCap)), bl(kThreads);
                if (g_variant == 10) hipLaunchKernelGGL((k_combine3_buf<T, OP, 4, 2, 2>), gr, bl, 0, st, out, a, b, g);
                if (g_variant == 11) hipLaunchKernelGGL((k_combine3_buf<T, OP, 4, 0, 2>), gr, bl, 0, st, out, a, b, g);
                if (g_variant == 12) hipLaunchKernelGGL((k_combine3_buf<T, OP, 4, 18, 18>), gr, bl, 0, st, out, a, b, g);
                if (g_variant == 13) hipLaunchKernelGGL((k_combine3_buf<T, OP, 2, 2, 2>), gr, bl, 0, st, out, a, b, g);
                if (g_variant == 14) hipLaunchKernelGGL((k_combine3_buf<T, OP, 1, 2, 2>), gr, bl, 0, st, out, a, b, g);
                return hip_ok(hipGetLastError());
            }
            case 15: return launch_x<T, OP, 256, 1>(out, a, b, n, st);
            case 16: return launch_x<T, OP, 512, 0>(out, a, b, n, st);
            case 17: return launch_x<T, OP, 1024, 0>(out, a, b, n, st);
            case 18: return launch_x<T, OP, 512, 1>(out, a, b, n, st);
            case 19: return launch_x<T, OP, 256, 0>(out, a, b, n, st);
            default: break;
        }
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

int sosx_set_combine_variant(int variant)
{
    int prev = g_variant;
    if (variant >= 0 && variant < kNumVariants) g_variant = variant;
    return prev;
}

int sosx_num_combine_variants(void) { return kNumVariants; }

const char *sosx_combine_variant_name(int variant)
{
    return (variant >= 0 && variant < kNumVariants) ? kVariants[variant].name : "";
}

const char *sosx_build_info(void)
{
    return "sos_amd: gfx950 HIP kernels (combine/fold/fill), hipcc " __clang_version__;
}

}  // extern "C"
