// variants.hip -- BENCH-ONLY library (tools/variants/libsos_variants.so): the kernel
// shapes the product defaults were chosen against, kept so the
// A/Bs can be re-run and so tests can prove every shape computes the same bits.  The
// product library (sos_amd/libsos_amd.so) contains only the defaults; nothing in it
// calls or links this file.  fp32 sum only (the headline op):
//   sosxv_combine : the local combine out = a + b, 20 shapes (0 = the product default)
//   sosxv_fold    : the 8-input LINEAR fold, 18 shapes (0 = the product default)
//   sosxv_prefix  : the 2..8-input prefix, 16 shapes (0 = the product default)
#include "combine_kernels.h"
#include "fold_kernels.h"

namespace sos {

// Buffer-descriptor variant: raw_buffer_load/store_b128 with explicit cache-policy
// bits (gfx950 aux: sc0 = 1, nt = 2, sc1 = 16), one wave-uniform descriptor per tile.
// Tuning variants only (tools/variants_bench.py).
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
// alternative (tools/variants_bench.py); for a pure 3-stream combine the LDS round trip
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

// Shape experiments (tools/variants_bench.py): TPB threads per workgroup (tile = TPB 16-B
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

// The default shape with the grid stride and the remainder block's index read once,
// before the tile loop (k_combine3 re-reads gridDim from the dispatch packet after every
// tile's store -- the stores may alias it -- and a wave then waits for that scalar load
// before it can exit).
template <class T, class OP>
__global__ __launch_bounds__(kThreads) void k_combine3_h(T *out, const T *a, const T *b, Geom g)
{
    constexpr int V = Pack<T>::N;
    const size_t nblk = gridDim.x;
    const size_t tiles = g.tiles;
    const u32x4 *A = reinterpret_cast<const u32x4 *>(a + g.head);
    const u32x4 *B = reinterpret_cast<const u32x4 *>(b + g.head);
    u32x4 *O = reinterpret_cast<u32x4 *>(out + g.head);
    for (size_t t = blockIdx.x; t < tiles; t += nblk) {
        const size_t i = t * (size_t)kThreads + threadIdx.x;
        const u32x4 ra = ldv<true>(A + i), rb = ldv<true>(B + i);
        stv<true>(O + i, apply<T, OP>(ra, rb));
    }
    if (g.has_rem && blockIdx.x == nblk - 1) {
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) out[i] = OP::f(a[i], b[i]);
        for (size_t i = g.head + tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            out[i] = OP::f(a[i], b[i]);
    }
}

// Tuning variants of k_fold (bench A/B, sosxv_fold): each workgroup takes S
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

// Lane-contiguous shapes: each lane reads U CONSECUTIVE 16-B vectors
// of every input (lane l of tile t covers vectors (t * kThreads + l) * U .. + U - 1), so a
// wave's U loads of one input cover U * 1 KiB contiguous with each lane's own 64 B run;
// the default interleaves lanes (load u covers kThreads vectors at stride 1).  Same tile
// geometry (make_geom with U), same element order.
template <class T, class OP, int NP, int ORDER, int U>
__global__ __launch_bounds__(kThreads) void k_fold_lc(T *out, FoldPtrs ins, Geom g)
{
    constexpr int V = Pack<T>::N;
    u32x4 *O = reinterpret_cast<u32x4 *>(out + g.head);
    for (size_t t = blockIdx.x; t < g.tiles; t += gridDim.x) {
        const size_t base = (t * (size_t)kThreads + threadIdx.x) * U;
        u32x4 x[U][NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const u32x4 *I = reinterpret_cast<const u32x4 *>((const T *)ins.p[k] + g.head);
#pragma unroll
            for (int u = 0; u < U; ++u) x[u][k] = ldv<true>(I + base + u);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) stv<true>(O + base + u, fold_pack<T, OP, NP, ORDER>(x[u]));
    }
    if (g.has_rem && blockIdx.x == gridDim.x - 1) {
        auto one = [&](size_t i) {
            T v[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) v[k] = ((const T *)ins.p[k])[i];
            out[i] = fold_elem<T, OP, NP, ORDER>(v);
        };
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) one(i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * U * V) + threadIdx.x; i < g.n; i += kThreads)
            one(i);
    }
}

template <class T, class OP, int NP, int U>
__global__ __launch_bounds__(kThreads) void k_prefix_lc(PrefixPtrs p, Geom g)
{
    constexpr int V = Pack<T>::N;
    for (size_t t = blockIdx.x; t < g.tiles; t += gridDim.x) {
        const size_t base = (t * (size_t)kThreads + threadIdx.x) * U;
        u32x4 x[U][NP];
#pragma unroll
        for (int k = 0; k < NP; ++k)
#pragma unroll
            for (int u = 0; u < U; ++u)
                x[u][k] = ldv<true>(reinterpret_cast<const u32x4 *>((const T *)p.in[k] + g.head) + base + u);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u32x4 acc = x[u][0];
            stv<true>(reinterpret_cast<u32x4 *>((T *)p.out[0] + g.head) + base + u, acc);
#pragma unroll
            for (int k = 1; k < NP; ++k) {
                acc = apply<T, OP>(acc, x[u][k]);
                stv<true>(reinterpret_cast<u32x4 *>((T *)p.out[k] + g.head) + base + u, acc);
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

// Buffer-descriptor fold / prefix (round 5): nontemporal loads, stores with explicit aux
// bits -- sc1 stores leave no line behind in the XCD's L2 (MI355X guide, store flavours),
// so a 9- or 16-stream kernel's L2 is not filled with written lines whose write-backs
// interleave with the read streams.  U = 1, one tile per workgroup, same element order.
template <class T, class OP, int NP, int AUXL, int AUXS>
__global__ __launch_bounds__(kThreads) void k_fold_buf(T *out, FoldPtrs ins, Geom g)
{
    constexpr int V = Pack<T>::N;
    constexpr int kTileBytes = kThreads * 16;
    for (size_t t = blockIdx.x; t < g.tiles; t += gridDim.x) {
        const size_t tb = t * (size_t)kTileBytes;
        u32x4 x[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            auto r = __builtin_amdgcn_make_buffer_rsrc((void *)((const char *)((const T *)ins.p[k] + g.head) + tb),
                                                       0, kTileBytes, 0x00020000);
            x[k] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)threadIdx.x * 16, 0, AUXL);
        }
        auto rO = __builtin_amdgcn_make_buffer_rsrc((void *)((char *)(out + g.head) + tb), 0, kTileBytes,
                                                    0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(fold_pack<T, OP, NP, SOSX_ORDER_LINEAR>(x), rO,
                                               (int)threadIdx.x * 16, 0, AUXS);
    }
    if (g.has_rem && blockIdx.x == gridDim.x - 1) {
        auto one = [&](size_t i) {
            T v[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) v[k] = ((const T *)ins.p[k])[i];
            out[i] = fold_elem<T, OP, NP, SOSX_ORDER_LINEAR>(v);
        };
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) one(i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            one(i);
    }
}

template <class T, class OP, int NP, int AUXL, int AUXS>
__global__ __launch_bounds__(kThreads) void k_prefix_buf(PrefixPtrs p, Geom g)
{
    constexpr int V = Pack<T>::N;
    constexpr int kTileBytes = kThreads * 16;
    for (size_t t = blockIdx.x; t < g.tiles; t += gridDim.x) {
        const size_t tb = t * (size_t)kTileBytes;
        u32x4 x[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            auto r = __builtin_amdgcn_make_buffer_rsrc((void *)((const char *)((const T *)p.in[k] + g.head) + tb),
                                                       0, kTileBytes, 0x00020000);
            x[k] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)threadIdx.x * 16, 0, AUXL);
        }
        u32x4 acc = x[0];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            if (k) acc = apply<T, OP>(acc, x[k]);
            auto rO = __builtin_amdgcn_make_buffer_rsrc((void *)((char *)((T *)p.out[k] + g.head) + tb), 0,
                                                        kTileBytes, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(acc, rO, (int)threadIdx.x * 16, 0, AUXS);
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
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            one(i);
    }
}

// Realigning 8-input fold variants (round 6): the product's
// k_fold_realign_np loads two aligned vectors per incongruent input and reached 1.30x the
// algorithmic read bytes in FETCH_SIZE with 6 of 8 inputs incongruent
// (profiles/r6_realign_pmc.txt).  MODE 1: the second vector by a plain load (may hit the
// line the first load brought into L2); MODE 2: both loads plain; MODE 3: the second
// vector from the next lane by DPP wave_shl:1 (lane 63 loads it); MODE 4: the same through
// __shfl_down; MODE 5: two loads, plain for the incongruent inputs and nt for the
// congruent ones; MODE 6: plain loads + DPP; MODE 7: MODE 5's policy + DPP; MODE 8: DPP
// + LDS across waves; MODE 9 / 10: one unaligned 16-B load per lane (nt / plain).  Same
// element order as k_fold_realign_np.
typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(4)));

template <class T, class OP, int NP, int ORDER, int MODE>
__global__ __launch_bounds__(kThreads) void k_fold_realign_v(T *out, FoldRealignArgs a, Geom g)
{
    const size_t nblk = gridDim.x;
    const bool last_lane = (threadIdx.x & 63) == 63;
    u32x4 *O = reinterpret_cast<u32x4 *>(out + g.head);
    const u32x4 *I[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k)
        I[k] = reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>((const T *)a.p[k] + g.head) - a.d[k]);
    for (size_t t = blockIdx.x; t < g.tiles; t += nblk) {
        const size_t i = t * (size_t)kThreads + threadIdx.x;
        u32x4 x[NP], y[NP];
        constexpr bool kSplit = MODE == 5 || MODE == 7;  // nt only for congruent inputs
        constexpr bool kNt = MODE == 0 || MODE == 1 || MODE == 3 || MODE == 4 || MODE == 8 || MODE == 9;
        if constexpr (MODE == 9 || MODE == 10) {
            // one 16-B load per lane straight from the element-aligned (4-B) address: the
            // memory pipeline splits what straddles, no second vector, no shift
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                const u32x4u *p = reinterpret_cast<const u32x4u *>(reinterpret_cast<const char *>(I[k] + i) + a.d[k]);
                if constexpr (MODE == 9) x[k] = __builtin_nontemporal_load(p);
                else x[k] = *p;
            }
            stv<true>(O + i, fold_pack<T, OP, NP, ORDER>(x));
            continue;
        }
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            if constexpr (kSplit) x[k] = a.d[k] ? ldv<false>(I[k] + i) : ldv<true>(I[k] + i);
            else x[k] = ldv<kNt>(I[k] + i);
        }
        if constexpr (MODE <= 2 || MODE == 5) {
#pragma unroll
            for (int k = 0; k < NP; ++k)
                if (a.d[k]) y[k] = ldv<MODE == 0>(I[k] + i + 1);
        } else if constexpr (MODE == 8) {
            // DPP within the wave; across waves the next wave's lane 0 vector through LDS,
            // so only the workgroup's last lane loads (one extra vector per tile, not four)
            __shared__ u32x4 first[kThreads / 64][NP];
            const unsigned wave = threadIdx.x >> 6;
            if ((threadIdx.x & 63) == 0) {
#pragma unroll
                for (int k = 0; k < NP; ++k)
                    if (a.d[k]) first[wave][k] = x[k];
            }
            const bool wg_last = threadIdx.x == kThreads - 1;
            if (wg_last) {
#pragma unroll
                for (int k = 0; k < NP; ++k)
                    if (a.d[k]) y[k] = ldv<true>(I[k] + i + 1);
            }
            __syncthreads();
            if (last_lane && !wg_last) {
#pragma unroll
                for (int k = 0; k < NP; ++k)
                    if (a.d[k]) y[k] = first[wave + 1][k];
            }
#pragma unroll
            for (int k = 0; k < NP; ++k)
                if (a.d[k]) {
                    const u32x4 nx = next_lane16(x[k]);
                    if (!last_lane) y[k] = nx;
                }
            __syncthreads();  // first[] is rewritten by the next tile
        } else {
            if (last_lane) {
#pragma unroll
                for (int k = 0; k < NP; ++k)
                    if (a.d[k]) y[k] = ldv<kNt>(I[k] + i + 1);
            }
#pragma unroll
            for (int k = 0; k < NP; ++k)
                if (a.d[k]) {
                    u32x4 nx;
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        if constexpr (MODE != 4)
                            nx[c] = (unsigned)__builtin_amdgcn_update_dpp((int)0, (int)x[k][c], 0x130, 0xf, 0xf, false);
                        else
                            nx[c] = __shfl_down(x[k][c], 1u);
                    }
                    if (!last_lane) y[k] = nx;
                }
        }
#pragma unroll
        for (int k = 0; k < NP; ++k)
            if (a.d[k]) x[k] = realign16(x[k], y[k], a.d[k]);
        stv<true>(O + i, fold_pack<T, OP, NP, ORDER>(x));
    }
    if (g.has_rem && blockIdx.x == nblk - 1) {
        constexpr int V = Pack<T>::N;
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) out[i] = fold_runtime_np_elem<T, OP, ORDER>(a, i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            out[i] = fold_runtime_np_elem<T, OP, ORDER>(a, i);
    }
}

}  // namespace sos

using namespace sos;

namespace {

using T = float;
using OP = OpSum;

const char *const kCombineNames[] = {
    "u1_nt",             // 0: the product default: U=1, nontemporal loads+stores, one tile/workgroup
    "u4_nt",             // 1: U=4 (round-1 default until the A/B in profiles/r1_combine_variants*)
    "u2_nt",             // 2
    "u8_nt",             // 3
    "u4_ntload",         // 4: nontemporal loads, plain stores
    "u4_plain",          // 5: plain loads/stores
    "u1_plain",          // 6
    "u4_nt_persist4096", // 7: grid-stride over 4096 workgroups
    "u2_nt_persist2048", // 8
    "u4_lds_dma",        // 9: partner tile via global_load_lds (LDS-DMA)
    "buf_u4_nt",         // 10: buffer loads/stores, aux nt
    "buf_u4_plainld_ntst",  // 11
    "buf_u4_sc1nt",      // 12: aux sc1|nt both ways
    "buf_u2_nt",         // 13
    "buf_u1_nt",         // 14
    "x256_xcd",          // 15: 256 threads, XCD-contiguous tiles
    "x512",              // 16: 512 threads per workgroup (8 KiB tiles)
    "x1024",             // 17: 1024 threads per workgroup
    "x512_xcd",          // 18
    "x256",              // 19: the k_combine3_x control (same shape as u1_nt)
    "u1_nt_hoist",       // 20: u1_nt with gridDim read once before the tile loop
    "u1_nt_occ4",        // 21: u1_nt, 40 KiB of unused dynamic LDS: at most 4 workgroups per CU
    "u1_nt_occ3",        // 22: 48 KiB: at most 3 per CU
    "u1_nt_occ2",        // 23: 64 KiB: at most 2 per CU
    "u2_nt_occ4",        // 24
};
constexpr int kNumCombine = (int)(sizeof(kCombineNames) / sizeof(kCombineNames[0]));

template <int U, bool NTL, bool NTS>
int combine_vec(T *out, const T *a, const T *b, size_t n, hipStream_t st, size_t cap, unsigned lds = 0)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), U);
    hipLaunchKernelGGL((k_combine3<T, OP, U, NTL, NTS>), dim3(grid_for(g, cap)), dim3(kThreads), lds,
                       st, out, a, b, g);
    return hip_ok(hipGetLastError());
}

template <int TPB, int XCD>
int combine_x(T *out, const T *a, const T *b, size_t n, hipStream_t st)
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

template <int U, int AUXL, int AUXS>
int combine_buf(T *out, const T *a, const T *b, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), U);
    hipLaunchKernelGGL((k_combine3_buf<T, OP, U, AUXL, AUXS>), dim3(grid_for(g, kNoCap)),
                       dim3(kThreads), 0, st, out, a, b, g);
    return hip_ok(hipGetLastError());
}

template <int NP, int U>
int fold_u(T *out, const FoldPtrs &ins, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), U);
    hipLaunchKernelGGL((k_fold<T, OP, NP, SOSX_ORDER_LINEAR, U>), dim3(grid_for(g, kNoCap)),
                       dim3(kThreads), 0, st, out, ins, g);
    return hip_ok(hipGetLastError());
}

template <int S, bool PF, bool XCD>
int fold_st(T *out, const FoldPtrs &ins, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), 1);
    const size_t groups = (g.tiles + S - 1) / S;
    unsigned blocks = (unsigned)(groups + (g.has_rem ? 1 : 0));
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL((k_fold_st<T, OP, 8, SOSX_ORDER_LINEAR, S, PF, XCD>), dim3(blocks),
                       dim3(kThreads), 0, st, out, ins, g, groups);
    return hip_ok(hipGetLastError());
}

// Occupancy-capped shapes (round 5): the default kernel launched with `lds` bytes of
// unused dynamic LDS, so at most 160 KiB / lds workgroups share a CU: fewer concurrent
// workgroups, hence fewer DRAM rows open across the 9 (fold) or 16 (prefix) streams.
template <int NP, int U>
int fold_u_lds(T *out, const FoldPtrs &ins, size_t n, hipStream_t st, unsigned lds)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), U);
    hipLaunchKernelGGL((k_fold<T, OP, NP, SOSX_ORDER_LINEAR, U>), dim3(grid_for(g, kNoCap)),
                       dim3(kThreads), lds, st, out, ins, g);
    return hip_ok(hipGetLastError());
}

template <int AUXL, int AUXS>
int fold_buf(T *out, const FoldPtrs &ins, size_t n, hipStream_t st, unsigned lds = 0)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), 1);
    hipLaunchKernelGGL((k_fold_buf<T, OP, 8, AUXL, AUXS>), dim3(grid_for(g, kNoCap)), dim3(kThreads), lds, st,
                       out, ins, g);
    return hip_ok(hipGetLastError());
}

template <int U>
int fold_lc(T *out, const FoldPtrs &ins, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(T), U);
    hipLaunchKernelGGL((k_fold_lc<T, OP, 8, SOSX_ORDER_LINEAR, U>), dim3(grid_for(g, kNoCap)),
                       dim3(kThreads), 0, st, out, ins, g);
    return hip_ok(hipGetLastError());
}

const char *const kFoldNames[] = {"u1", "u2", "u4", "st4", "st16", "xcd", "st4_pf", "st16_pf_xcd",
                                  "lc2", "lc4", "u1_occ4", "u1_occ2", "u2_occ4", "buf_nt_st_sc1",
                                  "buf_nt_st_nt", "buf_sc1_occ4", "buf_sc1_occ2", "u1_occ3"};
constexpr int kNumFold = 18;

const char *const kPrefixNames[] = {"u1_nt", "u2_nt", "u4_nt", "u1_plain", "u2_plain", "u8_nt",
                                    "split2_nt", "split2_seed_plain", "lc2", "lc4", "u1_occ4",
                                    "u1_occ2", "buf_nt_st_sc1", "buf_nt_st_nt", "u1_occ3",
                                    "buf_sc1_occ2"};
constexpr int kNumPrefix = 16;

// Continuation of a prefix from a seed vector: out[k] = seed OP in[0] OP ... OP in[k],
// left to right, so the second half of a split prefix is bit-identical to the fused one
// (the running value is always the left operand, as in SOS scan_ring,
// src/collectives.c:1188-1196).  The seed is read once and not stored.
template <class T, class OP, int NP, bool NT, bool SEED_NT>
__global__ __launch_bounds__(kThreads) void k_prefix_seeded(const T *seed, PrefixPtrs p, Geom g)
{
    constexpr int V = Pack<T>::N;
    for (size_t t = blockIdx.x; t < g.tiles; t += gridDim.x) {
        const size_t i = t * (size_t)kThreads + threadIdx.x;
        u32x4 acc = ldv<SEED_NT>(reinterpret_cast<const u32x4 *>(seed + g.head) + i);
        u32x4 x[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k)
            x[k] = ldv<NT>(reinterpret_cast<const u32x4 *>((const T *)p.in[k] + g.head) + i);
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            acc = apply<T, OP>(acc, x[k]);
            stv<NT>(reinterpret_cast<u32x4 *>((T *)p.out[k] + g.head) + i, acc);
        }
    }
    if (g.has_rem && blockIdx.x == gridDim.x - 1) {
        auto one = [&](size_t i) {
            T acc = seed[i];
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                acc = OP::f(acc, ((const T *)p.in[k])[i]);
                ((T *)p.out[k])[i] = acc;
            }
        };
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) one(i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            one(i);
    }
}

// Split prefix: a fused prefix over the first H = NP/2 inputs, then a seeded prefix over
// the rest, continuing from out[H-1].  Two 2H- and (2(NP-H)+1)-stream passes instead of one
// 2NP-stream pass: 1/(2NP) more bytes, fewer concurrent DRAM streams per kernel.
template <int NP, bool SEED_NT>
int prefix_split2(const PrefixPtrs &p, size_t n, hipStream_t st)
{
    constexpr int H = NP / 2;
    PrefixPtrs a, b;
    memset(&a, 0, sizeof(a));
    memset(&b, 0, sizeof(b));
    for (int k = 0; k < H; ++k) {
        a.in[k] = p.in[k];
        a.out[k] = p.out[k];
    }
    for (int k = H; k < NP; ++k) {
        b.in[k - H] = p.in[k];
        b.out[k - H] = p.out[k];
    }
    Geom g = make_geom((uintptr_t)p.out[0], n, sizeof(T), 1);
    hipLaunchKernelGGL((k_prefix<T, OP, H, 1, true>), dim3(grid_for(g, kNoCap)), dim3(kThreads), 0,
                       st, a, g);
    hipLaunchKernelGGL((k_prefix_seeded<T, OP, NP - H, true, SEED_NT>), dim3(grid_for(g, kNoCap)),
                       dim3(kThreads), 0, st, (const T *)p.out[H - 1], b, g);
    return hip_ok(hipGetLastError());
}

template <int NP, int U, bool NT>
int prefix_u(const PrefixPtrs &p, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)p.out[0], n, sizeof(T), U);
    hipLaunchKernelGGL((k_prefix<T, OP, NP, U, NT>), dim3(grid_for(g, kNoCap)), dim3(kThreads), 0,
                       st, p, g);
    return hip_ok(hipGetLastError());
}

template <int NP, int U>
int prefix_lc(const PrefixPtrs &p, size_t n, hipStream_t st)
{
    Geom g = make_geom((uintptr_t)p.out[0], n, sizeof(T), U);
    hipLaunchKernelGGL((k_prefix_lc<T, OP, NP, U>), dim3(grid_for(g, kNoCap)), dim3(kThreads), 0, st, p, g);
    return hip_ok(hipGetLastError());
}

template <int NP, int AUXL, int AUXS>
int prefix_buf(const PrefixPtrs &p, size_t n, hipStream_t st, unsigned lds = 0)
{
    Geom g = make_geom((uintptr_t)p.out[0], n, sizeof(T), 1);
    hipLaunchKernelGGL((k_prefix_buf<T, OP, NP, AUXL, AUXS>), dim3(grid_for(g, kNoCap)), dim3(kThreads), lds,
                       st, p, g);
    return hip_ok(hipGetLastError());
}

template <int NP>
int prefix_lds(const PrefixPtrs &p, size_t n, hipStream_t st, unsigned lds)
{
    Geom g = make_geom((uintptr_t)p.out[0], n, sizeof(T), 1);
    hipLaunchKernelGGL((k_prefix<T, OP, NP, 1, true>), dim3(grid_for(g, kNoCap)), dim3(kThreads), lds,
                       st, p, g);
    return hip_ok(hipGetLastError());
}

template <int NP>
int prefix_np(int v, const PrefixPtrs &p, size_t n, hipStream_t st)
{
    switch (v) {
        case 8: return prefix_lc<NP, 2>(p, n, st);
        case 9: return prefix_lc<NP, 4>(p, n, st);
        case 10: return prefix_lds<NP>(p, n, st, 40 << 10);
        case 11: return prefix_lds<NP>(p, n, st, 64 << 10);
        case 12: return prefix_buf<NP, 2, 16>(p, n, st);
        case 13: return prefix_buf<NP, 2, 2>(p, n, st);
        case 14: return prefix_lds<NP>(p, n, st, 48 << 10);
        case 15: return prefix_buf<NP, 2, 16>(p, n, st, 64 << 10);
        case 0: return prefix_u<NP, 1, true>(p, n, st);
        case 1: return prefix_u<NP, 2, true>(p, n, st);
        case 2: return prefix_u<NP, 4, true>(p, n, st);
        case 3: return prefix_u<NP, 1, false>(p, n, st);
        case 4: return prefix_u<NP, 2, false>(p, n, st);
        case 5: return prefix_u<NP, 8, true>(p, n, st);
        case 6: return prefix_split2<NP, true>(p, n, st);
        case 7: return prefix_split2<NP, false>(p, n, st);
    }
    return SOSX_ERR_ARG;
}

bool congruent16(const void *const *ps, int k, uintptr_t o)
{
    for (int i = 0; i < k; ++i)
        if ((((uintptr_t)ps[i]) ^ o) & 15) return false;
    return (o % sizeof(T)) == 0;
}

}  // namespace

// Ping-pong probe of a resident ("service") kernel: one lane polls a request word in
// pinned host memory and answers in another; the host measures the round trip.  Exits on
// `stop`, or after `idle_ticks` of the device wall clock without a request (every wave
// reaches the exit), storing `exited` last.
struct PingCtl {
    uint64_t req, done, stop, exited;
};

__global__ __launch_bounds__(64) void k_ping_service(PingCtl *c, long long idle_ticks, int nap)
{
    if (threadIdx.x != 0) return;
    uint64_t last = 0;
    long long t_idle = wall_clock64();
    while (true) {
        const uint64_t r = __hip_atomic_load(&c->req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (r != last) {
            last = r;
            __hip_atomic_store(&c->done, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            t_idle = wall_clock64();
            continue;
        }
        if (__hip_atomic_load(&c->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
        if (wall_clock64() - t_idle > idle_ticks) break;
        if (nap) __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(&c->exited, (uint64_t)1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The same with the request word where the kernel polls it (device memory the host
// writes over the link) and the answer where the host polls it (pinned host memory).
__global__ __launch_bounds__(64) void k_ping_split(uint64_t *req, uint64_t *ans, long long idle_ticks)
{
    if (threadIdx.x != 0) return;
    uint64_t last = 0;
    long long t_idle = wall_clock64();
    while (true) {
        const uint64_t r = __hip_atomic_load(req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (r == ~0ull) break;  // stop
        if (r != last) {
            last = r;
            __hip_atomic_store(ans, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            t_idle = wall_clock64();
            continue;
        }
        if (wall_clock64() - t_idle > idle_ticks) break;
    }
    __hip_atomic_store(ans + 1, (uint64_t)1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Stream ceilings (tools/stream_ceiling.py): the same tile shape as k_combine3 (one 16-B
// vector per lane per stream, nontemporal, one tile per workgroup) with R read streams and
// W write streams: R=1,W=0 read-only (the lanes' xor is stored only when impossible, so
// the loads stay), R=0,W=1 write-only, R=1,W=1 copy, R=2,W=1 the combine's shape.
template <int R, int W>
__global__ __launch_bounds__(kThreads) void k_stream(u32x4 *out, const u32x4 *a, const u32x4 *b, size_t nvec,
                                                     unsigned never)
{
    const size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= nvec) return;
    u32x4 x = {0u, 0u, 0u, 0u};
    if constexpr (R >= 1) x = __builtin_nontemporal_load(a + i);
    if constexpr (R >= 2) {
        const u32x4 y = __builtin_nontemporal_load(b + i);
        x = x ^ y;
    }
    if constexpr (W >= 1) {
        if constexpr (R == 0) x = u32x4{(unsigned)i, 1u, 2u, 3u};
        __builtin_nontemporal_store(x, out + i);
    } else {
        if (x[0] == never && x[1] == never && x[2] == never && x[3] == never) out[i] = x;
    }
}

// The product's 8-input fp32-sum LINEAR fold with a fast path: the chain of plain IEEE
// adds first; only when a lane of the wave ends in NaN, the exact chain with the x86 NaN
// rules (bit-exact either way: NaN is absorbing for +).  Same tile shape and cap as
// k_fold<float, OpSum, 8, LINEAR, 1>; the A/B of tools/stream_ceiling.py --multi.
__global__ __launch_bounds__(kThreads) void k_fold_fast8(float *out, FoldPtrs ins, Geom g)
{
    u32x4 *O = reinterpret_cast<u32x4 *>(out + g.head);
    for (size_t t = blockIdx.x; t < g.tiles; t += gridDim.x) {
        const size_t i = t * (size_t)kThreads + threadIdx.x;
        u32x4 x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = ldv<true>(reinterpret_cast<const u32x4 *>((const float *)ins.p[k] + g.head) + i);
        float r[4];
        bool nan = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float acc = __builtin_bit_cast(float, x[0][j]);
#pragma unroll
            for (int k = 1; k < 8; ++k) acc = acc + __builtin_bit_cast(float, x[k][j]);
            r[j] = acc;
            nan |= __builtin_isnan(acc);
        }
        u32x4 v = {__builtin_bit_cast(unsigned, r[0]), __builtin_bit_cast(unsigned, r[1]),
                   __builtin_bit_cast(unsigned, r[2]), __builtin_bit_cast(unsigned, r[3])};
        if (__builtin_expect(__any(nan), 0)) v = fold_pack<float, OpSum, 8, SOSX_ORDER_LINEAR>(x);
        stv<true>(O + i, v);
    }
}

// Multi-stream ceilings: R read streams, W write streams (1 or R), one vector per lane
// per stream: W == 1 the fold's shape (xor of the R reads), W == R the prefix's (running
// xor stored after each read), no arithmetic cost to speak of.
struct StreamPtrs {
    const u32x4 *in[8];
    u32x4 *out[8];
};

template <int R, int W>
__global__ __launch_bounds__(kThreads) void k_mstream(StreamPtrs p, size_t nvec)
{
    const size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= nvec) return;
    u32x4 x[R];
#pragma unroll
    for (int k = 0; k < R; ++k) x[k] = __builtin_nontemporal_load(p.in[k] + i);
    u32x4 acc = x[0];
    if constexpr (W == R) __builtin_nontemporal_store(acc, p.out[0] + i);
#pragma unroll
    for (int k = 1; k < R; ++k) {
        acc = acc ^ x[k];
        if constexpr (W == R) __builtin_nontemporal_store(acc, p.out[k] + i);
    }
    if constexpr (W == 1) __builtin_nontemporal_store(acc, p.out[0] + i);
}

extern "C" {

// 8 reads + 1 write (wide = 0) or 8 reads + 8 writes (wide = 1), under `lds` bytes of
// unused dynamic LDS (the product's occupancy cap: 48 KiB -> 3, 64 KiB -> 2 per CU).
int sosxv_mstream(int wide, void *const *outs, const void *const *ins, size_t nvec, unsigned lds, void *stream)
{
    StreamPtrs p;
    for (int k = 0; k < 8; ++k) {
        p.in[k] = (const u32x4 *)ins[k];
        p.out[k] = (u32x4 *)outs[wide ? k : 0];
    }
    const unsigned blocks = (unsigned)((nvec + kThreads - 1) / kThreads);
    if (wide) hipLaunchKernelGGL((k_mstream<8, 8>), dim3(blocks), dim3(kThreads), lds, as_stream(stream), p, nvec);
    else hipLaunchKernelGGL((k_mstream<8, 1>), dim3(blocks), dim3(kThreads), lds, as_stream(stream), p, nvec);
    return hip_ok(hipGetLastError());
}

// The fast-path fold above over n fp32 elements (16-B aligned, n a multiple of 1024),
// under `lds` bytes of unused dynamic LDS.
int sosxv_fold_fast8(void *out, const void *const *ins, size_t n, unsigned lds, void *stream)
{
    FoldPtrs p;
    memset(&p, 0, sizeof(p));
    for (int k = 0; k < 8; ++k) p.p[k] = ins[k];
    Geom g = make_geom((uintptr_t)out, n, sizeof(float), 1);
    if (g.head || g.has_rem) return SOSX_ERR_ARG;
    hipLaunchKernelGGL(k_fold_fast8, dim3(grid_for(g, kNoCap)), dim3(kThreads), lds, as_stream(stream),
                       (float *)out, p, g);
    return hip_ok(hipGetLastError());
}

// kind 0 read-only, 1 write-only, 2 copy, 3 two reads + one write; nvec 16-B vectors.
int sosxv_stream(int kind, void *out, const void *a, const void *b, size_t nvec, void *stream)
{
    const unsigned blocks = (unsigned)((nvec + kThreads - 1) / kThreads);
    const hipStream_t st = as_stream(stream);
    u32x4 *o = (u32x4 *)out;
    const u32x4 *x = (const u32x4 *)a, *y = (const u32x4 *)b;
    switch (kind) {
        case 0: hipLaunchKernelGGL((k_stream<1, 0>), dim3(blocks), dim3(kThreads), 0, st, o, x, y, nvec, 0x9E3779B9u); break;
        case 1: hipLaunchKernelGGL((k_stream<0, 1>), dim3(blocks), dim3(kThreads), 0, st, o, x, y, nvec, 0u); break;
        case 2: hipLaunchKernelGGL((k_stream<1, 1>), dim3(blocks), dim3(kThreads), 0, st, o, x, y, nvec, 0u); break;
        case 3: hipLaunchKernelGGL((k_stream<2, 1>), dim3(blocks), dim3(kThreads), 0, st, o, x, y, nvec, 0u); break;
        default: return SOSX_ERR_ARG;
    }
    return hip_ok(hipGetLastError());
}

int sosxv_ping_split_launch(void *req, void *ans, long long idle_ticks, void *stream)
{
    hipLaunchKernelGGL(k_ping_split, dim3(1), dim3(64), 0, as_stream(stream), (uint64_t *)req, (uint64_t *)ans,
                       idle_ticks);
    return hip_ok(hipGetLastError());
}

int sosxv_ping_launch(void *ctl, long long idle_ticks, int nap, void *stream)
{
    hipLaunchKernelGGL(k_ping_service, dim3(1), dim3(64), 0, as_stream(stream), (PingCtl *)ctl, idle_ticks, nap);
    return hip_ok(hipGetLastError());
}


// The 8-input LINEAR fp32-sum fold with inputs at other 16-B offsets, realign shape
// `mode` (k_fold_realign_v; 0 = the product's k_fold_realign_np loads).
int sosxv_fold_realign(int mode, void *out, const void *const *ins, size_t n, void *stream)
{
    Geom g = make_geom((uintptr_t)out, n, sizeof(float), 1);
    FoldRealignArgs a;
    memset(&a, 0, sizeof(a));
    a.np = 8;
    for (int k = 0; k < 8; ++k) {
        a.p[k] = ins[k];
        a.d[k] = (unsigned)((uintptr_t)((const float *)ins[k] + g.head) & 15);
        if ((uintptr_t)ins[k] % sizeof(float)) return SOSX_ERR_ARG;
    }
    const hipStream_t st = as_stream(stream);
    const dim3 grid(grid_for(g, kNoCap)), blk(kThreads);
    switch (mode) {
        case 0: hipLaunchKernelGGL((k_fold_realign_v<float, OpSum, 8, SOSX_ORDER_LINEAR, 0>), grid, blk, 0, st, (float *)out, a, g); break;
        case 1: hipLaunchKernelGGL((k_fold_realign_v<float, OpSum, 8, SOSX_ORDER_LINEAR, 1>), grid, blk, 0, st, (float *)out, a, g); break;
        case 2: hipLaunchKernelGGL((k_fold_realign_v<float, OpSum, 8, SOSX_ORDER_LINEAR, 2>), grid, blk, 0, st, (float *)out, a, g); break;
        case 3: hipLaunchKernelGGL((k_fold_realign_v<float, OpSum, 8, SOSX_ORDER_LINEAR, 3>), grid, blk, 0, st, (float *)out, a, g); break;
        case 4: hipLaunchKernelGGL((k_fold_realign_v<float, OpSum, 8, SOSX_ORDER_LINEAR, 4>), grid, blk, 0, st, (float *)out, a, g); break;
        case 5: hipLaunchKernelGGL((k_fold_realign_v<float, OpSum, 8, SOSX_ORDER_LINEAR, 5>), grid, blk, 0, st, (float *)out, a, g); break;
        case 6: hipLaunchKernelGGL((k_fold_realign_v<float, OpSum, 8, SOSX_ORDER_LINEAR, 6>), grid, blk, 0, st, (float *)out, a, g); break;
        case 7: hipLaunchKernelGGL((k_fold_realign_v<float, OpSum, 8, SOSX_ORDER_LINEAR, 7>), grid, blk, 0, st, (float *)out, a, g); break;
        case 8: hipLaunchKernelGGL((k_fold_realign_v<float, OpSum, 8, SOSX_ORDER_LINEAR, 8>), grid, blk, 0, st, (float *)out, a, g); break;
        case 9: hipLaunchKernelGGL((k_fold_realign_v<float, OpSum, 8, SOSX_ORDER_LINEAR, 9>), grid, blk, 0, st, (float *)out, a, g); break;
        case 10: hipLaunchKernelGGL((k_fold_realign_v<float, OpSum, 8, SOSX_ORDER_LINEAR, 10>), grid, blk, 0, st, (float *)out, a, g); break;
        default: return SOSX_ERR_ARG;
    }
    return hip_ok(hipGetLastError());
}

int sosxv_num_combine(void) { return kNumCombine; }
const char *sosxv_combine_name(int v) { return v >= 0 && v < kNumCombine ? kCombineNames[v] : ""; }

// out = a + b over n fp32 elements (out may alias a); operands 16-B congruent.
int sosxv_combine(int v, float *out, const float *a, const float *b, size_t n, void *stream)
{
    hipStream_t st = as_stream(stream);
    const void *ps[2] = {a, b};
    if (v < 0 || v >= kNumCombine || !out || !a || !b || !congruent16(ps, 2, (uintptr_t)out))
        return SOSX_ERR_ARG;
    if (n == 0) return SOSX_OK;
    switch (v) {
        case 0: return combine_vec<1, true, true>(out, a, b, n, st, kNoCap);
        case 1: return combine_vec<4, true, true>(out, a, b, n, st, kNoCap);
        case 2: return combine_vec<2, true, true>(out, a, b, n, st, kNoCap);
        case 3: return combine_vec<8, true, true>(out, a, b, n, st, kNoCap);
        case 4: return combine_vec<4, true, false>(out, a, b, n, st, kNoCap);
        case 5: return combine_vec<4, false, false>(out, a, b, n, st, kNoCap);
        case 6: return combine_vec<1, false, false>(out, a, b, n, st, kNoCap);
        case 7: return combine_vec<4, true, true>(out, a, b, n, st, 4096);
        case 8: return combine_vec<2, true, true>(out, a, b, n, st, 2048);
        case 9: {
            Geom g = make_geom((uintptr_t)out, n, sizeof(T), 4);
            hipLaunchKernelGGL((k_combine3_lds<T, OP, 4>), dim3(grid_for(g, kNoCap)), dim3(kThreads),
                               0, st, out, a, b, g);
            return hip_ok(hipGetLastError());
        }
        case 10: return combine_buf<4, 2, 2>(out, a, b, n, st);
        case 11: return combine_buf<4, 0, 2>(out, a, b, n, st);
        case 12: return combine_buf<4, 18, 18>(out, a, b, n, st);
        case 13: return combine_buf<2, 2, 2>(out, a, b, n, st);
        case 14: return combine_buf<1, 2, 2>(out, a, b, n, st);
        case 15: return combine_x<256, 1>(out, a, b, n, st);
        case 16: return combine_x<512, 0>(out, a, b, n, st);
        case 17: return combine_x<1024, 0>(out, a, b, n, st);
        case 18: return combine_x<512, 1>(out, a, b, n, st);
        case 19: return combine_x<256, 0>(out, a, b, n, st);
        case 20: {
            Geom g = make_geom((uintptr_t)out, n, sizeof(T), 1);
            hipLaunchKernelGGL((k_combine3_h<T, OP>), dim3(grid_for(g, kNoCap)), dim3(kThreads), 0, st,
                               out, a, b, g);
            return hip_ok(hipGetLastError());
        }
        case 21: return combine_vec<1, true, true>(out, a, b, n, st, kNoCap, 40 << 10);
        case 22: return combine_vec<1, true, true>(out, a, b, n, st, kNoCap, 48 << 10);
        case 23: return combine_vec<1, true, true>(out, a, b, n, st, kNoCap, 64 << 10);
        case 24: return combine_vec<2, true, true>(out, a, b, n, st, kNoCap, 40 << 10);
    }
    return SOSX_ERR_ARG;
}

int sosxv_num_fold(void) { return kNumFold; }
const char *sosxv_fold_name(int v) { return v >= 0 && v < kNumFold ? kFoldNames[v] : ""; }

// out = ((ins[0] + ins[1]) + ...) + ins[7] over n fp32 elements (the ring's LINEAR fold).
int sosxv_fold(int v, float *out, const void *const *ins, size_t n, void *stream)
{
    hipStream_t st = as_stream(stream);
    if (v < 0 || v >= kNumFold || !out || !ins || !congruent16(ins, 8, (uintptr_t)out))
        return SOSX_ERR_ARG;
    if (n == 0) return SOSX_OK;
    FoldPtrs fp;
    memset(&fp, 0, sizeof(fp));
    for (int k = 0; k < 8; ++k) fp.p[k] = ins[k];
    switch (v) {
        case 0: return fold_u<8, 1>(out, fp, n, st);
        case 1: return fold_u<8, 2>(out, fp, n, st);
        case 2: return fold_u<8, 4>(out, fp, n, st);
        case 3: return fold_st<4, false, false>(out, fp, n, st);
        case 4: return fold_st<16, false, false>(out, fp, n, st);
        case 5: return fold_st<1, false, true>(out, fp, n, st);
        case 6: return fold_st<4, true, false>(out, fp, n, st);
        case 7: return fold_st<16, true, true>(out, fp, n, st);
        case 8: return fold_lc<2>(out, fp, n, st);
        case 9: return fold_lc<4>(out, fp, n, st);
        case 10: return fold_u_lds<8, 1>(out, fp, n, st, 40 << 10);
        case 11: return fold_u_lds<8, 1>(out, fp, n, st, 64 << 10);
        case 12: return fold_u_lds<8, 2>(out, fp, n, st, 40 << 10);
        case 13: return fold_buf<2, 16>(out, fp, n, st);
        case 14: return fold_buf<2, 2>(out, fp, n, st);
        case 15: return fold_buf<2, 16>(out, fp, n, st, 40 << 10);
        case 16: return fold_buf<2, 16>(out, fp, n, st, 64 << 10);
        case 17: return fold_u_lds<8, 1>(out, fp, n, st, 48 << 10);
    }
    return SOSX_ERR_ARG;
}

int sosxv_num_prefix(void) { return kNumPrefix; }
const char *sosxv_prefix_name(int v) { return v >= 0 && v < kNumPrefix ? kPrefixNames[v] : ""; }

// outs[k] = ins[0] + ... + ins[k], k < np (2..8), over n fp32 elements.
int sosxv_prefix(int v, void *const *outs, const void *const *ins, int np, size_t n, void *stream)
{
    hipStream_t st = as_stream(stream);
    if (v < 0 || v >= kNumPrefix || np < 2 || np > 8 || !outs || !ins) return SOSX_ERR_ARG;
    const uintptr_t o = (uintptr_t)outs[0];
    if (!congruent16(ins, np, o) || !congruent16((const void *const *)outs, np, o)) return SOSX_ERR_ARG;
    if (n == 0) return SOSX_OK;
    PrefixPtrs pp;
    memset(&pp, 0, sizeof(pp));
    for (int k = 0; k < np; ++k) {
        pp.in[k] = ins[k];
        pp.out[k] = outs[k];
    }
    switch (np) {
        case 2: return prefix_np<2>(v, pp, n, st);
        case 3: return prefix_np<3>(v, pp, n, st);
        case 4: return prefix_np<4>(v, pp, n, st);
        case 5: return prefix_np<5>(v, pp, n, st);
        case 6: return prefix_np<6>(v, pp, n, st);
        case 7: return prefix_np<7>(v, pp, n, st);
        case 8: return prefix_np<8>(v, pp, n, st);
    }
    return SOSX_ERR_ARG;
}

}  // extern "C"
