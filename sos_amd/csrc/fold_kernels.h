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
    if (g.acquire) wg_acquire();  // a small grid reading a peer's bytes (carry_acquire)
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
// The P-way fold (2 <= P <= 8) when some inputs are NOT 16-B congruent with the output: a
// team reduction whose source and target sit at different 16-B offsets (the PE's own
// source chunk, or the peers' sources read in place, against exchange scratch congruent
// with the target).  16-B vectors throughout, two shapes:
//   k_fold_realign_np  inputs at different offsets: an input at byte offset d[k] != 0 is
//                      read as the two aligned vectors its bytes straddle and
//                      funnel-shifted into place (realign16; see k_combine3_realign for
//                      why the extra bytes are safe to load);
//   k_fold_outshift    every input at one offset: fold in the inputs' frame, realign the
//                      output.
// LINEAR: acc = in[0] OP in[1] OP ... (the ring); TREE: the recdbl_sw tree of fold_elem
// (the extras folded into the first P - p2 leaves, then distance 1, 2, 4 pairs, the lower
// subtree the left operand).  The ragged head and tail use the runtime-P element fold.
// Round 5 (profiles/r5_fold_outshift.txt): both with P at compile time and no occupancy
// cap; the runtime-P vector kernel they replace branched per input between its loads
// (3.2-3.8 TB/s with every input incongruent, 5.7 with one).
// ---------------------------------------------------------------------------------
struct FoldRealignArgs {
    const void *p[8];
    unsigned d[8];
    int np;
};

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

// Inputs at different offsets: every input's aligned vector is loaded once; an
// incongruent input's second vector -- the next lane's first -- comes from that lane by
// DPP (next_lane16), and only the wave's last lane loads its own.  Round 5 loaded the
// second vector in every lane: with nontemporal loads L2 did not keep the line for the
// second request, so reads reached 1.30x the algorithmic bytes with 6 of 8 inputs
// incongruent (profiles/r6_realign_pmc.txt).  Over 1..8 incongruent inputs of 8 x 16Mi
// fp32 (tools/realign_ab.py, profiles/r6_realign_ab.txt) this shape is the fastest or
// within 1 % up to 6 (m = 1 6.21, m = 3 6.10, m = 6 5.64 TB/s against 6.22 / 5.68 / 5.05
// for round 5's) and 2 % behind plain double loads at 8.  UL (elements of 4 or 8 bytes,
// most inputs incongruent): one unaligned 16-B load per input and lane instead, no DPP and
// no shift -- flat at 5.84-5.95 TB/s however many inputs are incongruent, against 5.03-5.11
// for the DPP shape with all 8 at mixed offsets and 5.37-5.64 with 6 of 8
// (profiles/r6_realign_unaligned.txt); the DPP shape stays ahead up to 4 of 8.
template <class T, class OP, int NP, int ORDER, bool UL = false>
__global__ __launch_bounds__(kThreads) void k_fold_realign_np(T *out, FoldRealignArgs a, Geom g)
{
    if (g.acquire) wg_acquire();  // a small grid reading a peer's bytes (carry_acquire)
    constexpr int V = Pack<T>::N;
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
        if constexpr (UL) {
#pragma unroll
            for (int k = 0; k < NP; ++k) x[k] = ldv_unaligned(reinterpret_cast<const char *>(I[k] + i) + a.d[k]);
            stv<true>(O + i, fold_pack<T, OP, NP, ORDER>(x));
            continue;
        }
#pragma unroll
        for (int k = 0; k < NP; ++k) x[k] = ldv<true>(I[k] + i);
        if (last_lane) {  // its next vector belongs to the next wave (or workgroup)
#pragma unroll
            for (int k = 0; k < NP; ++k)
                if (a.d[k]) y[k] = ldv<true>(I[k] + i + 1);
        }
#pragma unroll
        for (int k = 0; k < NP; ++k)
            if (a.d[k]) {
                const u32x4 nx = next_lane16(x[k]);
                if (!last_lane) y[k] = nx;
                x[k] = realign16(x[k], y[k], a.d[k]);
            }
        stv<true>(O + i, fold_pack<T, OP, NP, ORDER>(x));
    }
    if (g.has_rem && blockIdx.x == nblk - 1) {
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) out[i] = fold_runtime_np_elem<T, OP, ORDER>(a, i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            out[i] = fold_runtime_np_elem<T, OP, ORDER>(a, i);
    }
}

// Every input at the SAME 16-B offset d != 0 from the output (the inputs congruent with
// one another: the p2p ring's in-place fold of the peers' sources when source and target
// sit at different offsets in the symmetric heap).  Fold in the inputs' frame, one vector
// per input per lane, and realign the OUTPUT: out vector i = realign16(F_i, F_i+1, d),
// F_i+1 taken from the next lane (DPP); the last lane of each wave folds its F_i+1 itself
// (k_fold_realign_np would load two vectors per input: 4.2-4.4 TB/s here, 5.8-6.1 this way).
// Since round 6 only 1- and 2-byte elements take it by default: 4- and 8-byte ones load
// unaligned (k_fold_realign_np UL, equal or faster at every P: profiles/r6_outshift_ab.txt).
template <class T, class OP, int NP, int ORDER>
__global__ __launch_bounds__(kThreads) void k_fold_outshift(T *out, FoldRealignArgs a, Geom g)
{
    if (g.acquire) wg_acquire();  // a small grid reading a peer's bytes (carry_acquire)
    constexpr int V = Pack<T>::N;
    const size_t nblk = gridDim.x;
    const unsigned d = a.d[0];
    const bool last_lane = (threadIdx.x & 63) == 63;
    u32x4 *O = reinterpret_cast<u32x4 *>(out + g.head);
    const u32x4 *I[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k)
        I[k] = reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>((const T *)a.p[k] + g.head) - d);
    for (size_t t = blockIdx.x; t < g.tiles; t += nblk) {
        const size_t i = t * (size_t)kThreads + threadIdx.x;
        u32x4 x[NP], y[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) x[k] = ldv<true>(I[k] + i);
        if (last_lane) {  // its F_i+1 belongs to the next wave (or workgroup)
#pragma unroll
            for (int k = 0; k < NP; ++k) y[k] = ldv<true>(I[k] + i + 1);
        }
        const u32x4 f = fold_pack<T, OP, NP, ORDER>(x);
        u32x4 nx = next_lane16(f);  // DPP (round 6; __shfl_down was an LDS bpermute)
        if (last_lane) nx = fold_pack<T, OP, NP, ORDER>(y);
        stv<true>(O + i, realign16(f, nx, d));
    }
    if (g.has_rem && blockIdx.x == nblk - 1) {
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) out[i] = fold_runtime_np_elem<T, OP, ORDER>(a, i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            out[i] = fold_runtime_np_elem<T, OP, ORDER>(a, i);
    }
}

// Occupancy cap of the multi-stream streaming kernels (round 5): a
// fold or prefix reads/writes `streams` concurrent HBM streams, and with every CU full
// (8 workgroups) the chip holds ~2048 tiles x streams open DRAM rows at once.  Reserving
// unused dynamic LDS caps the workgroups per CU (160 KiB / bytes): fewer rows open, better
// row-buffer locality.  Interleaved A/Bs over 9 random buffer layouts, twice
// (profiles/r5_multistream_ab.json): the 8-input fold (9 streams) 6.10-6.14 -> 6.29-6.35
// TB/s at 3 per CU; the 8-input prefix (16 streams) 5.75-5.87 -> 5.96-6.07 at 2 per CU;
// the 4- and 2-input prefixes (8, 4 streams) +2.5 / +1.7 % at 3 per CU.  The 3-stream
// combine loses with any cap (6.61 -> 6.31 TB/s at 3 per CU), so it has none, and neither
// do the folds of 2-4 inputs (U > 1 vectors per lane; unmeasured with a cap).
inline unsigned occupancy_lds(int streams)
{
    if (streams >= 12) return 64u << 10;  // 2 workgroups per CU
    if (streams >= 4) return 48u << 10;   // 3 per CU
    return 0;
}

// The realigning fold / prefix take the unaligned-load form (UL) when at least this many
// inputs are incongruent (elements of 4 or 8 bytes).  Bench switch SOSX_REALIGN_UNALIGNED
// = the count (1: whenever one is; 9: never); both forms are bit-exact.
inline int realign_unaligned_min()
{
    static const int m = [] {
        const char *e = getenv("SOSX_REALIGN_UNALIGNED");
        return e && *e ? atoi(e) : 5;
    }();
    return m;
}

// The fold of one element order over any (type, op) (fold_order.hip, one object per
// order); sosx_fold dispatches to them.
int fold_linear(int op, int dtype, void *out, const FoldPtrs *ins, int nin, size_t n, hipStream_t st);
int fold_tree(int op, int dtype, void *out, const FoldPtrs *ins, int nin, size_t n, hipStream_t st);

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
    if (g.acquire) wg_acquire();  // a small grid reading a peer's bytes (carry_acquire)
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
// Inputs realigned as in k_fold_realign_np; every input vector of a tile is loaded before
// the first store, as in k_prefix (an output may alias an input: the aliased pair is
// congruent, so it is never read past its own vector).
struct PrefixRealignArgs {
    const void *in[8];
    void *out[8];
    unsigned d[8];
    int np;
};

// P known at compile time (round 5, as k_fold_realign_np; it replaced a runtime-P kernel
// that branched per input between its loads, profiles/r5_fold_outshift.txt): every
// input's aligned vector (the wave's last lane also loads its incongruent inputs' next
// vectors), the other lanes' next vectors by DPP from the neighbouring lane (round 6, as
// k_fold_realign_np: round 5's second load per lane read 1.42x the algorithmic bytes,
// profiles/r6_realign_pmc.txt), then the prefix.  Every load of the tile still precedes
// the first store (aliasing, as k_prefix).  UL: unaligned loads, as k_fold_realign_np.
template <class T, class OP, int NP, bool UL = false>
__global__ __launch_bounds__(kThreads) void k_prefix_realign_np(PrefixRealignArgs a, Geom g)
{
    if (g.acquire) wg_acquire();  // a small grid reading a peer's bytes (carry_acquire)
    constexpr int V = Pack<T>::N;
    const size_t nblk = gridDim.x;
    const bool last_lane = (threadIdx.x & 63) == 63;
    const u32x4 *I[NP];
    u32x4 *O[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        I[k] = reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>((const T *)a.in[k] + g.head) - a.d[k]);
        O[k] = reinterpret_cast<u32x4 *>((T *)a.out[k] + g.head);
    }
    for (size_t t = blockIdx.x; t < g.tiles; t += nblk) {
        const size_t i = t * (size_t)kThreads + threadIdx.x;
        u32x4 x[NP], y[NP];
        if constexpr (UL) {
#pragma unroll
            for (int k = 0; k < NP; ++k) x[k] = ldv_unaligned(reinterpret_cast<const char *>(I[k] + i) + a.d[k]);
        } else {
#pragma unroll
            for (int k = 0; k < NP; ++k) x[k] = ldv<true>(I[k] + i);
            if (last_lane) {
#pragma unroll
                for (int k = 0; k < NP; ++k)
                    if (a.d[k]) y[k] = ldv<true>(I[k] + i + 1);
            }
#pragma unroll
            for (int k = 0; k < NP; ++k)
                if (a.d[k]) {
                    const u32x4 nx = next_lane16(x[k]);
                    if (!last_lane) y[k] = nx;
                    x[k] = realign16(x[k], y[k], a.d[k]);
                }
        }
        u32x4 acc = x[0];
        stv<true>(O[0] + i, acc);
#pragma unroll
        for (int k = 1; k < NP; ++k) {
            acc = apply<T, OP>(acc, x[k]);
            stv<true>(O[k] + i, acc);
        }
    }
    if (g.has_rem && blockIdx.x == nblk - 1) {
        auto one = [&](size_t i) {
            T v[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) v[k] = ((const T *)a.in[k])[i];
            T acc = v[0];
            ((T *)a.out[0])[i] = acc;
#pragma unroll
            for (int k = 1; k < NP; ++k) {
                acc = OP::f(acc, v[k]);
                ((T *)a.out[k])[i] = acc;
            }
        };
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) one(i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            one(i);
    }
}

// Every input at the SAME 16-B offset d != 0 from the (congruent) outputs: the prefix in
// the inputs' frame, each output realigned (k_fold_outshift's scheme, once per output:
// the next lane's running value by DPP (next_lane16), the last lane of a wave folding the next
// vector itself).  Aliasing as k_prefix: every load of the tile before the first store.
template <class T, class OP, int NP>
__global__ __launch_bounds__(kThreads) void k_prefix_outshift(PrefixRealignArgs a, Geom g)
{
    if (g.acquire) wg_acquire();  // a small grid reading a peer's bytes (carry_acquire)
    constexpr int V = Pack<T>::N;
    const size_t nblk = gridDim.x;
    const unsigned d = a.d[0];
    const bool last_lane = (threadIdx.x & 63) == 63;
    const u32x4 *I[NP];
    u32x4 *O[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        I[k] = reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>((const T *)a.in[k] + g.head) - d);
        O[k] = reinterpret_cast<u32x4 *>((T *)a.out[k] + g.head);
    }
    for (size_t t = blockIdx.x; t < g.tiles; t += nblk) {
        const size_t i = t * (size_t)kThreads + threadIdx.x;
        u32x4 x[NP], y[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) x[k] = ldv<true>(I[k] + i);
        if (last_lane) {
#pragma unroll
            for (int k = 0; k < NP; ++k) y[k] = ldv<true>(I[k] + i + 1);
        }
        u32x4 acc = x[0], accn = y[0];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            if (k > 0) {
                acc = apply<T, OP>(acc, x[k]);
                if (last_lane) accn = apply<T, OP>(accn, y[k]);
            }
            u32x4 nx = next_lane16(acc);
            if (last_lane) nx = accn;
            stv<true>(O[k] + i, realign16(acc, nx, d));
        }
    }
    if (g.has_rem && blockIdx.x == nblk - 1) {
        auto one = [&](size_t i) {
            T v[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) v[k] = ((const T *)a.in[k])[i];
            T acc = v[0];
            ((T *)a.out[0])[i] = acc;
#pragma unroll
            for (int k = 1; k < NP; ++k) {
                acc = OP::f(acc, v[k]);
                ((T *)a.out[k])[i] = acc;
            }
        };
        for (size_t i = threadIdx.x; i < g.head; i += kThreads) one(i);
        for (size_t i = g.head + g.tiles * (size_t)(kThreads * V) + threadIdx.x; i < g.n; i += kThreads)
            one(i);
    }
}

}  // namespace sos
