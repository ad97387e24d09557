// elementwise.h -- shared device code for the SOS combine/fold kernels (gfx950).
//
// Element semantics follow src/shmem_internal_op.h exactly: OP::f(out, in) is
// calc(*out, *in) of FUNC_OP_CREATE (:23-33) with the op macros of :37-43.
//   * min/max are the ternaries (a)<(b)?(a):(b) / (a)>(b)?(a):(b): they return the
//     right operand (`in`) on ties and on any unordered compare -- NOT fmin/fmax
//     (hipcc lowers them to v_cmp + v_cndmask, checked in the .s);
//   * integer sum/prod wrap (computed in unsigned arithmetic, no UB);
//   * fp math is IEEE with no contraction (#pragma clang fp contract(off) and
//     -ffp-contract=off), fp32 denormals kept (hipcc default mode on gfx950);
//   * complex prod is GCC's inline (ac-bd) + (ad+bc)i plus libgcc's Annex G
//     recovery (__mulsc3/__muldc3) when both parts come out NaN.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <type_traits>

#include "carry.h"
#include "dtypes.h"
#include "ldbl.h"
#include "sosx.h"

#pragma clang fp contract(off)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

namespace sos {

struct cf32 { float re, im; };
struct cf64 { double re, im; };

// ---------------------------------------------------------------------------------
// Element operations: OP::f(out, in) == calc(*out, *in) of src/shmem_internal_op.h
// ---------------------------------------------------------------------------------
template <class T> struct wide { using type = T; };
template <> struct wide<uint8_t> { using type = uint32_t; };
template <> struct wide<uint16_t> { using type = uint32_t; };
template <> struct wide<int8_t> { using type = uint32_t; };
template <> struct wide<int16_t> { using type = uint32_t; };

// Annex G recovery exactly as libgcc's __mulsc3/__muldc3 (C99 G.5.1), called by
// GCC's inline complex multiply only when both parts of the naive product are NaN.
template <class F> __device__ __forceinline__ F csign(F m, F s)
{
    if constexpr (sizeof(F) == 4) return __builtin_copysignf(m, s);
    else return __builtin_copysign(m, s);
}

// x86 SSE NaN rule for `first + second` (Intel SDM vol.1 table 4-7): a NaN first
// operand wins, else a NaN second operand, both returned quieted; an invalid operation
// on non-NaN inputs returns the default NaN (sign set: 0xFFC00000 / 0xFFF8...).
template <class F> __device__ __forceinline__ F x86_nan(F r, F first, F second)
{
    using I = typename std::conditional<sizeof(F) == 4, uint32_t, uint64_t>::type;
    constexpr I qbit = sizeof(F) == 4 ? (I)0x00400000u : (I)0x0008000000000000ull;
    constexpr I dnan = sizeof(F) == 4 ? (I)0xFFC00000u : (I)0xFFF8000000000000ull;
    if (__builtin_isnan(r)) {
        I bits = __builtin_isnan(first)    ? (__builtin_bit_cast(I, first) | qbit)
                 : __builtin_isnan(second) ? (__builtin_bit_cast(I, second) | qbit)
                                           : dnan;
        r = __builtin_bit_cast(F, bits);
    }
    return r;
}
template <class F> __device__ __forceinline__ F x86_add(F first, F second)
{
    return x86_nan(first + second, first, second);
}
template <class F> __device__ __forceinline__ F x86_mul(F first, F second)
{
    return x86_nan(first * second, first, second);
}

template <class F>
__device__ __forceinline__ void cmul(F a, F b, F c, F d, F &x, F &y)
{
    F ac = a * c, bd = b * d, ad = a * d, bc = b * c;
    x = ac - bd;
    y = ad + bc;
    if (__builtin_expect(__builtin_isnan(x) && __builtin_isnan(y), 0)) {
        bool recalc = false;
        const F one = F(1), zero = F(0), inf = F(__builtin_inf());
        if (__builtin_isinf(a) || __builtin_isinf(b)) {
            a = csign<F>(__builtin_isinf(a) ? one : zero, a);
            b = csign<F>(__builtin_isinf(b) ? one : zero, b);
            if (__builtin_isnan(c)) c = csign<F>(zero, c);
            if (__builtin_isnan(d)) d = csign<F>(zero, d);
            recalc = true;
        }
        if (__builtin_isinf(c) || __builtin_isinf(d)) {
            c = csign<F>(__builtin_isinf(c) ? one : zero, c);
            d = csign<F>(__builtin_isinf(d) ? one : zero, d);
            if (__builtin_isnan(a)) a = csign<F>(zero, a);
            if (__builtin_isnan(b)) b = csign<F>(zero, b);
            recalc = true;
        }
        if (!recalc && (__builtin_isinf(ac) || __builtin_isinf(bd) || __builtin_isinf(ad) ||
                        __builtin_isinf(bc))) {
            if (__builtin_isnan(a)) a = csign<F>(zero, a);
            if (__builtin_isnan(b)) b = csign<F>(zero, b);
            if (__builtin_isnan(c)) c = csign<F>(zero, c);
            if (__builtin_isnan(d)) d = csign<F>(zero, d);
            recalc = true;
        }
        if (recalc) {
            x = inf * (a * c - b * d);
            y = inf * (a * d + b * c);
        }
    }
}

struct OpAnd {
    template <class T> __device__ __forceinline__ static T f(T a, T b) { return (T)(a & b); }
};
struct OpOr {
    template <class T> __device__ __forceinline__ static T f(T a, T b) { return (T)(a | b); }
};
struct OpXor {
    template <class T> __device__ __forceinline__ static T f(T a, T b) { return (T)(a ^ b); }
};
// (a) > (b) ? (a) : (b) -- returns `in` on ties and whenever a compare is unordered.
// long double: the chosen operand's 10 value bytes, the left operand's padding.
struct OpMax {
    template <class T> __device__ __forceinline__ static T f(T a, T b) { return a > b ? a : b; }
    __device__ __forceinline__ static ld80 f(ld80 a, ld80 b)
    {
        const ld80 &c = x87::gt(a, b) ? a : b;
        return x87::make(a, x87::se(c), c.m);
    }
};
struct OpMin {
    template <class T> __device__ __forceinline__ static T f(T a, T b) { return a < b ? a : b; }
    __device__ __forceinline__ static ld80 f(ld80 a, ld80 b)
    {
        const ld80 &c = x87::gt(b, a) ? a : b;  // (a) < (b) ? (a) : (b)
        return x87::make(a, x87::se(c), c.m);
    }
};
struct OpSum {
    template <class T> __device__ __forceinline__ static T f(T a, T b)
    {
        if constexpr (std::is_integral<T>::value) {
            using W = typename wide<T>::type;
            using U = typename std::make_unsigned<W>::type;
            return (T)((U)a + (U)b);
        } else {
            // gcc -O2: `addss in, out` -- the inout operand is SSE's first operand, whose
            // NaN wins; hipcc may commute a plain fadd, so the rule is explicit
            return x86_add(a, b);
        }
    }
    // gcc -O2 (x86-64) emits `addss in.re -> out.re` and `addss out.im -> in.im` for the
    // complex add of src/shmem_internal_op.h:219-223, and SSE returns its FIRST operand's
    // (quieted) NaN when both are NaN; x86_add reproduces that choice explicitly, since
    // hipcc is free to commute the operands of a plain fadd.
    __device__ __forceinline__ static cf32 f(cf32 a, cf32 b)
    {
        return cf32{x86_add(a.re, b.re), x86_add(b.im, a.im)};
    }
    __device__ __forceinline__ static cf64 f(cf64 a, cf64 b)
    {
        return cf64{x86_add(a.re, b.re), x86_add(b.im, a.im)};
    }
    __device__ __forceinline__ static ld80 f(ld80 a, ld80 b) { return x87::add(a, b); }
};
struct OpProd {
    template <class T> __device__ __forceinline__ static T f(T a, T b)
    {
        if constexpr (std::is_integral<T>::value) {
            using W = typename wide<T>::type;
            using U = typename std::make_unsigned<W>::type;
            return (T)((U)a * (U)b);
        } else {
            return x86_mul(a, b);  // `mulss in, out`: first-operand NaN rule as for sum
        }
    }
    __device__ __forceinline__ static cf32 f(cf32 a, cf32 b)
    {
        cf32 r;
        cmul<float>(a.re, a.im, b.re, b.im, r.re, r.im);
        return r;
    }
    __device__ __forceinline__ static cf64 f(cf64 a, cf64 b)
    {
        cf64 r;
        cmul<double>(a.re, a.im, b.re, b.im, r.re, r.im);
        return r;
    }
    __device__ __forceinline__ static ld80 f(ld80 a, ld80 b) { return x87::mul(a, b); }
};

// ---------------------------------------------------------------------------------
// 16-byte packets
// ---------------------------------------------------------------------------------
template <class T> struct Pack {
    static constexpr int N = 16 / (int)sizeof(T);
    T e[N];
};

template <class T, class OP>
__device__ __forceinline__ u32x4 apply(u32x4 a, u32x4 b)
{
    Pack<T> x = __builtin_bit_cast(Pack<T>, a);
    Pack<T> y = __builtin_bit_cast(Pack<T>, b);
#pragma unroll
    for (int j = 0; j < Pack<T>::N; ++j) x.e[j] = OP::f(x.e[j], y.e[j]);
    return __builtin_bit_cast(u32x4, x);
}

template <bool NT>
__device__ __forceinline__ u32x4 ldv(const u32x4 *p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
// A 16-B nontemporal load from an address that is only element-aligned (4 or 8 B): one
// global_load_dwordx4, which the memory pipeline splits where it straddles (ROCm runs the
// GPU in unaligned-access mode).  It reads exactly the 16 bytes asked for.
typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ u32x4 ldv_unaligned(const void *p)
{
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4u *>(p));
}

template <bool NT>
__device__ __forceinline__ void stv(u32x4 *p, u32x4 v)
{
    if constexpr (NT) {
        // The empty asm pins the value first: without it LLVM drops the !nontemporal
        // of this store when the value comes out of select chains (fp64/complex SUM/PROD
        // with the x86 NaN rule), leaving a cached store and ~12 % less HBM rate at
        // large n (profiles/r2_sweep.json).
        asm volatile("" : "+v"(v));
        __builtin_nontemporal_store(v, p);
    } else {
        *p = v;
    }
}

// The 16 bytes at offset d (1..15) of the 32-byte concatenation lo || hi: a vector of an
// operand that is not 16-B congruent with the kernel's grid, from the two aligned
// vectors its bytes straddle (v_alignbyte_b32; q = d / 4 is wave-uniform, so the dword
// choice is a uniform branch, not scratch).
__device__ __forceinline__ u32x4 realign16(const u32x4 &lo, const u32x4 &hi, unsigned d)
{
    const unsigned w[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    const unsigned q = d >> 2, r = d & 3;
    unsigned t[5];
#pragma unroll
    for (int j = 0; j < 5; ++j)
        t[j] = q == 0 ? w[j] : q == 1 ? w[j + 1] : q == 2 ? w[j + 2] : w[j + 3];
    u32x4 v;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_alignbyte(t[k + 1], t[k], r);
    return v;
}

// The 16-B vector of the next lane of the wave (lane l gets lane l + 1's; lane 63 gets
// zeros and must supply its own): four DPP wave_shl:1 moves, no LDS and no memory access.
__device__ __forceinline__ u32x4 next_lane16(const u32x4 &x)
{
    u32x4 v;
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)x[c], 0x130, 0xf, 0xf, false);
    return v;
}

constexpr int kThreads = 256;

// Geometry of one (out, a, b) or fold call, computed on the host:
//   elements [0, head)                  scalar, by the remainder workgroup
//   vectors  [0, tiles * kThreads * U)  16-B packets from element `head`
//   elements [head + tiles*kThreads*U*V, n) scalar, by the remainder workgroup
//   acquire: the launch carries the transport's consumer-side acquire (wg_acquire)
struct Geom {
    size_t n;
    size_t head;
    size_t tiles;
    int has_rem;
    int acquire;
};

// ---------------------------------------------------------------------------------
// The consumer half of the memory-visibility rule: a launch that
// reads bytes a peer published after a wait must not read lines this GPU's L2s kept from
// an earlier call.  A system-scope acquire (buffer_inv sc0 sc1) drops this CU's L1 and
// the non-local lines of its XCD's L2.  wg_acquire: lane 0 of the workgroup fences and
// waits for the invalidate; the workgroup's loads follow the barrier.  Small grids carry
// it this way (one invalidate per workgroup, no extra launch); streaming grids take the
// acquire kernel first (copy.hip k_acquire_system), since one invalidate per workgroup
// of a streaming grid costs 6x (profiles/r6_acquire_probe.txt).
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void acquire_system_lane()
{
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: buffer_inv sc0 sc1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void wg_acquire()
{
    if (threadIdx.x == 0) acquire_system_lane();
    __syncthreads();
}



constexpr size_t kNoCap = (size_t)1 << 31;  // hardware grid x-dimension limit

inline hipStream_t as_stream(void *s) { return (hipStream_t)s; }
inline int hip_ok(hipError_t e) { return e == hipSuccess ? SOSX_OK : SOSX_ERR_HIP; }

// Plan the vector geometry of a call over `n` elements of size `s` whose pointers all
// share `addr0 % 16`.  U = 16-B vectors per lane per tile.
inline Geom make_geom(uintptr_t addr0, size_t n, size_t s, int U)
{
    Geom g;
    g.n = n;
    size_t mis = addr0 & 15;
    size_t head = mis ? (16 - mis) / s : 0;
    if (head > n) head = n;
    g.head = head;
    const size_t V = 16 / s;
    const size_t nvec = (n - head) / V;
    g.tiles = nvec / (size_t)(kThreads * U);
    g.has_rem = (head > 0) || (g.tiles * (size_t)(kThreads * U) * V != n - head);
    g.acquire = 0;
    return g;
}

inline unsigned grid_for(const Geom &g, size_t cap)
{
    size_t blocks = g.tiles < cap ? g.tiles : cap;
    if (g.has_rem) blocks += 1;
    if (blocks == 0) blocks = 1;
    return (unsigned)blocks;
}

// Map (op, dtype) onto a storage type and op functor and invoke F::run<T, OP>(args...).
template <class F, class... A>
inline int dispatch(int op, int dt, A... args)
{
    int rc = sos_check_op(op, dt);
    if (rc) return rc;
    const SosDtypeInfo d = sos_dtype_info(dt);
#define SOS_INT_CASES(UT, ST)                                                        \
    switch (op) {                                                                    \
        case SOSX_OP_BAND: return F::template run<UT, OpAnd>(args...);               \
        case SOSX_OP_BOR: return F::template run<UT, OpOr>(args...);                 \
        case SOSX_OP_BXOR: return F::template run<UT, OpXor>(args...);               \
        case SOSX_OP_SUM: return F::template run<UT, OpSum>(args...);                \
        case SOSX_OP_PROD: return F::template run<UT, OpProd>(args...);              \
        case SOSX_OP_MIN: return F::template run<ST, OpMin>(args...);                \
        case SOSX_OP_MAX: return F::template run<ST, OpMax>(args...);                \
    }                                                                                \
    return SOSX_ERR_OP;
#define SOS_FP_CASES(FT)                                                             \
    switch (op) {                                                                    \
        case SOSX_OP_SUM: return F::template run<FT, OpSum>(args...);                \
        case SOSX_OP_PROD: return F::template run<FT, OpProd>(args...);              \
        case SOSX_OP_MIN: return F::template run<FT, OpMin>(args...);                \
        case SOSX_OP_MAX: return F::template run<FT, OpMax>(args...);                \
    }                                                                                \
    return SOSX_ERR_OP;
    switch (d.kind) {
        case K_S8: SOS_INT_CASES(uint8_t, int8_t)
        case K_U8: SOS_INT_CASES(uint8_t, uint8_t)
        case K_S16: SOS_INT_CASES(uint16_t, int16_t)
        case K_U16: SOS_INT_CASES(uint16_t, uint16_t)
        case K_S32: SOS_INT_CASES(uint32_t, int32_t)
        case K_U32: SOS_INT_CASES(uint32_t, uint32_t)
        case K_S64: SOS_INT_CASES(uint64_t, int64_t)
        case K_U64: SOS_INT_CASES(uint64_t, uint64_t)
        case K_F32: SOS_FP_CASES(float)
        case K_F64: SOS_FP_CASES(double)
        case K_C32:
            return op == SOSX_OP_SUM ? F::template run<cf32, OpSum>(args...)
                                     : F::template run<cf32, OpProd>(args...);
        case K_C64:
            return op == SOSX_OP_SUM ? F::template run<cf64, OpSum>(args...)
                                     : F::template run<cf64, OpProd>(args...);
        case K_LDBL: SOS_FP_CASES(ld80)
        default: return SOSX_ERR_DTYPE;
    }
#undef SOS_INT_CASES
#undef SOS_FP_CASES
}

}  // namespace sos
