// ldbl.h -- x87 80-bit extended precision on gfx950, for SOS's long double reductions.
//
// SOS's shmem_longdouble_* reductions run `*out = *out OP *in` on x86 `long double`
// (src/shmem_internal_op.h:209-212): the x87 80-bit format (1 sign, 15 exponent bits,
// explicit integer bit + 63 fraction bits) stored in 16 bytes, evaluated by the FPU
// at 64-bit precision (Linux default precision control), round to nearest even.  There
// is no such type on the GPU, so the ops are restated in integer arithmetic here:
//   add/mul  exact product/sum in 128 bits, one RNE rounding to 64 bits, gradual
//            underflow (denormals rounded at their own position), overflow to inf;
//   min/max  the ternary compare (`a > b ? a : b`): unordered -> the right operand;
//   specials inf - inf, 0 * inf and unsupported encodings (unnormals, pseudo-NaN/inf)
//            give the x87 default NaN (0xFFFF:C000000000000000); a NaN operand is
//            returned quieted.
// The 6 padding bytes of a 16-byte long double are not written by the x87 store
// (fstpt writes 10 bytes), so results keep the left operand's padding bytes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sos {

struct ld80 {
    uint64_t m;   // significand with explicit integer bit (bit 63)
    uint64_t hi;  // bits 0..15: sign | exponent; bits 16..63: padding (untouched)
};

namespace x87 {

typedef unsigned __int128 u128;

__device__ __forceinline__ uint32_t se(const ld80 &a) { return (uint32_t)(a.hi & 0xFFFFu); }
__device__ __forceinline__ ld80 make(const ld80 &pad_from, uint32_t sexp, uint64_t m)
{
    return ld80{m, (pad_from.hi & ~(uint64_t)0xFFFF) | sexp};
}
__device__ __forceinline__ bool is_nan(const ld80 &a)
{
    return (se(a) & 0x7FFF) == 0x7FFF && (a.m >> 63) && (a.m << 1);
}
// encodings the 387+ refuses: unnormals and pseudo-NaN/pseudo-infinity
__device__ __forceinline__ bool unsupported(const ld80 &a)
{
    const uint32_t e = se(a) & 0x7FFF;
    return e != 0 && !(a.m >> 63);
}
__device__ __forceinline__ bool is_inf(const ld80 &a)
{
    return (se(a) & 0x7FFF) == 0x7FFF && a.m == 0x8000000000000000ull;
}
__device__ __forceinline__ bool is_zero(const ld80 &a) { return (se(a) & 0x7FFF) == 0 && a.m == 0; }

__device__ __forceinline__ ld80 default_nan(const ld80 &pad) { return make(pad, 0xFFFF, 0xC000000000000000ull); }

// NaN operand(s): the NaN (larger significand of two) comes back quieted.
__device__ __forceinline__ ld80 nan_result(const ld80 &a, const ld80 &b)
{
    const bool na = is_nan(a), nb = is_nan(b);
    const ld80 &w = (na && nb) ? ((b.m | (1ull << 62)) > (a.m | (1ull << 62)) ? b : a) : (na ? a : b);
    return make(a, se(w), w.m | (1ull << 62));
}

__device__ __forceinline__ int clz128(u128 x)
{
    const uint64_t h = (uint64_t)(x >> 64), l = (uint64_t)x;
    return h ? __builtin_clzll(h) : 64 + (l ? __builtin_clzll(l) : 64);
}

// value = S * 2^L (S exact, `sticky` = nonzero bits already shifted out below S).
// Normalise, round once to 64 bits (RNE), handle denormals and overflow.
__device__ __forceinline__ ld80 round_pack(const ld80 &pad, uint32_t sign, u128 S, int L, bool sticky)
{
    if (S == 0) return make(pad, sign << 15, 0);
    const int lz = clz128(S);
    S <<= lz;
    L -= lz;
    // leading one at bit 127: value = 1.xxx * 2^(L + 127); biased exponent field:
    int biased = L + 127 + 16383;
    if (biased < 1) {  // gradual underflow: shift to exponent field 0 before rounding
        const int sh = 1 - biased;
        if (sh >= 128) {
            sticky |= S != 0;
            S = 0;
        } else {
            sticky |= (S & ((((u128)1) << sh) - 1)) != 0;
            S >>= sh;
        }
        biased = 0;
    }
    uint64_t m = (uint64_t)(S >> 64);
    const uint64_t lo = (uint64_t)S;
    const bool round = (lo >> 63) & 1;
    sticky |= (lo << 1) != 0;
    if (round && (sticky || (m & 1))) {
        m += 1;
        if (m == 0) {  // carried out of 64 bits
            m = 0x8000000000000000ull;
            biased += 1;
        } else if (biased == 0 && (m >> 63)) {
            biased = 1;  // rounded up into the smallest normal
        }
    }
    if (biased >= 0x7FFF) return make(pad, (sign << 15) | 0x7FFF, 0x8000000000000000ull);
    return make(pad, (sign << 15) | (uint32_t)biased, m);
}

// exponent (of the significand's LSB) of a finite operand; field 0 scales as field 1
__device__ __forceinline__ int lsb_exp(const ld80 &a)
{
    int e = (int)(se(a) & 0x7FFF);
    if (e == 0) e = 1;
    return e - 16383 - 63;
}

__device__ __forceinline__ ld80 add(const ld80 &a, const ld80 &b)
{
    if (unsupported(a) || unsupported(b)) return default_nan(a);
    if (is_nan(a) || is_nan(b)) return nan_result(a, b);
    const uint32_t sa = se(a) >> 15, sb = se(b) >> 15;
    if (is_inf(a) || is_inf(b)) {
        if (is_inf(a) && is_inf(b) && sa != sb) return default_nan(a);
        return make(a, is_inf(a) ? se(a) : se(b), 0x8000000000000000ull);
    }
    if (is_zero(a) && is_zero(b)) return make(a, (sa & sb) << 15, 0);
    // align on the larger exponent, 63 guard bits below the larger significand
    int la = lsb_exp(a), lb = lsb_exp(b);
    u128 A = (u128)a.m << 63, B = (u128)b.m << 63;
    la -= 63;
    lb -= 63;
    bool sticky = false;
    uint32_t s1 = sa, s2 = sb;
    if (la < lb || (la == lb && A < B)) {
        u128 t = A; A = B; B = t;
        int ti = la; la = lb; lb = ti;
        uint32_t ts = s1; s1 = s2; s2 = ts;
    }
    const int d = la - lb;
    if (d >= 128) {
        sticky = B != 0;
        B = 0;
    } else if (d > 0) {
        sticky = (B & ((((u128)1) << d) - 1)) != 0;
        B >>= d;
    }
    u128 S;
    if (s1 == s2) {
        S = A + B;  // A < 2^127, B <= A: no overflow of 128 bits
    } else {
        S = A - B;
        if (sticky) S -= 1;  // the shifted-out bits belong to B
        if (S == 0 && !sticky) return make(a, 0, 0);  // exact cancellation: +0 in RNE
    }
    return round_pack(a, s1, S, la, sticky);
}

__device__ __forceinline__ ld80 mul(const ld80 &a, const ld80 &b)
{
    if (unsupported(a) || unsupported(b)) return default_nan(a);
    if (is_nan(a) || is_nan(b)) return nan_result(a, b);
    const uint32_t sign = (se(a) ^ se(b)) >> 15;
    if (is_inf(a) || is_inf(b)) {
        if (is_zero(a) || is_zero(b)) return default_nan(a);
        return make(a, (sign << 15) | 0x7FFF, 0x8000000000000000ull);
    }
    if (a.m == 0 || b.m == 0) return make(a, sign << 15, 0);
    const u128 P = (u128)a.m * (u128)b.m;
    return round_pack(a, sign, P, lsb_exp(a) + lsb_exp(b), false);
}

// a > b in the x87 sense (false when unordered); +0 == -0.
__device__ __forceinline__ bool gt(const ld80 &a, const ld80 &b)
{
    if (unsupported(a) || unsupported(b) || is_nan(a) || is_nan(b)) return false;
    if (is_zero(a) && is_zero(b)) return false;
    const uint32_t sa = se(a) >> 15, sb = se(b) >> 15;
    if (sa != sb) return sb;  // a positive, b negative
    int ea = (int)(se(a) & 0x7FFF), eb = (int)(se(b) & 0x7FFF);
    if (ea == 0) ea = 1;
    if (eb == 0) eb = 1;
    const bool mag_gt = ea != eb ? ea > eb : a.m > b.m;
    const bool mag_eq = ea == eb && a.m == b.m;
    return sa ? (!mag_gt && !mag_eq) : mag_gt;
}

}  // namespace x87

}  // namespace sos
