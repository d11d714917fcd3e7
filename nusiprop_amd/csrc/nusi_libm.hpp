// nuSIprop MI355X -- elementary functions with a fixed fp64 operation sequence.
//
// Why: the reference's interaction integrals (nuSIprop.hpp:759-1520) cancel
// catastrophically for small |t|, s' (mphi >> sqrt(2 m E)): a 1-ulp change in
// a log or dilog moves some table entries by ~1e-5 relative.  The reference's
// own output therefore depends on the last bits of its libm/GSL.  To make the
// GPU reproduce the CPU oracle bit for bit, both evaluate these functions with
// the same algorithm built only from IEEE-correctly-rounded operations
// (+ - * / sqrt fma) -- the GPU's ocml and the host's glibc differ in the last
// ulp.  Algorithms: Sun fdlibm 5.3 (e_log.c, s_log1p.c, e_exp.c, s_atan.c,
// e_atan2.c, e_atanh.c, e_log10.c; "Developed at SunPro ... Permission to
// use, copy, modify, and distribute this software is freely granted, provided
// that this notice is preserved."), error < 1 ulp each.  pow(x>0, y) =
// exp(y*log(x)) (a few ulp; only the power-law source uses it).
// The oracle carries its own C copy of the same algorithms (oracle/ora_libm.c).
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

#ifndef NUSI_FN
#define NUSI_FN __host__ __device__ inline
#endif

// log/log1p/exp/atan/atan2 are real calls by default: inlined at their ~60 call
// sites they made the alpha kernel 225 KB of code (I-cache bound; 154 vs 95 ms
// per 1024-point step measured).  -DNUSI_INLINE_LIBM inlines them (A/B builds).
#ifndef NUSI_INLINE_LIBM
#define NUSI_LM __host__ __device__ inline __attribute__((noinline))
#else
#define NUSI_LM NUSI_FN
#endif

#include "nusi_logtab.hpp"

namespace nusi {
namespace nm {

NUSI_FN unsigned long long bits(double x) { return __builtin_bit_cast(unsigned long long, x); }
NUSI_FN double from_bits(unsigned long long b) { return __builtin_bit_cast(double, b); }
NUSI_FN int hiw(double x) { return (int)(bits(x) >> 32); }
NUSI_FN unsigned low(double x) { return (unsigned)bits(x); }
NUSI_FN double with_hi(double x, int hi)
{
    return from_bits((bits(x) & 0xffffffffULL) | ((unsigned long long)(unsigned)hi << 32));
}

constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
constexpr double two54 = 1.80143985094819840000e+16;

// log / log1p: table-driven, division-free (nusi_logtab.hpp, gen_logtab.py).  x = 2^k z,
// z in [0x1.6p-1, 0x1.6p+0), c ~ the centre of z's 1/128 subinterval (c = 1 next to 1.0):
//   log(x) = k ln2 + log(c) + log1p(r),  r = z/c - 1 = fma(z, invc, -1),  |r| < 2^-7,
// k ln2 + log(c) + r summed with exact (Fast2Sum) error terms, log1p(r) - r by its Taylor
// series to r^9.  Error < 0.52 ulp; replaces fdlibm e_log.c / s_log1p.c (one division and
// ~20 integer / branch instructions each) with one table load and ~25 fp64 operations.
constexpr double kLn2hi = 0x1.62e42fefa3800p-1, kLn2lo = 0x1.ef35793c76730p-45;   // k * kLn2hi exact
// log(2^kadj * x) + c / x for a normal positive double x = from_bits(ix); c: log1p's rounding
// correction of 1 + x (0 for log).  kC = false (log): c = 0 and the correction term, fma(-sc, r, sc) with sc = +0, is
// +0 -- which the sum it is added to never is -0 (its first addend is +0 or nonzero) -- so it is left out: the same bits
// without the correction's six instructions (the compiler cannot drop a product with 0 itself)
template <bool kC = true>
NUSI_FN double log_kernel(unsigned long long ix, double c, int kadj)
{
    const unsigned long long tmp = ix - 0x3fe6000000000000ULL;
    const int i = (int)((tmp >> (52 - kLogTabBits)) & ((1u << kLogTabBits) - 1));
    const int k = (int)((long long)tmp >> 52);
    const double z = from_bits(ix - (tmp & (0xfffULL << 52)));
    const double invc = kLogTab[i][0], lch = kLogTab[i][1], lcl = kLogTab[i][2];
    const double r = fma(z, invc, -1.0);
    const double kd = (double)(k + kadj);
    const double t = kd * kLn2hi;
    const double s1 = t + lch, e1 = (t - s1) + lch;   // |t| >= |lch| or t == 0
    const double s2 = s1 + r, e2 = (s1 - s2) + r;     // |s1| >= |r| or s1 == 0
    double q = fma(r, 1.0 / 9, -1.0 / 8);
    q = fma(r, q, 1.0 / 7);
    q = fma(r, q, -1.0 / 6);
    q = fma(r, q, 1.0 / 5);
    q = fma(r, q, -0.25);
    q = fma(r, q, 1.0 / 3);
    q = fma(r, q, -0.5);
    const double p = (r * r) * q;
    if (!kC) return s2 + ((fma(kd, kLn2lo, lcl) + (e1 + e2)) + p);
    // c / x = c invc 2^-k / (1 + r) ~ sc (1 - r); 2^-k = 0 past the normal range (c / x negligible)
    const double sc = c * (invc * ((k < 1023) ? from_bits((unsigned long long)(1023 - k) << 52) : 0.0));
    return s2 + (((fma(kd, kLn2lo, lcl) + (e1 + e2)) + p) + fma(-sc, r, sc));
}

NUSI_FN double log_i(double x)
{
    const unsigned long long ix = bits(x);
    if (ix - 0x0010000000000000ULL >= 0x7fe0000000000000ULL) {   // not a normal positive double
        if (x != x || x == 1.0 / 0.0) return x + x;
        if (x == 0.0) return -1.0 / 0.0;
        if (x < 0.0) return (x - x) / 0.0;
        return log_kernel<false>(bits(x * 0x1p52), 0.0, -52);    // subnormal
    }
    return log_kernel<false>(ix, 0.0, 0);
}

// log1p(x) = log(u) + c / u, u = 1 + x rounded, c its exact rounding error (Fast2Sum)
NUSI_FN double log1p_i(double x)
{
    if (!(x > -1.0) || x == 1.0 / 0.0) {
        if (x == -1.0) return -1.0 / 0.0;
        if (x != x || x > 0.0) return x + x;
        return (x - x) / (x - x);
    }
    const double u = 1.0 + x;
    const double c = (x >= 1.0) ? 1.0 - (u - x) : x - (u - 1.0);
    return log_kernel(bits(u), c, 0);
}

// e_exp.c
NUSI_FN double exp_i(double x)
{
    constexpr double invln2 = 1.44269504088896338700e+00;
    constexpr double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                     P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                     P5 = 4.13813679705723846039e-08;
    constexpr double o_threshold = 7.09782712893383973096e+02, u_threshold = -7.45133219101941108420e+02;
    constexpr double twom1000 = 9.33263618503218878990e-302;
    int hx = hiw(x);
    const int xsb = (hx >> 31) & 1;
    hx &= 0x7fffffff;
    if (hx >= 0x40862E42) {                      // |x| >= 709.78
        if (hx >= 0x7ff00000) {
            if (((hx & 0xfffff) | low(x)) != 0) return x + x;   // NaN
            return (xsb == 0) ? x : 0.0;
        }
        if (x > o_threshold) return 1.0 / 0.0;
        if (x < u_threshold) return 0.0;
    }
    double hi = 0.0, lo = 0.0;
    int k = 0;
    if (hx > 0x3fd62e42) {                       // |x| > 0.5 ln2
        if (hx < 0x3FF0A2B2) {                   // and |x| < 1.5 ln2
            hi = xsb ? x + ln2_hi : x - ln2_hi;
            lo = xsb ? -ln2_lo : ln2_lo;
            k = 1 - xsb - xsb;
        } else {
            k = (int)(invln2 * x + (xsb ? -0.5 : 0.5));
            const double t = k;
            hi = x - t * ln2_hi;                 // t*ln2_hi is exact here
            lo = t * ln2_lo;
        }
        x = hi - lo;
    } else if (hx < 0x3e300000) {                // |x| < 2^-28
        return 1.0 + x;
    }
    const double t = x * x;
    const double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
    const double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
    if (k >= -1021) return from_bits(bits(y) + ((unsigned long long)(long long)k << 52));
    return from_bits(bits(y) + ((unsigned long long)(long long)(k + 1000) << 52)) * twom1000;
}

// s_atan.c
NUSI_FN double atan_i(double x)
{
    constexpr double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                                  1.57079632679489655800e+00};
    constexpr double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                                  6.12323399573676603587e-17};
    constexpr double aT[11] = {3.33333333333329318027e-01,  -1.99999999998764832476e-01, 1.42857142725034663711e-01,
                               -1.11111104054623557880e-01, 9.09088713343650656196e-02,  -7.69187620504482999495e-02,
                               6.66107313738753120669e-02,  -5.83357013379057348645e-02, 4.97687799461593236017e-02,
                               -3.65315727442169155270e-02, 1.62858201153657823623e-02};
    const int hx = hiw(x);
    const int ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x44100000) {                      // |x| >= 2^66
        if (ix > 0x7ff00000 || (ix == 0x7ff00000 && low(x) != 0)) return x + x;
        return (hx > 0) ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3fdc0000) {                       // |x| < 0.4375
        if (ix < 0x3e200000) return x;           // |x| < 2^-29
        id = -1;
    } else {
        // the four argument reductions share one division (same operands, same result bits as
        // fdlibm's per-range divisions; one v_div sequence instead of four under divergence)
        x = fabs(x);
        double num, den;
        if (ix < 0x3ff30000) {                   // |x| < 1.1875
            if (ix < 0x3fe60000) {               // 7/16 <= |x| < 11/16
                id = 0;
                num = 2.0 * x - 1.0;
                den = 2.0 + x;
            } else {                             // 11/16 <= |x| < 19/16
                id = 1;
                num = x - 1.0;
                den = x + 1.0;
            }
        } else {
            if (ix < 0x40038000) {               // |x| < 2.4375
                id = 2;
                num = x - 1.5;
                den = 1.0 + 1.5 * x;
            } else {                             // 2.4375 <= |x| < 2^66
                id = 3;
                num = -1.0;
                den = x;
            }
        }
        x = num / den;
    }
    const double z = x * x;
    const double w = z * z;
    const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const double r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return (hx < 0) ? -r : r;
}

// e_atan2.c
NUSI_FN double atan2_full(double y, double x)
{
    constexpr double pi_o_2 = 1.5707963267948965580E+00, pi = 3.1415926535897931160E+00,
                     pi_lo = 1.2246467991473531772E-16, pi_o_4 = 7.8539816339744827900E-01;
    const int hx = hiw(x), hy = hiw(y);
    const unsigned lx = low(x), ly = low(y);
    const int ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    if (((unsigned)ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000u || ((unsigned)iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000u)
        return x + y;                            // NaN
    if (hx == 0x3ff00000 && lx == 0u) return atan_i(y);   // x = 1.0 (fdlibm subtracts, overflowing int)
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);         // 2*sign(x)+sign(y)
    if ((iy | (int)ly) == 0) {                   // y = 0
        switch (m) {
        case 0:
        case 1: return y;
        case 2: return pi;
        default: return -pi;
        }
    }
    if ((ix | (int)lx) == 0) return (hy < 0) ? -pi_o_2 : pi_o_2;
    if (ix == 0x7ff00000) {                      // x = +-inf
        if (iy == 0x7ff00000) {
            switch (m) {
            case 0: return pi_o_4;
            case 1: return -pi_o_4;
            case 2: return 3.0 * pi_o_4;
            default: return -3.0 * pi_o_4;
            }
        }
        switch (m) {
        case 0: return 0.0;
        case 1: return -0.0;
        case 2: return pi;
        default: return -pi;
        }
    }
    if (iy == 0x7ff00000) return (hy < 0) ? -pi_o_2 : pi_o_2;
    const int k = (iy - ix) >> 20;
    double z;
    if (k > 60) z = pi_o_2 + 0.5 * pi_lo;        // |y/x| > 2^60
    else if (hx < 0 && k < -60) z = 0.0;         // |y|/x < -2^60
    else z = atan_i(fabs(y / x));
    switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
    }
}

// atan2 without fdlibm's special-case branches, for the common case: y and x finite and nonzero, x != 1.0 and
// |k| <= 60 (k = (iy - ix) >> 20, the exponent difference).  There e_atan2.c computes z = atan(|y / x|) and fixes the
// octant, and s_atan.c reduces |y / x| by range; here the range's numerator and denominator, the table constants and
// the octant are selected instead of branched on (range -1 divides by 1.0, exactly), the same operations on the same
// operands, so the same bits.  Every branch of the full version kept an exec mask live in SGPRs -- inside GSL's complex
// dilogarithm that spilled SGPRs into VGPR lanes -- and the wave votes for this path once (a wave with any other
// argument takes atan2_full; tests/test_specfun.py compares the two bit for bit).
NUSI_FN bool atan2_plain(double y, double x)
{
    const int hx = hiw(x), hy = hiw(y);
    const int ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const int k = (iy - ix) >> 20;
    return ix < 0x7ff00000 && iy < 0x7ff00000 && ((unsigned)ix | low(x)) != 0u && ((unsigned)iy | low(y)) != 0u &&
           !(hx == 0x3ff00000 && low(x) == 0u) && k <= 60 && k >= -60;
}
NUSI_FN double atan2_sel(double y, double x)
{
    constexpr double pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
    constexpr double aT[11] = {3.33333333333329318027e-01,  -1.99999999998764832476e-01, 1.42857142725034663711e-01,
                               -1.11111104054623557880e-01, 9.09088713343650656196e-02,  -7.69187620504482999495e-02,
                               6.66107313738753120669e-02,  -5.83357013379057348645e-02, 4.97687799461593236017e-02,
                               -3.65315727442169155270e-02, 1.62858201153657823623e-02};
    const double t = fabs(y / x);   // s_atan.c's argument, >= 0 and finite here
    const int it = hiw(t);
    const bool r_1 = it < 0x3fdc0000, r0 = it < 0x3fe60000, r1 = it < 0x3ff30000, r2 = it < 0x40038000;
    const double num = r_1 ? t : r0 ? 2.0 * t - 1.0 : r1 ? t - 1.0 : r2 ? t - 1.5 : -1.0;
    const double den = r_1 ? 1.0 : r0 ? 2.0 + t : r1 ? t + 1.0 : r2 ? 1.0 + 1.5 * t : t;
    const double xr = num / den;
    const double z = xr * xr;
    const double w = z * z;
    const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    const double ahi = r0 ? 4.63647609000806093515e-01 : r1 ? 7.85398163397448278999e-01
                     : r2 ? 9.82793723247329054082e-01 : 1.57079632679489655800e+00;
    const double alo = r0 ? 2.26987774529616870924e-17 : r1 ? 3.06161699786838301793e-17
                     : r2 ? 1.39033110312309984516e-17 : 6.12323399573676603587e-17;
    double at = r_1 ? xr - xr * (s1 + s2) : ahi - ((xr * (s1 + s2) - alo) - xr);
    if (it < 0x3e200000) at = t;   // |t| < 2^-29 (a select)
    const int m = ((hiw(y) >> 31) & 1) | ((hiw(x) >> 30) & 2);   // 2 sign(x) + sign(y)
    const double zz = at - pi_lo;
    return m == 0 ? at : m == 1 ? -at : m == 2 ? pi - zz : zz - pi;
}
NUSI_FN bool wave_all_l(bool p)
{
#ifdef __HIP_DEVICE_COMPILE__
    return __all(p);
#else
    return p;
#endif
}
// the rare waves' fdlibm atan2 as a call: inlined at every atan2 site it was most of k_alpha_mcorner's code (~1 700
// of its 8 600 instructions per site, against an instruction cache shared by two CUs); NUSI_ATAN2_RARE_INLINE: inline
NUSI_LM double atan2_rare(double y, double x) { return atan2_full(y, x); }
NUSI_FN double atan2_i(double y, double x)
{
#ifndef NUSI_ATAN2_FULL   // (A/B: fdlibm's branches only)
    if (wave_all_l(atan2_plain(y, x))) return atan2_sel(y, x);
#ifndef NUSI_ATAN2_RARE_INLINE
    return atan2_rare(y, x);
#endif
#endif
    return atan2_full(y, x);
}

// Out-of-line entry points (see NUSI_LM); the *_i bodies above are inlined where a caller wants
// them inline (the polylogarithms, which are themselves out of line).
NUSI_LM double log(double x) { return log_i(x); }
NUSI_LM double log1p(double x) { return log1p_i(x); }
NUSI_LM double exp(double x) { return exp_i(x); }
NUSI_LM double atan(double x) { return atan_i(x); }
NUSI_LM double atan2(double y, double x) { return atan2_i(y, x); }

// e_atanh.c
NUSI_FN double atanh(double x)
{
    const int hx = hiw(x);
    const int ix = hx & 0x7fffffff;
    if (ix > 0x3ff00000 || (ix == 0x3ff00000 && low(x) != 0)) return (x - x) / (x - x);   // |x| > 1
    if (ix == 0x3ff00000 && low(x) == 0) return x / 0.0;
    if (ix < 0x3e300000) return x;               // |x| < 2^-28
    const double ax = fabs(x);
    double t;
    if (ix < 0x3fe00000) {                       // |x| < 0.5
        t = ax + ax;
        t = 0.5 * log1p(t + t * ax / (1.0 - ax));
    } else
        t = 0.5 * log1p((ax + ax) / (1.0 - ax));
    return (hx >= 0) ? t : -t;
}

// e_log10.c
NUSI_FN double log10(double x)
{
    constexpr double ivln10 = 4.34294481903251816668e-01, log10_2hi = 3.01029995663611771306e-01,
                     log10_2lo = 3.69423907715893078616e-13;
    int hx = hiw(x);
    int k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | low(x)) == 0) return -1.0 / 0.0;
        if (hx < 0) return (x - x) / 0.0;
        k -= 54;
        x *= two54;
        hx = hiw(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    const int i = (int)(((unsigned)k & 0x80000000u) >> 31);
    hx = (hx & 0x000fffff) | ((0x3ff - i) << 20);
    const double y = (double)(k + i);
    x = with_hi(x, hx);
    const double z = y * log10_2lo + ivln10 * log(x);
    return z + y * log10_2hi;
}

// x > 0
NUSI_FN double pow(double x, double y) { return exp(y * log(x)); }

}  // namespace nm
}  // namespace nusi
