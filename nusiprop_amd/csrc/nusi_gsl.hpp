// nuSIprop MI355X -- GSL's dilogarithm algorithms, the arithmetic of NUSI_OPT_REFERENCE_ORDER.
//
// The reference evaluates its closed forms with GSL (version unpinned, the Homebrew build of setup.py:10-11):
//   gsl_sf_dilog(x)                      aux.hpp:112,129,147,165   nuSIprop.hpp:1098,1202,1375-1398
//   gsl_sf_complex_dilog_xy_e(x, y, ..)  aux.hpp:92-93             nuSIprop.hpp:1444-1451
// Where the closed forms cancel (the s-t / s-u interference of Gamma, alphaTilde and alpha), a one-ulp change in a
// dilogarithm moves a table entry by up to 1e-6, so "the reference's arithmetic" means GSL's algorithm, not just
// an accurate Li2.  These functions are GSL 2.x specfunc/dilog.c (with clausen.c, log.c's complex log, trig.c's
// angle reduction, cheb_eval.c) restated: the same branch points (real: 0.25 / 0.5 / 1 / 1.01 / 2 and the x < 0
// reduction; complex: |z|^2 ~ 1 Lewin, 1/z for |z| > 1, 1 - z for x > 0.732, series_1 / series_2 / series_3 at
// |z| 0.25 / 0.98), series, loop bounds and stopping tests, in the same operation order, on this repository's
// shared libm (nm::log, nm::atan2) -- the oracle runs the same sequence (oracle/ora_gsl.c), bit for bit.
//
// GPU shape (the values are unchanged by any of it):
//   * each heavy piece exists once in the code: gsl_cli2 forms its unit-disk argument (1/z or z), unitdisk its
//     fundamental-region argument (1 - z or z), and one call each of the series runs; dilog_xge0 forms its series
//     argument and runs one series_2 loop for its four branches that need one.  Inlined per branch they made the
//     function ~30 000 instructions (instruction-cache bound);
//   * series_1 and series_2_c share one loop (cseries): the same recurrence with the term's denominator k^2 or
//     k^2 (k + 1), so a wave whose lanes take different series runs one loop, not two;
//   * GSL stops a series when fabs(a / b) < 2^-p (p = 52, 53 or 104).  For a, b >= 0 and b 2^-p a normal number,
//     RN(a / b) < 2^-p  <=>  a < b 2^-p: the doubles below 2^-p b are those at or below its predecessor, which
//     lies below the rounding boundary 2^-p b (1 - 2^-54).  So the test is one multiply and one compare
//     (quot_lt);
//   * the series' term a / d_k with d_k = k^2 or k^2 (k + 1) (exact integers below 2^30) is RN(a / d_k) as
//     fma(a, y_k, RN(a l_k)), y_k + l_k the reciprocal to 2^-106 (y_k = RN(1 / d_k), l_k = RN(1 / d_k - y_k)): the sum
//     is a / d_k to a relative 2^-105, and a / d_k is never a rounding midpoint nor within 2^-84 of one (a midpoint
//     m = M 2^e has an odd 54-bit M, and a = m d_k would need the odd part of M d_k, >= M, in 53 bits; a nearer one
//     leaves |a - m d_k| >= 2^e >= a 2^-84 for d_k < 2^30), so the one rounding of the fma is the division's.  Two
//     operations per term instead of a five-operation residual correction (tests/test_specfun.py runs the device
//     functions against the oracle's divisions).  GSL's (k - 1)/k squared of series_1 is a table of the same values;
//   * both rewrites need their operands in the normal range; a series whose argument is below 2^-400 (which the
//     tables never meet) runs a second instance of its loop with GSL's divisions (kExact), so the loops have no
//     per-iteration branch.
#pragma once

#include "nusi_libm.hpp"

// The elementary functions inside the GSL functions: inline by default (each call from an out-of-line function costs
// the callee's register save / restore and the call; NUSI_GSL_CALL_LIBM: calls, A/B builds).  The same functions.
#ifdef NUSI_GSL_CALL_LIBM
#define GSL_LOG nm::log
#define GSL_ATAN2 nm::atan2
#else
#define GSL_LOG nm::log_i
#define GSL_ATAN2 nm::atan2_i
#endif

namespace nusi {
namespace gsl {

constexpr double kEps = 2.2204460492503131e-16;       // GSL_DBL_EPSILON
constexpr double kSqrtEps = 1.4901161193847656e-08;   // GSL_SQRT_DBL_EPSILON
constexpr double kPiD = 3.14159265358979323846;       // M_PI

// per-k constants of the series: d1 = k^2 and d2 = k^2 (k + 1) (exact), their rounded reciprocals and the
// reciprocals' low parts, side by side (one 48-byte scalar load per iteration, k being uniform), and
// rr = ((k - 1) / k)^2 as series_1 forms it (every value the compiler's IEEE evaluation of GSL's expression)
constexpr int kKTab = 1000;
struct KRow { double d1, d2, y1, y2, l1, l2; };
struct KTab {
    KRow row[kKTab];
    double rr[kKTab];
};
// RN(1 / d - y) for y = RN(1 / d): e = 1 - y d exactly (Dekker's product y d = p + err, 1 - p exact by Sterbenz, and
// e a multiple of ulp(y) below d ulp(y) / 2, representable), then RN(e / d) -- constexpr, no fma
constexpr double recip_lo(double d, double y)
{
    const double cy = 134217729.0 * y, yh = cy - (cy - y), yl = y - yh;
    const double cd_ = 134217729.0 * d, dh = cd_ - (cd_ - d), dl = d - dh;
    const double p = y * d, err = ((yh * dh - p) + yh * dl + yl * dh) + yl * dl;
    return ((1.0 - p) - err) / d;
}
constexpr KTab make_ktab()
{
    KTab t{};
    for (int k = 1; k < kKTab; ++k) {
        t.row[k].d1 = (double)k * k;
        t.row[k].d2 = (double)k * k * (k + 1.0);
        t.row[k].y1 = 1.0 / t.row[k].d1;
        t.row[k].y2 = 1.0 / t.row[k].d2;
        t.row[k].l1 = recip_lo(t.row[k].d1, t.row[k].y1);
        t.row[k].l2 = recip_lo(t.row[k].d2, t.row[k].y2);
        const double rk = (k - 1.0) / k;
        t.rr[k] = rk * rk;
    }
    return t;
}
constexpr KTab kKT = make_ktab();
#ifndef NUSI_S2_VLOAD   // A/B: 0 = waves of both complex series select each lane's row columns (scalar row)
#define NUSI_S2_VLOAD 1
#endif
constexpr bool kS2VecRows = NUSI_S2_VLOAD != 0;

// RN(a / d) for the series' terms.  kExact: the division; else fma(a, y, RN(a l)) from the two-part reciprocal
// y + l (header comment), valid for a, d > 0 with a l normal (a >= 2^-900) -- the callers take kExact for arguments
// that could reach below (a series argument under 2^-400, never met in the tables)
template <bool kExact>
NUSI_FN double div_k(double a, double d, double y, double l)
{
    if (kExact) return a / d;
    return fma(a, y, a * l);
}

// fabs(a / b) < c of GSL's stopping tests for a, b >= 0 and c a power of two: kExact the division, else a < b c
// (header comment; exact for b c a normal number, b >= 2^-900 -- the callers' kExact covers the rest)
template <bool kExact>
NUSI_FN bool quot_lt(double a, double b, double c)
{
    if (kExact) return a / b < c;
    return a < b * c;
}

// hypot(x, y) (libm; dilogc_unitdisk): sqrt(a^2 + b^2) and one correction step from the exact residual
// (oracle/ora_gsl.c ora_hypot)
NUSI_FN double hypot(double x, double y)
{
    double a = fabs(x), b = fabs(y);
    if (a < b) { const double t = a; a = b; b = t; }
#ifdef __HIP_DEVICE_COMPILE__
    // the common case (2^-500 <= b <= a <= 2^500) voted once per wave: the same operations without the scaling
    // branches, whose exec masks stayed live in SGPRs
    if (__all(b >= 0x1p-500 && a <= 0x1p+500)) {
        const double a2 = a * a, ea = fma(a, a, -a2), b2 = b * b, eb = fma(b, b, -b2);
        double h = sqrt(a2 + b2);
        const double h2 = h * h, eh = fma(h, h, -h2);
        const double r = ((a2 - h2) + b2) + ((ea + eb) - eh);
        return h + r / (2.0 * h);
    }
#endif
    if (b == 0.0 || !(a <= 1.79769313486231570815e+308)) return a + b;
    double s = 1.0;
    if (a > 0x1p+500) { a *= 0x1p-600; b *= 0x1p-600; s = 0x1p+600; }
    else if (b < 0x1p-500) { a *= 0x1p+600; b *= 0x1p+600; s = 0x1p-600; }
    const double a2 = a * a, ea = fma(a, a, -a2), b2 = b * b, eb = fma(b, b, -b2);
    double h = sqrt(a2 + b2);
    const double h2 = h * h, eh = fma(h, h, -h2);
    const double r = ((a2 - h2) + b2) + ((ea + eb) - eh);
    h = h + r / (2.0 * h);
    return h * s;
}

// Wave-uniform votes for the series' first loops (below): every active lane's predicate / any active lane's.  On the
// host (tests/hostcheck) a "wave" is the one call.
NUSI_FN bool wave_all(bool p)
{
#ifdef __HIP_DEVICE_COMPILE__
    return __all(p);
#else
    return p;
#endif
}
NUSI_FN bool wave_any(bool p)
{
#ifdef __HIP_DEVICE_COMPILE__
    return __any(p);
#else
    return p;
#endif
}

// ------------------------------------------------------------------------------------------------- real --
// dilog_series_1: sum x^k / k^2, 0 < x <= 1/4.  (Not kExact: the partial sums are below x pi^2 / 6, so GSL's test
// term < 2^-52 sum cannot hold while term >= 2^-50 x: the first loop runs without it, as cseries_t's.)
template <bool kExact>
NUSI_FN double dilog_series_1_t(double x)
{
    double sum = x, term = x;
    int k = 2;
    bool done = false;
    if (!kExact) {
        const double big = x * 0x1p-50;
        bool small = false;
        while (k < 1000) {
            term *= x;
            term *= kKT.rr[k];
            sum += term;
            small = wave_any(term < big);
            if (small) break;
            ++k;
        }
        if (small) {
            done = quot_lt<false>(fabs(term), fabs(sum), 0x1p-52);
            ++k;
        }
    }
    if (!done)
        for (; k < 1000; k++) {
            term *= x;
            term *= kKT.rr[k];   // rk * rk, rk = (k - 1.0) / k
            sum += term;
            if (quot_lt<kExact>(fabs(term), fabs(sum), 0x1p-52)) break;   // fabs(term / sum) < GSL_DBL_EPSILON
        }
    return sum;
}
NUSI_FN double dilog_series_1(double x)
{
    return x < 0x1p-400 ? dilog_series_1_t<true>(x) : dilog_series_1_t<false>(x);
}
// series_2: sum r^k / (k^2 (k + 1)) with the first nine terms unconditionally (d2 = k * k * (k + 1.0), exact).
// (Not kExact: the partial sums are below 0.65 x, so GSL's test ds < 2^-53 sum cannot hold while ds >= 2^-51 x.)
template <bool kExact>
NUSI_FN double series_2_t(double x)
{
    double rk = x, sum = 0.5 * x;
    int k;
#pragma unroll
    for (k = 2; k < 10; k++) {
        rk *= x;
        sum += div_k<kExact>(rk, kKT.row[k].d2, kKT.row[k].y2, kKT.row[k].l2);
    }
    bool done = false;
    if (!kExact) {
        const double big = x * 0x1p-51;
        double ds = 0.0;
        bool small = false;
        while (k < 100) {
            rk *= x;
            ds = div_k<false>(rk, kKT.row[k].d2, kKT.row[k].y2, kKT.row[k].l2);
            sum += ds;
            small = wave_any(ds < big);
            if (small) break;
            ++k;
        }
        if (small) {
            done = quot_lt<false>(fabs(ds), fabs(sum), 0x1p-53);
            ++k;
        }
    }
    if (!done)
        for (; k < 100; k++) {
            rk *= x;
            const double ds = div_k<kExact>(rk, kKT.row[k].d2, kKT.row[k].y2, kKT.row[k].l2);
            sum += ds;
            if (quot_lt<kExact>(fabs(ds), fabs(sum), 0x1p-53)) break;   // fabs(ds / sum) < 0.5 GSL_DBL_EPSILON
        }
    return sum;
}
// dilog_series_2: Li2(x) = 1 + (1 - x) log(1 - x) / x + series_2(x)
NUSI_FN double dilog_series_2(double x)
{
    double sum = x < 0x1p-100 ? series_2_t<true>(x) : series_2_t<false>(x);   // (x^9 stays above 2^-900)
    double t;
    if (x > 0.01) t = (1.0 - x) * GSL_LOG(1.0 - x) / x;
    else {
        const double c3 = 1.0 / 3.0, c4 = 1.0 / 4.0, c5 = 1.0 / 5.0, c6 = 1.0 / 6.0, c7 = 1.0 / 7.0, c8 = 1.0 / 8.0;
        const double t68 = c6 + x * (c7 + x * c8);
        const double t38 = c3 + x * (c4 + x * (c5 + x * t68));
        t = (x - 1.0) * (1.0 + x * (0.5 + x * t38));
    }
    sum += 1.0 + t;
    return sum;
}
// dilog_xge0: Re Li2(x), x >= 0.  Branches: x > 2 (series_2 of 1/x), 1.01 < x <= 2 (of 1 - 1/x), 1 < x <= 1.01
// (the series about 1), x == 1, 1/2 < x < 1 (series_2 of 1 - x), 1/4 < x <= 1/2 (of x), 0 < x <= 1/4 (series_1)
NUSI_FN_OUT double dilog_xge0(double x)
{
    if (x > 1.0 && x <= 1.01) {   // series around x = 1
        const double eps = x - 1.0, lne = GSL_LOG(eps);
        const double c0 = kPiD * kPiD / 6.0, c1 = 1.0 - lne, c2 = -(1.0 - 2.0 * lne) / 4.0, c3 = (1.0 - 3.0 * lne) / 9.0;
        const double c4 = -(1.0 - 4.0 * lne) / 16.0, c5 = (1.0 - 5.0 * lne) / 25.0, c6 = -(1.0 - 6.0 * lne) / 36.0;
        const double c7 = (1.0 - 7.0 * lne) / 49.0, c8 = -(1.0 - 8.0 * lne) / 64.0;
        return c0 + eps * (c1 + eps * (c2 + eps * (c3 + eps * (c4 + eps * (c5 + eps * (c6 + eps * (c7 + eps * c8)))))));
    }
    if (x == 1.0) return kPiD * kPiD / 6.0;
    if (!(x > 0.25)) return x > 0.0 ? dilog_series_1(x) : 0.0;   // (x == 0 and NaN: GSL's last branch, 0)
    const int br = x > 2.0 ? 0 : x > 1.01 ? 1 : x > 0.5 ? 2 : 3;
    const double u = br == 0 ? 1.0 / x : br == 1 ? 1.0 - 1.0 / x : br == 2 ? 1.0 - x : x;   // GSL's series argument
    const double ser = dilog_series_2(u);
    if (br == 3) return ser;
    const double log_x = GSL_LOG(x);
    const double log_u = br == 0 ? 0.0 : GSL_LOG(u);   // log(1 - 1/x) resp. log(1 - x)
    if (br == 0) {
        const double t1 = kPiD * kPiD / 3.0, t2 = ser, t3 = 0.5 * log_x * log_x;
        return t1 - t2 - t3;
    }
    if (br == 1) {
        const double log_term = log_x * (log_u + 0.5 * log_x);
        const double t1 = kPiD * kPiD / 6.0, t2 = ser, t3 = log_term;
        return t1 + t2 - t3;
    }
    const double t1 = kPiD * kPiD / 6.0, t2 = ser, t3 = log_x * log_u;
    return t1 - t2 - t3;
}

// ---------------------------------------------------------------------------------------------- Clausen --
// gsl_sf_angle_restrict_pos_e (trig.c): [0, 2 pi) with the synthetic extended-precision 2 pi
NUSI_FN double angle_restrict_pos(double theta)
{
    const double P1 = 4 * 7.85398125648498535156e-01, P2 = 4 * 3.77489470793079817668e-08;
    const double P3 = 4 * 2.69515142907905952645e-15, TwoPi = 2 * (P1 + P2 + P3);
    const double y = 2 * floor(theta / TwoPi);
    double r = ((theta - y * P1) - y * P2) - y * P3;
    if (r > TwoPi) r = (((r - 2 * P1) - 2 * P2) - 2 * P3);
    else if (r < 0) r = (((r + 2 * P1) + 2 * P2) + 2 * P3);
    return r;
}
// gsl_sf_clausen_e: Cl2(x); aclaus_cs (clausen.c) summed by cheb_eval_e (order 14 on [-1, 1])
NUSI_FN_OUT double clausen(double x)
{
    constexpr double kC[15] = {2.142694363766688447e+00, 0.723324281221257925e-01, 0.101642475021151164e-02,
                               0.3245250328531645e-04,   0.133315187571472e-05,    0.6213240591653e-07,
                               0.313004135337e-08,       0.16635723056e-09,        0.919659293e-11,
                               0.52400462e-12,           0.3058040e-13,            0.18197e-14,
                               0.1100e-15,               0.68e-17,                 0.4e-18};
    const double x_cut = kPiD * kSqrtEps;
    double sgn = 1.0;
    if (x < 0.0) { x = -x; sgn = -1.0; }
    x = angle_restrict_pos(x);
    if (x > kPiD) {
        const double p0 = 6.28125, p1 = 0.19353071795864769253e-02;
        x = (p0 - x) + p1;
        sgn = -sgn;
    }
    double val;
    if (x == 0.0) val = 0.0;
    else if (x < x_cut) val = x * (1.0 - GSL_LOG(x));
    else {
        const double t = 2.0 * (x * x / (kPiD * kPiD) - 0.5);
        const double a = -1.0, b = 1.0;
        double d = 0.0, dd = 0.0;
        const double yy = (2.0 * t - a - b) / (b - a), y2 = 2.0 * yy;
#pragma unroll
        for (int j = 14; j >= 1; j--) {
            const double temp = d;
            d = y2 * d - dd + kC[j];
            dd = temp;
        }
        d = yy * d - dd + 0.5 * kC[0];
        val = x * (d - GSL_LOG(x));
    }
    return val * sgn;
}

// ---------------------------------------------------------------------------------------------- complex --
// dilogc_series_1 (s2 = false: sum r^k e^(i k theta) / k^2, first term r e^(i theta), kmax 50 + 22 / (-log r))
// and series_2_c (s2 = true: sum z^k / (k^2 (k + 1)), first term r e^(i theta) / 2, kmax 30 + 18 / (-log r)) as
// one loop; every operation is GSL's.  kS2: 0 / 1 every lane of the wave runs series_1 / series_2_c (the table
// column a constant), 2 per lane (s2).
//
// GSL tests |term|^2 < 2^-104 |sum|^2 after every term.  The partial sums are bounded by the sum of the moduli,
// |sum| <= r sum_k r^(k-1) / k^2 <= r pi^2 / 6 (series_2_c's terms are smaller still), and |term| = q (ck^2 +
// sk^2)^(1/2) with q = RN(r^k / d_k) and the rotated (ck, sk) of modulus 1 to ~1e-13 (<= 1000 rotations); so while q
// >= 2^-50 r (2.4 times the bound's 1.645 2^-52 r) the test is false, and the loop runs without it until the first
// term below, whose test is GSL's test at that k (the values are unchanged: the same terms, the same break).
template <bool kExact, int kS2>
NUSI_FN void cseries_t(bool s2, double r, double lr, double x, double y, double& re, double& im)
{
    const bool t2 = kS2 == 2 ? s2 : kS2 == 1;
    const double cos_theta = x / r, sin_theta = y / r;
    const double alpha = 1.0 - cos_theta, beta = sin_theta;
    double ck = cos_theta, sk = sin_theta, rk = r;
    double real_sum = t2 ? 0.5 * r * ck : r * ck;
    double imag_sum = t2 ? 0.5 * r * sk : r * sk;
    const double nlr = -lr;   // -log(r)
    const int kmax = (t2 ? 30 : 50) + (int)((t2 ? 18.0 : 22.0) / nlr);   // (one division for a wave of both series)
    KRow next = kKT.row[2];   // (the table row of the next iteration is loaded one iteration ahead; kmax <= 921)
    // kS2 == 2 (a wave of both series): each lane loads its own columns of the row (vector loads at its t2 offset from
    // the row's uniform address) instead of selecting between the scalar row's columns -- three 64-bit selects a term
    constexpr bool vrow = kS2 == 2 && kS2VecRows;
    const int toff = t2 ? 1 : 0;
    double nd = 0.0, ny = 0.0, nl = 0.0;
    if (vrow) {
        const double* rp = &kKT.row[2].d1;
        nd = rp[toff]; ny = rp[2 + toff]; nl = rp[4 + toff];
    }
    double q = 0.0, dr = 0.0, di = 0.0;
    auto term = [&](int k) {
        double d, yk, lk;
        if (vrow) {
            d = nd; yk = ny; lk = nl;
            const double* rp = &kKT.row[k + 1].d1;
            nd = rp[toff]; ny = rp[2 + toff]; nl = rp[4 + toff];
        } else {
            const KRow kr = next;
#ifdef NUSI_GSL_ROW_STUB   // timing A/B only (wrong values): every term reads row 2 (no table load in the loop)
            (void)k;
#else
            next = kKT.row[k + 1];
#endif
            d = t2 ? kr.d2 : kr.d1;   // (double) k * k * (k + 1.0) or (double) k * k
            yk = t2 ? kr.y2 : kr.y1;
            lk = t2 ? kr.l2 : kr.l1;
        }
        const double ck_tmp = ck;
        ck = ck - (alpha * ck + beta * sk);
        sk = sk - (alpha * sk - beta * ck_tmp);
        rk *= r;
        q = div_k<kExact>(rk, d, yk, lk);
        dr = q * ck;
        di = q * sk;
        real_sum += dr;
        imag_sum += di;
    };
    auto stop = [&]() { return quot_lt<kExact>(dr * dr + di * di, real_sum * real_sum + imag_sum * imag_sum, 0x1p-104); };
    int k = 2;
    bool done = false;
#ifdef NUSI_GSL_STUB_SERIES   // timing A/B only (wrong values): the complex series without its terms
    if (k < kmax) {
        re = real_sum;
        im = imag_sum;
        return;
    }
#endif
    if (!kExact) {
        // the first loop leaves together (wave votes), so k stays wave-uniform and the table rows scalar loads: at the
        // first k where a lane reaches its kmax (no term k), or where a lane's term falls below its bound (term k
        // added, then each lane's test at k -- false for the lanes still above it)
        const double big = r * 0x1p-50;
        bool small = false;
        // two terms per kmax vote while both are below every lane's kmax (the same terms and exit as one at a time)
        while (wave_all(k + 1 < kmax)) {
            term(k);
            small = wave_any(q < big);
            if (small) break;
            ++k;
            term(k);
            small = wave_any(q < big);
            if (small) break;
            ++k;
        }
        if (!small)
            while (wave_all(k < kmax)) {
                term(k);
                small = wave_any(q < big);
                if (small) break;
                ++k;
            }
        if (small) {
            done = stop();
            ++k;
        }
    }
    if (!done)
        for (; k < kmax; k++) {
            term(k);
            if (stop()) break;
        }
    re = real_sum;
    im = imag_sum;
}
// (the terms r^k stay above 2^-960 and |sum|^2 above 2^-900 unless r < 2^-400: the series breaks at a term
// below 2^-52 of the sum, and kmax bounds r^k for larger r)
NUSI_FN void cseries(bool s2, double r, double lr, double x, double y, double& re, double& im)
{
    if (r < 0x1p-400) {
        cseries_t<true, 2>(s2, r, lr, x, y, re, im);
        return;
    }
#ifdef __HIP_DEVICE_COMPILE__
    const unsigned long long act = __ballot(1), two = __ballot(s2);
    if (two == act) cseries_t<false, 1>(s2, r, lr, x, y, re, im);
    else if (two == 0) cseries_t<false, 0>(s2, r, lr, x, y, re, im);
    else cseries_t<false, 2>(s2, r, lr, x, y, re, im);
#else
    cseries_t<false, 2>(s2, r, lr, x, y, re, im);
#endif
}
// dilogc_series_3: |z| near 1, sum_{n <= 6} (log r)^n / n! H_n(theta)
NUSI_FN void cseries_3(double r, double lr, double x, double y, double& re, double& im)
{
    const double theta = GSL_ATAN2(y, x);
    const double cos_theta = x / r, sin_theta = y / r;
    const double a = lr;   // log(r)
    const double omc = 1.0 - cos_theta, omc2 = omc * omc;
    double H_re[7], H_im[7];
    H_re[0] = kPiD * kPiD / 6.0 + 0.25 * (theta * theta - 2.0 * kPiD * fabs(theta));
    H_im[0] = clausen(theta);
    H_re[1] = -0.5 * GSL_LOG(2.0 * omc);
    H_im[1] = -GSL_ATAN2(-sin_theta, omc);
    H_re[2] = -0.5;
    H_im[2] = 0.5 * sin_theta / omc;
    H_re[3] = -0.5 / omc;
    H_im[3] = 0.0;
    H_re[4] = 0.0;
    H_im[4] = -0.5 * sin_theta / omc2;
    H_re[5] = 0.5 * (2.0 + cos_theta) / omc2;
    H_im[5] = 0.0;
    H_re[6] = 0.0;
    H_im[6] = 0.5 * sin_theta / (omc2 * omc2 * omc) * (8.0 * omc - sin_theta * sin_theta * (3.0 + cos_theta));
    double sum_re = H_re[0], sum_im = H_im[0], an = 1.0, nfact = 1.0;
#pragma unroll
    for (int n = 1; n <= 6; n++) {
        an *= a;
        nfact *= n;
        const double t = an / nfact;
        sum_re += t * H_re[n];
        sum_im += t * H_im[n];
    }
    re = sum_re;
    im = sum_im;
}
// dilogc_fundamental (r < 1, x <= 0.732): series_3 above r = 0.98, dilogc_series_2 above 0.25, else series_1.  Every
// branch takes log(r) (series_3's expansion variable, the series' kmax): formed once, and returned in lr for
// unitdisk's log(1 - z) of a reflected argument (the same call on the same value)
NUSI_FN cd fundamental_body(double r, double x, double y, double& lr)
{
    double re, im;
    lr = GSL_LOG(r);
    if (r > 0.98) {
        cseries_3(r, lr, x, y, re, im);
        return cd{re, im};
    }
    const bool s2 = r > 0.25;
    cseries(s2, r, lr, x, y, re, im);
    if (!s2) return cd{re, im};
    // dilogc_series_2: + (1 - z) log(1 - z) / z + 1, log(1 - z) by gsl_sf_complex_log_e
    const double zr = 1.0 - x, zi = -y;
    const double ax = fabs(zr), ay = fabs(zi);
    const double mn = ax < ay ? ax : ay, mx = ax > ay ? ax : ay;
    const double ln_r = GSL_LOG(mx) + 0.5 * GSL_LOG(1.0 + (mn / mx) * (mn / mx));
    const double ln_t = GSL_ATAN2(zi, zr);
    const double t_x = (ln_r * x + ln_t * y) / (r * r);
    const double t_y = (-ln_r * y + ln_t * x) / (r * r);
    const double r_x = (1.0 - x) * t_x + y * t_y;
    const double r_y = (1.0 - x) * t_y - y * t_x;
    return cd{re + r_x + 1.0, im + r_y};
}
NUSI_FN_OUT cd fundamental(double r, double x, double y, double& lr) { return fundamental_body(r, x, y, lr); }
// dilogc_unitdisk: |z| < 1; x > 0.732 reflected, Li2(z) = -Li2(1 - z) + zeta2 - log(z) log(1 - z).  kInl: fundamental
// inline (the member-corner kernel's single call site, gsl_cli2_inl), else the out-of-line instance
template <bool kInl = false>
NUSI_FN cd unitdisk(double x, double y)
{
    const double zeta2 = kPiD * kPiD / 6.0;
    const bool refl = x > 0.732;
    const double x_tmp = 1.0 - x, y_tmp = -y;
    // the fundamental region's argument and its modulus: one hypot call site (GSL forms |z| and, reflected,
    // |1 - z|); |z| of a reflected argument after the call
    const double fx = refl ? x_tmp : x, fy = refl ? y_tmp : y;
    const double rf = gsl::hypot(fx, fy);
    double lr;
    const cd f = kInl ? fundamental_body(rf, fx, fy, lr) : fundamental(rf, fx, fy, lr);   // one call site
    if (!refl) return f;
    const double r = gsl::hypot(x, y);
    const double lnz = GSL_LOG(r), lnomz = lr;   // log(r_tmp)
    const double argz = GSL_ATAN2(y, x), argomz = GSL_ATAN2(y_tmp, x_tmp);
    return cd{-f.r + zeta2 - lnz * lnomz + argz * argomz, -f.i - argz * lnomz - argomz * lnz};
}

}  // namespace gsl

// A cost estimate of gsl_cli2(x, y), used only to order work (no value depends on it): the iterations of the series
// GSL's dispatch selects -- 0 on the real axis / unit circle, 8 for dilogc_series_3, else ~36 / -log r of the
// fundamental-region radius r (the terms fall as r^k), plus the series_2 post-processing
NUSI_FN double gsl_cli2_cost(double x, double y)
{
    const double r2 = x * x + y * y;
    if (y == 0.0 || fabs(r2 - 1.0) < gsl::kEps) return 0.0;
    double ux = x, uy = y;
    if (!(r2 < 1.0)) { ux = x / r2; uy = -y / r2; }
    const double fx = ux > 0.732 ? 1.0 - ux : ux, fy = uy;
    const double r = sqrt(fx * fx + fy * fy);
    if (r > 0.98) return 8.0;
    const double n = 36.0 / -GSL_LOG(r);
    return r > 0.25 ? 10.0 + n : n;
}

// gsl_sf_dilog (x < 0: -dilog_xge0(-x) + dilog_xge0(x^2) / 2)
NUSI_FN_OUT double gsl_li2(double x)
{
    if (x >= 0.0) return gsl::dilog_xge0(x);
    const double d1 = gsl::dilog_xge0(-x), d2 = gsl::dilog_xge0(x * x);
    return -d1 + 0.5 * d2;
}

// gsl_sf_complex_dilog_xy_e on the real axis (gsl_cli2's y == 0 branch, alone: a caller with real arguments keeps
// the complex series' registers out of its own budget)
NUSI_FN cd gsl_cli2_real(double x) { return cd{gsl_li2(x), (x >= 1.0) ? -gsl::kPiD * GSL_LOG(x) : 0.0}; }

// gsl_sf_complex_dilog_xy_e: the real axis; |z| within eps of 1 (Lewin A.2.4.1 / A.2.4.2); the unit disk; 1/z
// into the unit disk, unwound with Li2(z) + Li2(1/z) = -zeta2 - log(-z)^2 / 2.  gsl_cli2_t<true> (gsl_cli2_inl) is the
// whole call inline -- the member-corner kernel's one call site, where the call boundaries' argument moves, SGPR
// lane spills and callee-saved register traffic were VALU work of their own; gsl_cli2 the out-of-line instance the
// table kernels call from many sites
template <bool kInl>
NUSI_FN cd gsl_cli2_t(double x, double y)
{
    const double zeta2 = gsl::kPiD * gsl::kPiD / 6.0;
    const double r2 = x * x + y * y;
    if (y == 0.0) return cd{gsl_li2(x), (x >= 1.0) ? -gsl::kPiD * GSL_LOG(x) : 0.0};
    if (fabs(r2 - 1.0) < gsl::kEps) {
        const double theta = GSL_ATAN2(y, x);
        const double term1 = theta * theta / 4.0, term2 = gsl::kPiD * fabs(theta) / 2.0;
        return cd{zeta2 + term1 - term2, gsl::clausen(theta)};
    }
    const bool inv = !(r2 < 1.0);
    const cd u = gsl::unitdisk<kInl>(inv ? x / r2 : x, inv ? -y / r2 : y);   // one instance
    if (!inv) return u;
    const double r = sqrt(r2);
    const double theta = GSL_ATAN2(y, x), theta_abs = fabs(theta), theta_sgn = (theta < 0.0 ? -1.0 : 1.0);
    const double ln_minusz_re = GSL_LOG(r), ln_minusz_im = theta_sgn * (theta_abs - gsl::kPiD);
    const double lmz2_re = ln_minusz_re * ln_minusz_re - ln_minusz_im * ln_minusz_im;
    const double lmz2_im = 2.0 * ln_minusz_re * ln_minusz_im;
    return cd{-u.r - 0.5 * lmz2_re - zeta2, -u.i - 0.5 * lmz2_im};
}

NUSI_FN_OUT cd gsl_cli2(double x, double y) { return gsl_cli2_t<false>(x, y); }
#ifndef NUSI_MC_CALL   // (A/B: the member-corner kernel's GSL call out of line, as before round 6)
NUSI_FN cd gsl_cli2_inl(double x, double y) { return gsl_cli2_t<true>(x, y); }
#else
NUSI_FN cd gsl_cli2_inl(double x, double y) { return gsl_cli2(x, y); }
#endif

}  // namespace nusi
