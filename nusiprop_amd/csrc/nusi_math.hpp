// nuSIprop MI355X -- fp64 special functions for the table-build kernels.
//
// Replaces the reference's third-party arithmetic boundary:
//   gsl_sf_dilog                 aux.hpp:112,129,147,165  nuSIprop.hpp:1098,1202,1375-1398
//   gsl_sf_complex_dilog_xy_e    aux.hpp:92-93            nuSIprop.hpp:1444-1451
//   polylogarithm::Li2 / Li3     nuSIprop.hpp:628-636
// and restates the cancellation-safe differences of aux.hpp:63-166.
//
// Algorithms are branch-light so that a wavefront stays converged:
//   * real / complex Li2: map z -> 1/z (|z| > 1) and z -> 1-z (Re z > 1/2),
//     then the Bernoulli series in u = -log(1-z) (|u| <= pi/3) -- one log1p
//     and a fixed-length Horner polynomial, no data-dependent iteration count;
//   * Li3 on [-1, 1/2]: Taylor series of Li3(1 - e^-u), |u| <= ln 2.
// GSL conventions kept: gsl_sf_dilog(x>1) = Re Li2(x); complex dilog on the
// real axis (y == 0) has Im = -pi*log(x) for x >= 1 and 0 below.
//
// Everything is NUSI_FN (host+device) so that tests/ can compile the same
// source for the CPU and check it against the oracle; the product library
// only ever executes it on the GPU.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

#include "nusi_coeffs.hpp"
#include "nusi_libm.hpp"

#define NUSI_FN __host__ __device__ inline
// Polylogarithms are called from many sites; outlining them keeps the table
// kernels' code small (NUSI_INLINE_POLYLOG inlines them everywhere, A/B builds).
#ifdef NUSI_INLINE_POLYLOG
#define NUSI_FN_OUT NUSI_FN
#else
#define NUSI_FN_OUT __host__ __device__ inline __attribute__((noinline))
#endif

// Inside the (out-of-line) polylogarithms the elementary functions are inlined: a call there
// costs a register save/restore round trip per log (-DNUSI_POLY_CALL_LIBM: calls, A/B builds).
#ifdef NUSI_POLY_CALL_LIBM
#define NUSI_PLOG nm::log
#define NUSI_PLOG1P nm::log1p
#define NUSI_PATAN2 nm::atan2
#else
#define NUSI_PLOG nm::log_i
#define NUSI_PLOG1P nm::log1p_i
#define NUSI_PATAN2 nm::atan2_i
#endif

namespace nusi {

constexpr double kPi = 3.14159265358979323846;
constexpr double kZeta2 = 1.64493406684822643647;  // pi^2/6

// ---------------------------------------------------------------------------
// complex double with C99 `double _Complex` semantics (GNU C): real operands
// are not promoted in +,-,* ; division uses Smith's algorithm like libgcc's
// __divdc3 does for finite operands.
// ---------------------------------------------------------------------------
struct cd {
    double r, i;
};
NUSI_FN cd C(double r, double i = 0.0) { return cd{r, i}; }
NUSI_FN cd operator+(cd a, cd b) { return cd{a.r + b.r, a.i + b.i}; }
NUSI_FN cd operator-(cd a, cd b) { return cd{a.r - b.r, a.i - b.i}; }
NUSI_FN cd operator-(cd a) { return cd{-a.r, -a.i}; }
NUSI_FN cd operator+(cd a, double s) { return cd{a.r + s, a.i}; }
NUSI_FN cd operator+(double s, cd a) { return cd{s + a.r, a.i}; }
NUSI_FN cd operator-(cd a, double s) { return cd{a.r - s, a.i}; }
NUSI_FN cd operator-(double s, cd a) { return cd{s - a.r, -a.i}; }
NUSI_FN cd operator*(cd a, cd b) { return cd{a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
NUSI_FN cd operator*(double s, cd a) { return cd{s * a.r, s * a.i}; }
NUSI_FN cd operator*(cd a, double s) { return cd{a.r * s, a.i * s}; }
NUSI_FN cd operator/(cd a, double s) { return cd{a.r / s, a.i / s}; }
NUSI_FN cd operator/(cd a, cd b)
{
    const double c = b.r, d = b.i;
    if (fabs(c) < fabs(d)) {
        const double ratio = c / d, den = (c * ratio) + d;
        return cd{((a.r * ratio) + a.i) / den, ((a.i * ratio) - a.r) / den};
    }
    const double ratio = d / c, den = (d * ratio) + c;
    return cd{((a.i * ratio) + a.r) / den, (a.i - (a.r * ratio)) / den};
}
NUSI_FN cd operator/(double s, cd b) { return C(s) / b; }
NUSI_FN cd conj(cd a) { return cd{a.r, -a.i}; }
NUSI_FN double carg(cd z) { return nm::atan2(z.i, z.r); }
NUSI_FN double carg_i(cd z) { return nm::atan2_i(z.i, z.r); }
NUSI_FN double carg_real(double x) { return nm::atan2(0.0, x); }  // carg of a real promoted to complex
NUSI_FN double cabs(cd z) { return sqrt(z.r * z.r + z.i * z.i); }
NUSI_FN cd clog(cd z) { return cd{0.5 * nm::log(z.r * z.r + z.i * z.i), carg(z)}; }
NUSI_FN cd clog_p(cd z) { return cd{0.5 * NUSI_PLOG(z.r * z.r + z.i * z.i), NUSI_PATAN2(z.i, z.r)}; }   // clog, polylog-internal
NUSI_FN cd clog_real(double x) { return clog(C(x, 0.0)); }   // clog of a promoted real
NUSI_FN cd sqr(cd a) { return a * a; }
constexpr cd kI = {0.0, 1.0};

// ---------------------------------------------------------------------------
// polylogarithms
// ---------------------------------------------------------------------------
// u - u^2/4 + sum_k B_2k u^(2k+1)/(2k+1)!  for |u| <= ln 2 (10 terms reach 1e-17)
NUSI_FN double li2_useries(double u)
{
    const double u2 = u * u;
    double p = kLi2Bern[9];
#pragma unroll
    for (int k = 8; k >= 0; --k) p = fma(p, u2, kLi2Bern[k]);
    return fma(u * u2, p, u - 0.25 * u2);
}

// Re Li2(x) for real x (gsl_sf_dilog semantics)
NUSI_FN_OUT double li2(double x)
{
    double add = 0.0, sgn = 1.0;
    if (fabs(x) > 1.0) {   // x > 1: 2 zeta2 - log^2(x)/2 ; x < -1: -zeta2 - log^2(-x)/2 (one log for both)
        const double L = NUSI_PLOG(fabs(x));
        add = (x > 1.0 ? 2.0 * kZeta2 : -kZeta2) - 0.5 * L * L;
        sgn = -1.0;
        x = 1.0 / x;
    }
    if (x == 1.0) return add + sgn * kZeta2;
    if (x > 0.5) {   // Li2(x) = zeta2 - log(x) log(1-x) - Li2(1-x); the series of Li2(1-x) takes u = -log(x)
        const double lx = NUSI_PLOG(x);
        add += sgn * (kZeta2 - lx * NUSI_PLOG1P(-x));
        return add - sgn * li2_useries(-lx);
    }
    if (x == 0.0) return add;
    return add + sgn * li2_useries(-NUSI_PLOG1P(-x));
}

// Re Li2(x) (li2's algorithm and bits) together with log|1 - x| and, for |x| > 1, log|x| -- the
// logarithms li2 forms on its way (log1p(-x) of the series argument, or log|x| + log1p(-1/x) after the
// x -> 1/x map), for the near-axis complex path below; x != 1
NUSI_FN double li2_ext(double x, double& L1m, double& Lx)
{
    double add = 0.0, sgn = 1.0, L = 0.0;
    if (fabs(x) > 1.0) {
        L = NUSI_PLOG(fabs(x));
        add = (x > 1.0 ? 2.0 * kZeta2 : -kZeta2) - 0.5 * L * L;
        sgn = -1.0;
        x = 1.0 / x;
    }
    Lx = L;
    if (x > 0.5) {
        const double lx = NUSI_PLOG(x), l1 = NUSI_PLOG1P(-x);
        L1m = L + l1;
        add += sgn * (kZeta2 - lx * l1);
        return add - sgn * li2_useries(-lx);
    }
    if (x == 0.0) {
        L1m = 0.0;
        return add;
    }
    const double l1 = NUSI_PLOG1P(-x);
    L1m = L + l1;
    return add + sgn * li2_useries(-l1);
}

// Li2 about a real point x0 (x0 != 0, 1): the Taylor series in d = z - x0 (radius |1 - x0|, the distance to
// the branch point),
//   Li2(x0 + d) = sum_n c_n d^n,  c_n = Li2^(n)(x0) / n!,
//   c_0 = Li2(x0) + i pi s log(x0) [x0 > 1],  c_1 = -log(1 - z) / z (log(1 - z) = log(x0 - 1) - i pi s for
//   x0 > 1), c_{n+1} = (g^n / (n (n + 1)) - c_n n / (n + 1)) / x0 with g = 1 / (1 - x0)
// (from z Li2'(z) = -log(1 - z)); s = +-1 is the side of the cut x0 > 1 the point x0 + d lies on.
// Summed by Horner in d, truncated after kLi2AxisTerms: for |d| <= kLi2AxisRatio min(|x0|, |1 - x0|) the
// remainder is below kLi2AxisRatio^7 ~ 1e-18 relative.  The coefficients are one real Li2 (whose
// logarithms give log|1 - x0| and log x0) and two divisions; the evaluation is 6 complex fma steps.
// Used (a) for arguments next to the real axis (cli2: x0 = Re z, d = i Im z), and (b) by the alpha table's
// member leaves, whose arguments w = (1 + S + t) / (2 + t - i gr) all lie close to the real point
// (1 + S + t) / (2 + t) that the points of a batch share: the coefficients are formed once per batch,
// each point only evaluates.  Same algorithm as the oracle (ora_specfun.c ora_li2_taylor_*).
constexpr int kLi2AxisTerms = 6;
constexpr double kLi2AxisRatio = 2.5e-3;
struct Li2Taylor {
    double c[kLi2AxisTerms + 1];   // real parts of c_n
    double r, b0;                  // 1 / x0 ; pi log(x0) for x0 > 1, else 0
};
NUSI_FN void li2_taylor_coeffs(double x0, Li2Taylor& T)
{
    constexpr double kA[kLi2AxisTerms] = {0.0, 1.0 / 2, 1.0 / 6, 1.0 / 12, 1.0 / 20, 1.0 / 30};   // 1 / (n (n + 1))
    constexpr double kB[kLi2AxisTerms] = {0.0, 1.0 / 2, 2.0 / 3, 3.0 / 4, 4.0 / 5, 5.0 / 6};     // n / (n + 1)
    const double r = 1.0 / x0, g = 1.0 / (1.0 - x0);
    double L1m, Lx;   // log|1 - x0|, log x0 (x0 > 1)
    T.c[0] = li2_ext(x0, L1m, Lx);
    T.c[1] = -L1m * r;
    double gn = g;
#pragma unroll
    for (int n = 1; n < kLi2AxisTerms; ++n) {
        T.c[n + 1] = (gn * kA[n] - kB[n] * T.c[n]) * r;
        gn = gn * g;
    }
    T.r = r;
    T.b0 = (x0 > 1.0) ? kPi * Lx : 0.0;
}
NUSI_FN cd li2_taylor_eval(const Li2Taylor& T, double dr, double di, double side)
{
    constexpr double kB[kLi2AxisTerms] = {0.0, 1.0 / 2, 2.0 / 3, 3.0 / 4, 4.0 / 5, 5.0 / 6};
    double b[kLi2AxisTerms + 1];   // imaginary parts of c_n (x0 > 1 only): b_1 = pi s / x0, b_{n+1} = -b_n n / (n + 1) / x0
    b[0] = side * T.b0;
    b[1] = (T.b0 != 0.0) ? side * kPi * T.r : 0.0;
#pragma unroll
    for (int n = 1; n < kLi2AxisTerms; ++n) b[n + 1] = -(kB[n] * b[n]) * T.r;
    double sr = T.c[kLi2AxisTerms], si = b[kLi2AxisTerms];
#pragma unroll
    for (int n = kLi2AxisTerms - 1; n >= 0; --n) {
        const double tr = T.c[n] + (sr * dr - si * di), ti = b[n] + (sr * di + si * dr);
        sr = tr;
        si = ti;
    }
    return cd{sr, si};
}
// Li2(x + iy) close to the real axis, |y| <= kLi2AxisRatio min(|x|, |1 - x|)
NUSI_FN cd cli2_axis(double x, double y)
{
    Li2Taylor T;
    li2_taylor_coeffs(x, T);
    return li2_taylor_eval(T, 0.0, y, y > 0.0 ? 1.0 : -1.0);
}

// principal-branch Li2(x+iy); y == 0 follows gsl_sf_complex_dilog_xy_e.  cli2_body is the inline body
// (one call site of the big-batch alpha kernel inlines it), cli2 the out-of-line entry point.  The shared-algorithm
// series; NUSI_OPT_REFERENCE_ORDER runs GSL's own algorithm instead (gsl_cli2, nusi_gsl.hpp)
NUSI_FN cd cli2_body(double x, double y)
{
    if (y == 0.0) return cd{li2(x), (x >= 1.0) ? -kPi * NUSI_PLOG(x) : 0.0};
    {
        const double ax = fabs(x), a1 = fabs(1.0 - x);
        if (fabs(y) <= kLi2AxisRatio * (ax < a1 ? ax : a1)) return cli2_axis(x, y);
    }
    cd z = C(x, y), add = C(0.0), lz;
    double sgn = 1.0;
    bool have_lz = false;
    const double n2 = x * x + y * y;
    if (n2 > 1.0) {   // Li2(z) = -zeta2 - log^2(-z)/2 - Li2(1/z)
        const double hl = 0.5 * NUSI_PLOG(n2);
        double am;   // arg(-z); for x > 0 it comes from arg z (no cancellation: |arg z| < pi/2),
        if (x > 0.0) {   // which then also gives log(1/z) = -log z for the reflection below
            const double t = NUSI_PATAN2(y, x);
            am = t - copysign(kPi, y);
            lz = C(-hl, -t);
            have_lz = true;
        } else {
            am = NUSI_PATAN2(-y, -x);
        }
        add = C(-kZeta2 - 0.5 * (hl * hl - am * am), -(hl * am));
        sgn = -1.0;
        const double ri = 1.0 / n2;   // 1/z = conj(z)/|z|^2
        z = C(x * ri, -(y * ri));
    }
    cd u;   // u = -log(1 - z) of the series' argument
    if (z.r > 0.5) {   // Li2(z) = zeta2 - log(z) log(1-z) - Li2(1-z); for Li2(1-z), u = -log(z)
        if (!have_lz) lz = clog_p(z);
        add = add + sgn * (kZeta2 - lz * clog_p(1.0 - z));
        sgn = -sgn;
        u = C(-lz.r, -lz.i);
    } else {   // formed without the cancellation of 1 - z for small z
        const double a = -z.r, b = -z.i;
        u = C(-0.5 * NUSI_PLOG1P(2.0 * a + (a * a + b * b)), -NUSI_PATAN2(b, 1.0 + a));
    }
    const cd u2 = u * u;
    cd p = C(kLi2Bern[kLi2Terms - 1]);
#pragma unroll
    for (int k = kLi2Terms - 2; k >= 0; --k) p = p * u2 + kLi2Bern[k];
    const cd s = (u - 0.25 * u2) + (u * u2) * p;
    return add + sgn * s;
}
NUSI_FN_OUT cd cli2(double x, double y) { return cli2_body(x, y); }
NUSI_FN cd cli2(cd z) { return cli2(z.r, z.i); }
}  // namespace nusi

#include "nusi_gsl.hpp"

namespace nusi {
// the dilogarithms of a gsl_sf_dilog / gsl_sf_complex_dilog_xy_e call site: the shared-algorithm series, or
// (kRef, NUSI_OPT_REFERENCE_ORDER) GSL's algorithm
template <bool kRef>
NUSI_FN cd cli2_t(cd z) { return kRef ? gsl_cli2(z.r, z.i) : cli2(z.r, z.i); }
template <bool kRef>
NUSI_FN cd cli2_t(double x, double y) { return kRef ? gsl_cli2(x, y) : cli2(x, y); }
template <bool kRef>
NUSI_FN double li2_t(double x) { return kRef ? gsl_li2(x) : li2(x); }
template <bool kRef>
NUSI_FN cd cli2_real_t(double x) { return kRef ? gsl_cli2_real(x) : cli2(x, 0.0); }

// Li3(x), x in [-1, 1/2] (the DSNB source only reaches [-1, 0))
NUSI_FN double li3(double x)
{
    const double u = -nm::log1p(-x);
    double p = kLi3U[kLi3Terms - 1];
#pragma unroll
    for (int k = kLi3Terms - 2; k >= 0; --k) p = fma(p, u, kLi3U[k]);
    return p * u;
}

// ---------------------------------------------------------------------------
// aux.hpp restatements (same thresholds and Taylor coefficients)
// ---------------------------------------------------------------------------
// 3-point Gauss-Legendre, aux.hpp:53-54
constexpr double kGLw[3] = {5. / 9., 8. / 9., 5. / 9.};
constexpr double kGLx[3] = {-0.7745966692414834, 0.0, 0.7745966692414834};  // sqrt(3./5.)

// aux.hpp:63-75
NUSI_FN double atandiff(double x, double y)
{
    if (fabs(x) < 1e2 || fabs(y) < 1e2 || x * y < 0) return nm::atan(x) - nm::atan(y);
    const double ix = 1. / x, iy = 1. / y;
    return -ix + ix * ix * ix / 3. - (-iy + iy * iy * iy / 3.);
}

// large-|z| Li2 used by aux.hpp:84-89
NUSI_FN cd li2_asym(cd z)
{
    const double s = (z.i >= 0) ? 1.0 : -1.0;
    const cd L = clog(z);
    const cd z2 = z * z;
    const cd t = (-s * 2 * kPi) * L - kI * (L * L);
    return -1 / (16. * (z2 * z2)) - 1 / (9. * (z * z * z)) - 1 / (4. * z2) - 1 / z - C(0.0, 0.5) * t;
}

// aux.hpp:77-96 (kRef: GSL's complex dilogarithm, NUSI_OPT_REFERENCE_ORDER)
template <bool kRef = false>
NUSI_FN cd dilogdiff_c(cd x, cd y)
{
    if (cabs(x) > 1e2 && cabs(y) > 1e2) return li2_asym(x) - li2_asym(y);
    const cd a = cli2_t<kRef>(x), b = cli2_t<kRef>(y);
    return C(a.r - b.r, a.i - b.i);
}

// aux.hpp:98-113 : Li2(-x) - Li2(-y)
template <bool kRef = false>
NUSI_FN double dilogdiff(double x, double y)
{
    if (x > 1e2 && y > 1e2) {
        const double lx = nm::log(x), ly = nm::log(y), ix = 1. / x, iy = 1. / y;
        return -lx * lx / 2. + ix - ix * ix / 4. + ix * ix * ix / 9. - (ix * ix) * (ix * ix) / 16
               - (-ly * ly / 2. + iy - iy * iy / 4. + iy * iy * iy / 9. - (iy * iy) * (iy * iy) / 16);
    }
    if (x < 1e-2 && y < 1e-2)
        return -x + x * x / 4. - x * x * x / 9. + (x * x) * (x * x) / 16.
               - (-y + y * y / 4. - y * y * y / 9. + (y * y) * (y * y) / 16.);
    return li2_t<kRef>(-x) - li2_t<kRef>(-y);
}

// aux.hpp:115-130 : Li2(-1-x) - Li2(-1-y)
NUSI_FN double d1m_big(double v)
{
    const double l = nm::log(v);
    return -l * l / 2. + (1 - l) / v + (-7 + 2 * l) / (4. * (v * v)) + (19 - 3 * l) / (9. * (v * v * v))
           + (-125 + 12 * l) / (48. * ((v * v) * (v * v)));
}
NUSI_FN double d1m_small(double v)
{
    const double ln2 = 0.6931471805599453, ln4 = 1.3862943611198906;
    return -v * ln2 + (v * v * (-1 + ln4)) / 4. + (v * v * v * (5 - 8 * ln2)) / 24.
           + (v * v) * (v * v) * (-1. / 6. + ln2 / 4.);
}
template <bool kRef = false>
NUSI_FN double dilog1mdiff(double x, double y)
{
    if (x > 1e2 && y > 1e2) return d1m_big(x) - d1m_big(y);
    if (x < 1e-2 && y < 1e-2) return d1m_small(x) - d1m_small(y);
    return li2_t<kRef>(-1 - x) - li2_t<kRef>(-1 - y);
}

// aux.hpp:132-148 : Li2(1+x) - Li2(1+y), x,y < 0
NUSI_FN double d1p_big(double v)
{
    const double l = nm::log(-v);
    return (-1 - 3 * l) / (9. * (v * v * v)) + (-1 - l) / v - l * l / 2. + (1 + 2 * l) / (4. * (v * v))
           + (1 + 4 * l) / (16. * ((v * v) * (v * v)));
}
NUSI_FN double d1p_small(double v)
{
    const double l = nm::log(-v);
    return v * (1 - l) + (v * v * (-1 + 2 * l)) / 4. + (v * v * v * (1 - 3 * l)) / 9.
           + ((v * v) * (v * v) * (-1 + 4 * l)) / 16.;
}
template <bool kRef = false>
NUSI_FN double dilog1pdiff(double x, double y)
{
    if (-x > 1e2 && -y > 1e2) return d1p_big(x) - d1p_big(y);
    if (-x < 1e-2 && -y < 1e-2) return d1p_small(x) - d1p_small(y);
    return li2_t<kRef>(1 + x) - li2_t<kRef>(1 + y);
}

// aux.hpp:150-166 : Li2(1/(1-x)) - Li2(1/(1-y)), x,y < 0
NUSI_FN double d1o_big(double v)
{
    return -25 / (48. * ((v * v) * (v * v))) - 11 / (18. * (v * v * v)) - 3 / (4. * (v * v)) - 1 / v;
}
NUSI_FN double d1o_small(double v)
{
    const double l = nm::log(-v);
    return ((v * v) * (v * v) * (-19 - 12 * l)) / 48. + (v * v * v * (-7 - 6 * l)) / 18.
           + (v * v * (-1 - 2 * l)) / 4. + v * (1 - l);
}
template <bool kRef = false>
NUSI_FN double dilog1over1mdiff(double x, double y)
{
    if (-x > 1e2 && -y > 1e2) return d1o_big(x) - d1o_big(y);
    if (-x < 1e-2 && -y < 1e-2) return d1o_small(x) - d1o_small(y);
    return li2_t<kRef>(1 / (1 - x)) - li2_t<kRef>(1 / (1 - y));
}

// Edge-shared forms (k_gamma_alphat, the Gamma / alphaTilde kernel): a difference f(x) - f(y) of the two edges of a
// bin takes its branch from both arguments, and in the middle branch it evaluates f at each edge -- a function of one
// bin edge, equal bit for bit for the two bins an edge bounds (hi[n] == lo[n + 1]).  The *_mid predicates are the
// branch tests, the *_pre forms take the middle branch's two values from the caller (evaluated once per edge); the
// other branches are the functions above, unchanged.
NUSI_FN bool dilogdiff_mid(double x, double y) { return !(x > 1e2 && y > 1e2) && !(x < 1e-2 && y < 1e-2); }
NUSI_FN bool dilog1mdiff_mid(double x, double y) { return dilogdiff_mid(x, y); }
NUSI_FN bool dilog1pdiff_mid(double x, double y) { return !(-x > 1e2 && -y > 1e2) && !(-x < 1e-2 && -y < 1e-2); }
NUSI_FN bool dilog1over1mdiff_mid(double x, double y) { return dilog1pdiff_mid(x, y); }
NUSI_FN bool dilogdiff_c_mid(cd x, cd y) { return !(cabs(x) > 1e2 && cabs(y) > 1e2); }
NUSI_FN double dilogdiff_pre(double x, double y, double lx, double ly)
{
    return dilogdiff_mid(x, y) ? lx - ly : dilogdiff<false>(x, y);   // (the other branches call no dilogarithm)
}
NUSI_FN double dilog1mdiff_pre(double x, double y, double lx, double ly)
{
    return dilog1mdiff_mid(x, y) ? lx - ly : dilog1mdiff<false>(x, y);
}
NUSI_FN double dilog1pdiff_pre(double x, double y, double lx, double ly)
{
    return dilog1pdiff_mid(x, y) ? lx - ly : dilog1pdiff<false>(x, y);
}
NUSI_FN double dilog1over1mdiff_pre(double x, double y, double lx, double ly)
{
    return dilog1over1mdiff_mid(x, y) ? lx - ly : dilog1over1mdiff<false>(x, y);
}
NUSI_FN cd dilogdiff_c_pre(cd x, cd y, cd a, cd b)
{
    return dilogdiff_c_mid(x, y) ? C(a.r - b.r, a.i - b.i) : dilogdiff_c<false>(x, y);
}

}  // namespace nusi
