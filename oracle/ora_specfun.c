/*
 * nuSIprop oracle -- special functions.  TEST INFRASTRUCTURE ONLY.
 * See ora_specfun.h for what is restated and how it is pinned.
 */
#define _GNU_SOURCE
#include <complex.h>
#include <math.h>
#include "ora_specfun.h"
#include "coeffs.h"

typedef long double _Complex lcplx;

static const long double LPI = 3.141592653589793238462643383279502884L;
#define LZETA2 (LPI * LPI / 6.0L)
static const long double LEPS = 1.0e-21L;

/* Li2(z) = u - u^2/4 + sum_k B_2k u^(2k+1)/(2k+1)!,  u = -log(1-z)  (real) */
static long double li2_bern_real(long double x)
{
    const long double u = -log1pl(-x);
    const long double u2 = u * u;
    long double sum = u - 0.25L * u2;
    long double p = u;
    for (int k = 0; k < ORA_LI2_NB; ++k) {
        p *= u2;
        const long double t = ora_li2_bern[k] * p;
        sum += t;
        if (fabsl(t) <= LEPS * fabsl(sum)) break;
    }
    return sum;
}

/* Re Li2(x) for every real x (GSL gsl_sf_dilog semantics). */
static long double li2_real_ld(long double x)
{
    if (x > 1.0L) {                  /* Re Li2(x) = pi^2/3 - ln^2(x)/2 - Li2(1/x) */
        const long double L = logl(x);
        return 2.0L * LZETA2 - 0.5L * L * L - li2_real_ld(1.0L / x);
    }
    if (x == 1.0L) return LZETA2;
    if (x > 0.5L)                    /* Li2(x) = pi^2/6 - ln(x) ln(1-x) - Li2(1-x) */
        return LZETA2 - logl(x) * log1pl(-x) - li2_real_ld(1.0L - x);
    if (x < -1.0L) {                 /* Li2(x) = -pi^2/6 - ln^2(-x)/2 - Li2(1/x) */
        const long double L = logl(-x);
        return -LZETA2 - 0.5L * L * L - li2_real_ld(1.0L / x);
    }
    if (x == 0.0L) return 0.0L;
    return li2_bern_real(x);         /* -1 <= x <= 1/2: |u| <= ln 2 */
}

/* log(1+w) without the cancellation of forming 1+w for small w */
static lcplx clog1pl(lcplx w)
{
    const long double a = creall(w), b = cimagl(w);
    const long double re = 0.5L * log1pl(2.0L * a + (a * a + b * b));
    const long double im = atan2l(b, 1.0L + a);
    return re + im * I;
}

/* principal-branch complex Li2 */
static lcplx li2_cplx_ld(lcplx z)
{
    const long double x = creall(z), y = cimagl(z);
    if (x * x + y * y > 1.0L) {      /* Li2(z) = -pi^2/6 - ln^2(-z)/2 - Li2(1/z) */
        const lcplx l = clogl(-z);
        return -LZETA2 - 0.5L * l * l - li2_cplx_ld(1.0L / z);
    }
    if (x > 0.5L)                    /* Li2(z) = pi^2/6 - ln z ln(1-z) - Li2(1-z) */
        return LZETA2 - clogl(z) * clogl(1.0L - z) - li2_cplx_ld(1.0L - z);
    if (x == 0.0L && y == 0.0L) return 0.0L;
    const lcplx u = -clog1pl(-z);
    const lcplx u2 = u * u;
    lcplx sum = u - 0.25L * u2;
    lcplx p = u;
    for (int k = 0; k < ORA_LI2_NB; ++k) {
        p *= u2;
        const lcplx t = ora_li2_bern[k] * p;
        sum += t;
        if (cabsl(t) <= LEPS * cabsl(sum)) break;
    }
    return sum;
}

double ora_dilog(double x) { return (double)li2_real_ld((long double)x); }

double ora_li2(double x) { return (double)li2_real_ld((long double)x); }

void ora_complex_dilog_xy(double x, double y, double *re, double *im)
{
    if (y == 0.0) {
        /* GSL: on the real axis the imaginary part is -pi*log(x) for x >= 1 */
        *im = (x >= 1.0) ? -M_PI * log(x) : 0.0;
        *re = ora_dilog(x);
        return;
    }
    const lcplx r = li2_cplx_ld((long double)x + (long double)y * I);
    *re = (double)creall(r);
    *im = (double)cimagl(r);
}

/* Li3(x), real x in [-1, 1/2]. */
double ora_li3(double xd)
{
    const long double x = xd;
    if (x == 0.0L) return 0.0;
    if (x >= -0.5L && x <= 0.5L) {   /* sum x^k / k^3 */
        long double sum = 0.0L, p = 1.0L;
        for (int k = 1; k < 400; ++k) {
            p *= x;
            const long double t = p / ((long double)k * k * k);
            sum += t;
            if (fabsl(t) <= LEPS * fabsl(sum)) break;
        }
        return (double)sum;
    }
    if (x < -0.5L && x >= -1.0L) {   /* Li3(-e^w) = -sum_k eta(3-k) w^k/k!,  w = ln(-x) */
        const long double w = logl(-x);
        long double sum = 0.0L, p = 1.0L;
        for (int k = 0; k < ORA_LI3_NE; ++k) {
            const long double t = ora_li3_eta[k] * p;
            sum += t;
            if (k > 4 && fabsl(t) <= LEPS * fabsl(sum) && t != 0.0L) break;
            p *= w;
        }
        return (double)(-sum);
    }
    return NAN;  /* not reached by the reference's Lum_int (argument -exp(-y) in [-1,0)) */
}
