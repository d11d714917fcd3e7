/*
 * nuSIprop oracle -- special functions.  TEST INFRASTRUCTURE ONLY.
 * See ora_specfun.h for what is restated and how it is pinned.
 *
 * Two implementations:
 *   ora_dilog / ora_complex_dilog_xy / ora_li2 / ora_li3  (used by the
 *     restatement): fp64, Bernoulli series in u = -log(1-z) after the
 *     z->1/z, z->1-z maps (Li2) and the Taylor series of Li3(1-e^-u), built
 *     from ora_libm.c and correctly rounded IEEE operations only, so that the
 *     GPU, which runs the same sequence, reproduces them bit for bit;
 *   ora_*_ld: the same functions in x87 long double, ~0.5 ulp after the
 *     final rounding -- an independent accuracy yardstick for the tests.
 */
#define _GNU_SOURCE
#include <complex.h>
#include <math.h>
#include "ora_specfun.h"
#include "ora_libm.h"
#include "ora_cplx.h"
#include "coeffs.h"

/* ------------------------------------------------------------------ fp64 -- */
static const double ZETA2 = 1.64493406684822643647;   /* pi^2/6 */
static const double PI_D = 3.14159265358979323846;

static double li2_useries(double u)
{
    const double u2 = u * u;
    double p = ora_li2_bern_d[9];
    for (int k = 8; k >= 0; --k) p = fma(p, u2, ora_li2_bern_d[k]);
    return fma(u * u2, p, u - 0.25 * u2);
}

/* reference-order arithmetic (ora_set_reference_order, test infrastructure): 1 = GSL's algorithms (ora_gsl.c) for
 * every gsl_sf_dilog / gsl_sf_complex_dilog_xy_e call site, 2 = the long-double evaluation (precision probe);
 * read-only while tables are built */
static int g_gsl_level = 0;
void ora_cdilog_set_general(int level) { g_gsl_level = level; }

/* the shared-algorithm real Li2 (the Bernoulli series after the maps; polylogarithm::Li2 always takes it) */
static double li2_bern(double x)
{
    double add = 0.0, sgn = 1.0;
    if (x > 1.0) {
        const double L = ora_log(x);
        add = 2.0 * ZETA2 - 0.5 * L * L;
        sgn = -1.0;
        x = 1.0 / x;
    } else if (x < -1.0) {
        const double L = ora_log(-x);
        add = -ZETA2 - 0.5 * L * L;
        sgn = -1.0;
        x = 1.0 / x;
    }
    if (x == 1.0) return add + sgn * ZETA2;
    if (x > 0.5) {   /* Li2(x) = zeta2 - log(x) log(1-x) - Li2(1-x); the series of Li2(1-x) takes u = -log(x) */
        const double lx = ora_log(x);
        add += sgn * (ZETA2 - lx * ora_log1p(-x));
        return add - sgn * li2_useries(-lx);
    }
    if (x == 0.0) return add;
    return add + sgn * li2_useries(-ora_log1p(-x));
}

/* gsl_sf_dilog call sites */
double ora_dilog(double x)
{
    if (g_gsl_level == 1) return ora_gsl_dilog(x);
    if (g_gsl_level == 2) return ora_dilog_ld(x);
    return li2_bern(x);
}

/* polylogarithm::Li2 (the DSNB source, nuSIprop.hpp:628-632): not GSL, the shared algorithm in every mode */
double ora_li2(double x) { return li2_bern(x); }

/* ora_dilog (same operations) with log|1 - x| and, for |x| > 1, log|x| (the logarithms it forms on its
 * way: log1p(-x), or log|x| + log1p(-1/x) after the x -> 1/x map); x != 1 */
static double dilog_ext(double x, double *L1m, double *Lx)
{
    double add = 0.0, sgn = 1.0, L = 0.0;
    if (fabs(x) > 1.0) {
        L = ora_log(fabs(x));
        add = (x > 1.0 ? 2.0 * ZETA2 : -ZETA2) - 0.5 * L * L;
        sgn = -1.0;
        x = 1.0 / x;
    }
    *Lx = L;
    if (x > 0.5) {
        const double lx = ora_log(x), l1 = ora_log1p(-x);
        *L1m = L + l1;
        add += sgn * (ZETA2 - lx * l1);
        return add - sgn * li2_useries(-lx);
    }
    if (x == 0.0) {
        *L1m = 0.0;
        return add;
    }
    const double l1 = ora_log1p(-x);
    *L1m = L + l1;
    return add + sgn * li2_useries(-l1);
}

/* Li2 about a real point x0 != 0, 1: Taylor series in d = z - x0 (radius |1 - x0|), c_0 = Li2(x0) +
 * i pi s log x0 [x0 > 1], c_1 = -log(1 - z)/z, c_{n+1} = (g^n/(n(n+1)) - c_n n/(n+1))/x0 with g = 1/(1 - x0)
 * (from z Li2'(z) = -log(1 - z)), s = +-1 the side of the cut x0 > 1, Horner in d, AXIS_TERMS + 1 terms
 * (remainder < AXIS_RATIO^7 ~ 1e-18 relative for |d| <= AXIS_RATIO min(|x0|, |1 - x0|)).  Used near the
 * real axis (d = i y) and for the alpha table's member leaves (nusi_oracle.c member_dc).  The GPU runs the
 * same sequence (nusi_math.hpp li2_taylor_*); pinned by the mpmath KATs (tests/test_specfun.py). */
#define AXIS_TERMS ORA_LI2T_TERMS
static const double AXIS_RATIO = ORA_LI2T_RATIO;
static const double kA_[AXIS_TERMS] = {0.0, 1.0 / 2, 1.0 / 6, 1.0 / 12, 1.0 / 20, 1.0 / 30};
static const double kB_[AXIS_TERMS] = {0.0, 1.0 / 2, 2.0 / 3, 3.0 / 4, 4.0 / 5, 5.0 / 6};

void ora_li2_taylor_coeffs(double x0, ora_li2t *T)
{
    const double r = 1.0 / x0, g = 1.0 / (1.0 - x0);
    double L1m, Lx;
    T->c[0] = dilog_ext(x0, &L1m, &Lx);
    T->c[1] = -L1m * r;
    double gn = g;
    for (int n = 1; n < AXIS_TERMS; ++n) {
        T->c[n + 1] = (gn * kA_[n] - kB_[n] * T->c[n]) * r;
        gn = gn * g;
    }
    T->r = r;
    T->b0 = (x0 > 1.0) ? PI_D * Lx : 0.0;
}

void ora_li2_taylor_eval(const ora_li2t *T, double dr, double di, double side, double *re, double *im)
{
    double b[AXIS_TERMS + 1];
    b[0] = side * T->b0;
    b[1] = (T->b0 != 0.0) ? side * PI_D * T->r : 0.0;
    for (int n = 1; n < AXIS_TERMS; ++n) b[n + 1] = -(kB_[n] * b[n]) * T->r;
    double sr = T->c[AXIS_TERMS], si = b[AXIS_TERMS];
    for (int n = AXIS_TERMS - 1; n >= 0; --n) {
        const double tr = T->c[n] + (sr * dr - si * di), ti = b[n] + (sr * di + si * dr);
        sr = tr;
        si = ti;
    }
    *re = sr;
    *im = si;
}

static void cdilog_axis(double x, double y, double *re, double *im)
{
    ora_li2t T;
    ora_li2_taylor_coeffs(x, &T);
    ora_li2_taylor_eval(&T, 0.0, y, y > 0.0 ? 1.0 : -1.0, re, im);
}

void ora_complex_dilog_xy(double x, double y, double *re, double *im)
{
    if (g_gsl_level == 1) {   /* GSL's algorithm (ora_gsl.c) */
        ora_gsl_complex_dilog_xy(x, y, re, im);
        return;
    }
    if (y == 0.0) {
        /* GSL: on the real axis the imaginary part is -pi*log(x) for x >= 1 */
        *re = ora_dilog(x);
        *im = (x >= 1.0) ? -PI_D * ora_log(x) : 0.0;
        return;
    }
    if (g_gsl_level == 2) {   /* (precision probe: the long-double evaluation) */
        ora_complex_dilog_xy_ld(x, y, re, im);
        return;
    }
    {
        const double ax = fabs(x), a1 = fabs(1.0 - x);
        if (fabs(y) <= AXIS_RATIO * (ax < a1 ? ax : a1)) {
            cdilog_axis(x, y, re, im);
            return;
        }
    }
    zc z = zmk(x, y), add = zmk(0.0, 0.0), lz = zmk(0.0, 0.0);
    double sgn = 1.0;
    int have_lz = 0;
    const double n2 = x * x + y * y;
    if (n2 > 1.0) {   /* Li2(z) = -zeta2 - log^2(-z)/2 - Li2(1/z) */
        const double hl = 0.5 * ora_log(n2);
        double am;   /* arg(-z): for x > 0 from arg z (|arg z| < pi/2, no cancellation), */
        if (x > 0.0) {   /* which also gives log(1/z) = -log z for the reflection below */
            const double t = ora_atan2(y, x);
            am = t - copysign(PI_D, y);
            lz = zmk(-hl, -t);
            have_lz = 1;
        } else {
            am = ora_atan2(-y, -x);
        }
        add = zmk(-ZETA2 - 0.5 * (hl * hl - am * am), -(hl * am));
        sgn = -1.0;
        const double ri = 1.0 / n2;   /* 1/z = conj(z)/|z|^2 */
        z = zmk(x * ri, -(y * ri));
    }
    zc u;   /* u = -log(1 - z) of the series' argument */
    if (z.r > 0.5) {   /* Li2(z) = zeta2 - log(z) log(1-z) - Li2(1-z); for Li2(1-z), u = -log(z) */
        if (!have_lz) lz = zlog(z);
        const zc P = zmul(lz, zlog(zmk(1.0 - z.r, -z.i)));
        add = zadd(add, zscale(sgn, zmk(ZETA2 - P.r, -P.i)));
        sgn = -sgn;
        u = zmk(-lz.r, -lz.i);
    } else {
        const double a = -z.r, b = -z.i;
        u = zmk(-0.5 * ora_log1p(2.0 * a + (a * a + b * b)), -ora_atan2(b, 1.0 + a));
    }
    const zc u2 = zmul(u, u);
    zc p = zmk(ora_li2_bern_d[ORA_LI2D_N - 1], 0.0);
    for (int k = ORA_LI2D_N - 2; k >= 0; --k) {
        p = zmul(p, u2);
        p.r = p.r + ora_li2_bern_d[k];
    }
    const zc q = zscale(0.25, u2);
    const zc s = zadd(zmk(u.r - q.r, u.i - q.i), zmul(zmul(u, u2), p));
    const zc r = zadd(add, zscale(sgn, s));
    *re = r.r;
    *im = r.i;
}

double ora_li3(double x)
{
    const double u = -ora_log1p(-x);
    double p = ora_li3_u_d[ORA_LI3U_N - 1];
    for (int k = ORA_LI3U_N - 2; k >= 0; --k) p = fma(p, u, ora_li3_u_d[k]);
    return p * u;
}

/* ----------------------------------------------------------- long double -- */
typedef long double _Complex lcplx;
static const long double LPI = 3.141592653589793238462643383279502884L;
#define LZETA2 (LPI * LPI / 6.0L)
static const long double LEPS = 1.0e-21L;

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

static long double li2_real_ld(long double x)
{
    if (x > 1.0L) {
        const long double L = logl(x);
        return 2.0L * LZETA2 - 0.5L * L * L - li2_real_ld(1.0L / x);
    }
    if (x == 1.0L) return LZETA2;
    if (x > 0.5L) return LZETA2 - logl(x) * log1pl(-x) - li2_real_ld(1.0L - x);
    if (x < -1.0L) {
        const long double L = logl(-x);
        return -LZETA2 - 0.5L * L * L - li2_real_ld(1.0L / x);
    }
    if (x == 0.0L) return 0.0L;
    return li2_bern_real(x);
}

static lcplx clog1pl(lcplx w)
{
    const long double a = creall(w), b = cimagl(w);
    return 0.5L * log1pl(2.0L * a + (a * a + b * b)) + atan2l(b, 1.0L + a) * I;
}

static lcplx li2_cplx_ld(lcplx z)
{
    const long double x = creall(z), y = cimagl(z);
    if (x * x + y * y > 1.0L) {
        const lcplx l = clogl(-z);
        return -LZETA2 - 0.5L * l * l - li2_cplx_ld(1.0L / z);
    }
    if (x > 0.5L) return LZETA2 - clogl(z) * clogl(1.0L - z) - li2_cplx_ld(1.0L - z);
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

double ora_dilog_ld(double x) { return (double)li2_real_ld((long double)x); }

void ora_complex_dilog_xy_ld(double x, double y, double *re, double *im)
{
    if (y == 0.0) {
        *im = (x >= 1.0) ? (double)(-LPI * logl((long double)x)) : 0.0;
        *re = ora_dilog_ld(x);
        return;
    }
    const lcplx r = li2_cplx_ld((long double)x + (long double)y * I);
    *re = (double)creall(r);
    *im = (double)cimagl(r);
}

double ora_li3_ld(double xd)
{
    const long double x = xd;
    if (x == 0.0L) return 0.0;
    if (x >= -0.5L && x <= 0.5L) {
        long double sum = 0.0L, p = 1.0L;
        for (int k = 1; k < 400; ++k) {
            p *= x;
            const long double t = p / ((long double)k * k * k);
            sum += t;
            if (fabsl(t) <= LEPS * fabsl(sum)) break;
        }
        return (double)sum;
    }
    if (x < -0.5L && x >= -1.0L) {   /* Li3(-e^w) = -sum_k eta(3-k) w^k/k! */
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
    return NAN;
}
