/*
 * nuSIprop oracle -- GSL's dilogarithm algorithms, restated.  TEST INFRASTRUCTURE ONLY.
 *
 * The reference evaluates its closed forms with two GSL functions (GSL version unpinned: the Homebrew build named
 * in setup.py:10-11; GSL is absent from this image and from /root/reference):
 *   gsl_sf_dilog(x)                      aux.hpp:112,129,147,165   nuSIprop.hpp:1098,1202,1375-1398
 *   gsl_sf_complex_dilog_xy_e(x,y,..)    aux.hpp:92-93             nuSIprop.hpp:1444-1451
 * This file restates their published algorithm (GSL 2.x specfunc/dilog.c, with the helpers it calls from
 * specfunc/clausen.c, specfunc/log.c, specfunc/trig.c and specfunc/cheb_eval.c), function by function, with the
 * same branch points, series, loop bounds and stopping tests, in the same operation order:
 *   real:    dilog_xge0 (x > 2: 1/x map; 1.01 < x <= 2: 1 - 1/x map; 1 < x <= 1.01: series about 1; x == 1;
 *            1/2 < x < 1: 1 - x map; 1/4 < x <= 1/2: dilog_series_2; 0 < x <= 1/4: dilog_series_1), and
 *            x < 0 as -dilog_xge0(-x) + dilog_xge0(x^2)/2;
 *   complex: y == 0 -> the real function with Im = -pi log x for x >= 1; |z|^2 within eps of 1 -> Lewin's
 *            formula with Clausen's function; |z| > 1 -> 1/z, unwound with log(-z)^2; in the unit disk
 *            dilogc_unitdisk maps x > 0.732 to 1 - z, and dilogc_fundamental sums dilogc_series_1 (|z| <= 1/4),
 *            dilogc_series_2 (1/4 < |z| <= 0.98: the one-step accelerated series) or dilogc_series_3 (|z| > 0.98:
 *            the expansion in log|z| about the unit circle).
 * Only the values are kept (GSL's error estimates do not feed the reference).  The elementary functions are the
 * shared fp64 ones of ora_libm.c (log, atan2) plus ora_hypot below; sqrt, floor and the four operations are
 * IEEE.  So this is GSL's algorithm on this repository's libm: the GPU (nusi_math.hpp gsl_*) runs the same
 * sequence bit for bit.  What it cannot restate is the platform the reference was built on (Apple's libm, and
 * g++-14 -O3 -std=gnu++11 on arm64, which contracts a*b + c into fused multiply-adds by default): DESIGN.md sec. 2.
 * Accuracy pinned by the mpmath known-answer vectors (tests/test_specfun.py).
 */
#define _GNU_SOURCE
#include <math.h>
#include "ora_specfun.h"
#include "ora_libm.h"

#define GSL_DBL_EPSILON 2.2204460492503131e-16
#define GSL_SQRT_DBL_EPSILON 1.4901161193847656e-08

/* iteration counts of the series loops (ora_gsl_stats; analysis only) */
static _Thread_local long g_stat[8];
void ora_gsl_stats(long *out, int reset)
{
    for (int i = 0; i < 8; ++i) {
        if (out) out[i] = g_stat[i];
        if (reset) g_stat[i] = 0;
    }
}

/* hypot(x, y) (C99 libm, called by dilogc_unitdisk): sqrt(a^2 + b^2) with one correction step from the exact
 * residual a^2 + b^2 - h^2 (the products' low parts by fma); the GPU runs the same sequence (nm::hypot) */
double ora_hypot(double x, double y)
{
    double a = fabs(x), b = fabs(y);
    if (a < b) { const double t = a; a = b; b = t; }
    if (b == 0.0 || !(a <= 1.79769313486231570815e+308)) return a + b;   /* 0, inf, nan */
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

/* ---------------------------------------------------------------- real -- */
/* dilog_series_1: sum x^k / k^2, |x| <= 1/4 */
static double dilog_series_1(const double x)
{
    const int kmax = 1000;
    double sum = x;
    double term = x;
    int k;
    for (k = 2; k < kmax; k++) {
        const double rk = (k - 1.0) / k;
        term *= x;
        term *= rk * rk;
        sum += term;
        if (fabs(term / sum) < GSL_DBL_EPSILON) break;
    }
    g_stat[0] += k;
    return sum;
}

/* series_2: sum r^k / (k^2 (k + 1)), the first nine terms unconditionally */
static double series_2(double r)
{
    static const int kmax = 100;
    double rk = r;
    double sum = 0.5 * r;
    int k;
    for (k = 2; k < 10; k++) {
        double ds;
        rk *= r;
        ds = rk / (k * k * (k + 1.0));
        sum += ds;
    }
    for (; k < kmax; k++) {
        double ds;
        rk *= r;
        ds = rk / (k * k * (k + 1.0));
        sum += ds;
        if (fabs(ds / sum) < 0.5 * GSL_DBL_EPSILON) break;
    }
    g_stat[1] += k;
    return sum;
}

/* dilog_series_2: Li2(x) = 1 + (1 - x) log(1 - x) / x + series_2(x), -1 < x < 1 */
static double dilog_series_2(double x)
{
    double val = series_2(x);
    double t;
    if (x > 0.01)
        t = (1.0 - x) * ora_log(1.0 - x) / x;
    else {
        static const double c3 = 1.0 / 3.0;
        static const double c4 = 1.0 / 4.0;
        static const double c5 = 1.0 / 5.0;
        static const double c6 = 1.0 / 6.0;
        static const double c7 = 1.0 / 7.0;
        static const double c8 = 1.0 / 8.0;
        const double t68 = c6 + x * (c7 + x * c8);
        const double t38 = c3 + x * (c4 + x * (c5 + x * t68));
        t = (x - 1.0) * (1.0 + x * (0.5 + x * t38));
    }
    val += 1.0 + t;
    return val;
}

/* dilog_xge0: Li2(x), x >= 0 (Re Li2 for x > 1) */
static double dilog_xge0(const double x)
{
    if (x > 2.0) {
        const double ser = dilog_series_2(1.0 / x);
        const double log_x = ora_log(x);
        const double t1 = M_PI * M_PI / 3.0;
        const double t2 = ser;
        const double t3 = 0.5 * log_x * log_x;
        return t1 - t2 - t3;
    } else if (x > 1.01) {
        const double ser = dilog_series_2(1.0 - 1.0 / x);
        const double log_x = ora_log(x);
        const double log_term = log_x * (ora_log(1.0 - 1.0 / x) + 0.5 * log_x);
        const double t1 = M_PI * M_PI / 6.0;
        const double t2 = ser;
        const double t3 = log_term;
        return t1 + t2 - t3;
    } else if (x > 1.0) {
        /* series around x = 1.0 */
        const double eps = x - 1.0;
        const double lne = ora_log(eps);
        const double c0 = M_PI * M_PI / 6.0;
        const double c1 = 1.0 - lne;
        const double c2 = -(1.0 - 2.0 * lne) / 4.0;
        const double c3 = (1.0 - 3.0 * lne) / 9.0;
        const double c4 = -(1.0 - 4.0 * lne) / 16.0;
        const double c5 = (1.0 - 5.0 * lne) / 25.0;
        const double c6 = -(1.0 - 6.0 * lne) / 36.0;
        const double c7 = (1.0 - 7.0 * lne) / 49.0;
        const double c8 = -(1.0 - 8.0 * lne) / 64.0;
        return c0 + eps * (c1 + eps * (c2 + eps * (c3 + eps * (c4 + eps * (c5 + eps * (c6 + eps * (c7 + eps * c8)))))));
    } else if (x == 1.0) {
        return M_PI * M_PI / 6.0;
    } else if (x > 0.5) {
        const double ser = dilog_series_2(1.0 - x);
        const double log_x = ora_log(x);
        const double t1 = M_PI * M_PI / 6.0;
        const double t2 = ser;
        const double t3 = log_x * ora_log(1.0 - x);
        return t1 - t2 - t3;
    } else if (x > 0.25) {
        return dilog_series_2(x);
    } else if (x > 0.0) {
        return dilog_series_1(x);
    }
    return 0.0;   /* x == 0.0 */
}

/* gsl_sf_dilog_e */
double ora_gsl_dilog(const double x)
{
    if (x >= 0.0) return dilog_xge0(x);
    const double d1 = dilog_xge0(-x);
    const double d2 = dilog_xge0(x * x);
    return -d1 + 0.5 * d2;
}

/* ------------------------------------------------------------- Clausen -- */
/* gsl_sf_angle_restrict_pos_e (trig.c): theta -> [0, 2 pi) with the synthetic extended-precision 2 pi */
static double angle_restrict_pos(const double theta)
{
    const double P1 = 4 * 7.85398125648498535156e-01;
    const double P2 = 4 * 3.77489470793079817668e-08;
    const double P3 = 4 * 2.69515142907905952645e-15;
    const double TwoPi = 2 * (P1 + P2 + P3);
    const double y = 2 * floor(theta / TwoPi);
    double r = ((theta - y * P1) - y * P2) - y * P3;
    if (r > TwoPi) r = (((r - 2 * P1) - 2 * P2) - 2 * P3);
    else if (r < 0) r = (((r + 2 * P1) + 2 * P2) + 2 * P3);
    return r;
}

/* aclaus_cs (clausen.c): Chebyshev series of Cl2(x)/x + log(x) in t = 2 (x^2/pi^2 - 1/2) on [-1, 1] */
static const double aclaus_data[15] = {
    2.142694363766688447e+00, 0.723324281221257925e-01, 0.101642475021151164e-02, 0.3245250328531645e-04,
    0.133315187571472e-05,    0.6213240591653e-07,      0.313004135337e-08,       0.16635723056e-09,
    0.919659293e-11,          0.52400462e-12,           0.3058040e-13,            0.18197e-14,
    0.1100e-15,               0.68e-17,                 0.4e-18};

/* cheb_eval_e (cheb_eval.c), order 14 on [a, b] = [-1, 1] */
static double cheb_eval_aclaus(const double x)
{
    const double a = -1.0, b = 1.0;
    double d = 0.0;
    double dd = 0.0;
    const double y = (2.0 * x - a - b) / (b - a);
    const double y2 = 2.0 * y;
    for (int j = 14; j >= 1; j--) {
        const double temp = d;
        d = y2 * d - dd + aclaus_data[j];
        dd = temp;
    }
    d = y * d - dd + 0.5 * aclaus_data[0];
    return d;
}

/* gsl_sf_clausen_e: Cl2(x) */
double ora_gsl_clausen(double x)
{
    const double x_cut = M_PI * GSL_SQRT_DBL_EPSILON;
    double sgn = 1.0;
    double val;
    if (x < 0.0) {
        x = -x;
        sgn = -1.0;
    }
    x = angle_restrict_pos(x);
    if (x > M_PI) {
        /* simulated extra precision: 2PI = p0 + p1 */
        const double p0 = 6.28125;
        const double p1 = 0.19353071795864769253e-02;
        x = (p0 - x) + p1;
        sgn = -sgn;
    }
    if (x == 0.0) val = 0.0;
    else if (x < x_cut) val = x * (1.0 - ora_log(x));
    else {
        const double t = 2.0 * (x * x / (M_PI * M_PI) - 0.5);
        const double c = cheb_eval_aclaus(t);
        val = x * (c - ora_log(x));
    }
    return val * sgn;
}

/* ------------------------------------------------------------- complex -- */
/* dilogc_series_1: sum r^k e^(i k theta) / k^2, small r */
static void dilogc_series_1(const double r, const double x, const double y, double *re, double *im)
{
    const double cos_theta = x / r;
    const double sin_theta = y / r;
    const double alpha = 1.0 - cos_theta;
    const double beta = sin_theta;
    double ck = cos_theta;
    double sk = sin_theta;
    double rk = r;
    double real_sum = r * ck;
    double imag_sum = r * sk;
    const int kmax = 50 + (int)(22.0 / (-ora_log(r)));
    int k;
    for (k = 2; k < kmax; k++) {
        double dr, di;
        const double ck_tmp = ck;
        ck = ck - (alpha * ck + beta * sk);
        sk = sk - (alpha * sk - beta * ck_tmp);
        rk *= r;
        dr = rk / ((double)k * k) * ck;
        di = rk / ((double)k * k) * sk;
        real_sum += dr;
        imag_sum += di;
        if (fabs((dr * dr + di * di) / (real_sum * real_sum + imag_sum * imag_sum)) < GSL_DBL_EPSILON * GSL_DBL_EPSILON) break;
    }
    g_stat[2] += k;
    *re = real_sum;
    *im = imag_sum;
}

/* series_2_c: sum z^k / (k^2 (k + 1)) */
static void series_2_c(double r, double x, double y, double *sum_re, double *sum_im)
{
    const double cos_theta = x / r;
    const double sin_theta = y / r;
    const double alpha = 1.0 - cos_theta;
    const double beta = sin_theta;
    double ck = cos_theta;
    double sk = sin_theta;
    double rk = r;
    double real_sum = 0.5 * r * ck;
    double imag_sum = 0.5 * r * sk;
    const int kmax = 30 + (int)(18.0 / (-ora_log(r)));
    int k;
    for (k = 2; k < kmax; k++) {
        double dr, di;
        const double ck_tmp = ck;
        ck = ck - (alpha * ck + beta * sk);
        sk = sk - (alpha * sk - beta * ck_tmp);
        rk *= r;
        dr = rk / ((double)k * k * (k + 1.0)) * ck;
        di = rk / ((double)k * k * (k + 1.0)) * sk;
        real_sum += dr;
        imag_sum += di;
        if (fabs((dr * dr + di * di) / (real_sum * real_sum + imag_sum * imag_sum)) < GSL_DBL_EPSILON * GSL_DBL_EPSILON) break;
    }
    g_stat[3] += k;
    *sum_re = real_sum;
    *sum_im = imag_sum;
}

/* gsl_sf_complex_log_e (log.c): log|z| = log(max) + log(1 + (min/max)^2)/2, arg z = atan2 */
static void complex_log(const double zr, const double zi, double *lnr, double *theta)
{
    const double ax = fabs(zr);
    const double ay = fabs(zi);
    const double min = ax < ay ? ax : ay;
    const double max = ax > ay ? ax : ay;
    *lnr = ora_log(max) + 0.5 * ora_log(1.0 + (min / max) * (min / max));
    *theta = ora_atan2(zi, zr);
}

/* dilogc_series_2: Li2(z) = 1 + (1 - z) log(1 - z) / z + series_2_c(z), r < 1 */
static void dilogc_series_2(const double r, const double x, const double y, double *re, double *im)
{
    if (r == 0.0) {
        *re = 0.0;
        *im = 0.0;
        return;
    }
    double sum_re, sum_im, ln_omz_r, ln_omz_theta;
    series_2_c(r, x, y, &sum_re, &sum_im);
    complex_log(1.0 - x, -y, &ln_omz_r, &ln_omz_theta);   /* t = ln(1-z)/z */
    const double t_x = (ln_omz_r * x + ln_omz_theta * y) / (r * r);
    const double t_y = (-ln_omz_r * y + ln_omz_theta * x) / (r * r);
    const double r_x = (1.0 - x) * t_x + y * t_y;   /* (1-z) ln(1-z)/z */
    const double r_y = (1.0 - x) * t_y - y * t_x;
    *re = sum_re + r_x + 1.0;
    *im = sum_im + r_y;
}

/* dilogc_series_3: |z| near 1, Li2(z) = sum_n a^n / n! H_n(theta), a = log r (n <= 6) */
static void dilogc_series_3(const double r, const double x, const double y, double *re, double *im)
{
    const double theta = ora_atan2(y, x);
    const double cos_theta = x / r;
    const double sin_theta = y / r;
    const double a = ora_log(r);
    const double omc = 1.0 - cos_theta;
    const double omc2 = omc * omc;
    double H_re[7];
    double H_im[7];
    double an, nfact;
    double sum_re, sum_im;
    int n;

    H_re[0] = M_PI * M_PI / 6.0 + 0.25 * (theta * theta - 2.0 * M_PI * fabs(theta));
    H_im[0] = ora_gsl_clausen(theta);
    H_re[1] = -0.5 * ora_log(2.0 * omc);
    H_im[1] = -ora_atan2(-sin_theta, omc);
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

    sum_re = H_re[0];
    sum_im = H_im[0];
    an = 1.0;
    nfact = 1.0;
    for (n = 1; n <= 6; n++) {
        double t;
        an *= a;
        nfact *= n;
        t = an / nfact;
        sum_re += t * H_re[n];
        sum_im += t * H_im[n];
    }
    g_stat[4] += 1;
    *re = sum_re;
    *im = sum_im;
}

/* dilogc_fundamental: the unit disk with x < 0.732 */
static void dilogc_fundamental(double r, double x, double y, double *re, double *im)
{
    if (r > 0.98) dilogc_series_3(r, x, y, re, im);
    else if (r > 0.25) {
        double sr, si;
        dilogc_series_2(r, x, y, &sr, &si);
        *re = sr;
        *im = si;
    } else dilogc_series_1(r, x, y, re, im);
}

/* dilogc_unitdisk: |z| < 1; x > 0.732 is reflected, Li2(z) = -Li2(1-z) + zeta2 - log(z) log(1-z) */
static void dilogc_unitdisk(double x, double y, double *re, double *im)
{
    static const double MAGIC_SPLIT_VALUE = 0.732;
    static const double zeta2 = M_PI * M_PI / 6.0;
    const double r = ora_hypot(x, y);
    if (x > MAGIC_SPLIT_VALUE) {
        const double x_tmp = 1.0 - x;
        const double y_tmp = -y;
        const double r_tmp = ora_hypot(x_tmp, y_tmp);
        double re_tmp, im_tmp;
        dilogc_fundamental(r_tmp, x_tmp, y_tmp, &re_tmp, &im_tmp);
        const double lnz = ora_log(r);                 /* log(|z|)   */
        const double lnomz = ora_log(r_tmp);           /* log(|1-z|) */
        const double argz = ora_atan2(y, x);           /* arg(z)     */
        const double argomz = ora_atan2(y_tmp, x_tmp); /* arg(1-z)   */
        *re = -re_tmp + zeta2 - lnz * lnomz + argz * argomz;
        *im = -im_tmp - argz * lnomz - argomz * lnz;
    } else
        dilogc_fundamental(r, x, y, re, im);
}

/* gsl_sf_complex_dilog_xy_e */
void ora_gsl_complex_dilog_xy(const double x, const double y, double *re, double *im)
{
    const double zeta2 = M_PI * M_PI / 6.0;
    const double r2 = x * x + y * y;
    if (y == 0.0) {
        *im = (x >= 1.0) ? -M_PI * ora_log(x) : 0.0;
        *re = ora_gsl_dilog(x);
    } else if (fabs(r2 - 1.0) < GSL_DBL_EPSILON) {
        /* Lewin A.2.4.1 and A.2.4.2 */
        const double theta = ora_atan2(y, x);
        const double term1 = theta * theta / 4.0;
        const double term2 = M_PI * fabs(theta) / 2.0;
        *re = zeta2 + term1 - term2;
        *im = ora_gsl_clausen(theta);
    } else if (r2 < 1.0) {
        dilogc_unitdisk(x, y, re, im);
    } else {
        /* reduce the argument to the unit disk, then unwind Li2(z) + Li2(1/z) = -zeta2 - log(-z)^2 / 2 */
        const double r = sqrt(r2);
        const double x_tmp = x / r2;
        const double y_tmp = -y / r2;
        double re_tmp, im_tmp;
        dilogc_unitdisk(x_tmp, y_tmp, &re_tmp, &im_tmp);
        const double theta = ora_atan2(y, x);
        const double theta_abs = fabs(theta);
        const double theta_sgn = (theta < 0.0 ? -1.0 : 1.0);
        const double ln_minusz_re = ora_log(r);
        const double ln_minusz_im = theta_sgn * (theta_abs - M_PI);
        const double lmz2_re = ln_minusz_re * ln_minusz_re - ln_minusz_im * ln_minusz_im;
        const double lmz2_im = 2.0 * ln_minusz_re * ln_minusz_im;
        *re = -re_tmp - 0.5 * lmz2_re - zeta2;
        *im = -im_tmp - 0.5 * lmz2_im;
    }
}
