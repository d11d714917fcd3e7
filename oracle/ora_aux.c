/*
 * nuSIprop oracle -- restatement of aux.hpp.  TEST INFRASTRUCTURE ONLY.
 * Every function keeps the reference's branch thresholds and Taylor
 * coefficients; GSL calls go to ora_specfun.c.
 */
#define _GNU_SOURCE
#include <math.h>
#include "ora_aux.h"
#include "ora_libm.h"
#include "ora_specfun.h"

#define SQ(a) ((a) * (a))
#define CU(a) ((a) * (a) * (a))

/* aux.hpp:53-54 -- 3-point Gauss-Legendre */
const double ora_gl_w[3] = {5. / 9., 8. / 9., 5. / 9.};
const double ora_gl_x[3] = {-0.7745966692414834, 0.0, 0.7745966692414834}; /* = sqrt(3./5.) exactly */

/* aux.hpp:63-75 */
double ora_atandiff(double x, double y)
{
    if (fabs(x) < 1e2 || fabs(y) < 1e2 || x * y < 0) return ora_atan(x) - ora_atan(y);
    const double ix = 1. / x, iy = 1. / y;
    return -ix + CU(ix) / 3. - (-iy + CU(iy) / 3.);
}

static zc cli2(zc z)
{
    double re, im;
    ora_complex_dilog_xy(z.r, z.i, &re, &im);
    return zmk(re, im);
}

/* asymptotic Li2 for |z| >> 1 used by aux.hpp:84-89:
 *   -1/(16 z^4) - 1/(9 z^3) - 1/(4 z^2) - 1/z - (I/2)(-s 2 pi log z - I log^2 z) */
static zc li2_asym(zc z)
{
    const double s = (z.i >= 0) ? 1.0 : -1.0;
    const zc L = zlog(z);
    const zc z2 = zmul(z, z);
    const zc t = zsub(zscale(-s * 2 * M_PI, L), zmul(zmk(0.0, 1.0), zmul(L, L)));
    zc r = zrdiv(-1, zscale(16., zmul(z2, z2)));
    r = zsub(r, zrdiv(1, zscale(9., zmul(zmul(z, z), z))));
    r = zsub(r, zrdiv(1, zscale(4., z2)));
    r = zsub(r, zrdiv(1, z));
    return zsub(r, zmul(zmk(0.0, 0.5), t));
}

/* aux.hpp:77-96 */
zc ora_dilogdiff_c(zc x, zc y)
{
    if (zabs(x) > 1e2 && zabs(y) > 1e2) return zsub(li2_asym(x), li2_asym(y));
    const zc a = cli2(x), b = cli2(y);
    return zmk(a.r - b.r, a.i - b.i);
}

/* aux.hpp:98-113 : Li2(-x) - Li2(-y) */
double ora_dilogdiff(double x, double y)
{
    if (x > 1e2 && y > 1e2) {
        const double lx = ora_log(x), ly = ora_log(y), ix = 1. / x, iy = 1. / y;
        return -SQ(lx) / 2. + ix - SQ(ix) / 4. + CU(ix) / 9. - SQ(SQ(ix)) / 16
               - (-SQ(ly) / 2. + iy - SQ(iy) / 4. + CU(iy) / 9. - SQ(SQ(iy)) / 16);
    }
    if (x < 1e-2 && y < 1e-2)
        return -x + SQ(x) / 4. - CU(x) / 9. + SQ(SQ(x)) / 16.
               - (-y + SQ(y) / 4. - CU(y) / 9. + SQ(SQ(y)) / 16.);
    return ora_dilog(-x) - ora_dilog(-y);
}

/* aux.hpp:115-130 : Li2(-1-x) - Li2(-1-y) */
static double d1m_big(double v)
{
    const double l = ora_log(v);
    return -SQ(l) / 2. + (1 - l) / v + (-7 + 2 * l) / (4. * SQ(v)) + (19 - 3 * l) / (9. * CU(v))
           + (-125 + 12 * l) / (48. * SQ(SQ(v)));
}
static double d1m_small(double v)
{
    return -v * 0.6931471805599453 + (SQ(v) * (-1 + 1.3862943611198906)) / 4. + (CU(v) * (5 - 8 * 0.6931471805599453)) / 24.
           + SQ(SQ(v)) * (-1. / 6. + 0.6931471805599453 / 4.);
}
double ora_dilog1mdiff(double x, double y)
{
    if (x > 1e2 && y > 1e2) return d1m_big(x) - d1m_big(y);
    if (x < 1e-2 && y < 1e-2) return d1m_small(x) - d1m_small(y);
    return ora_dilog(-1 - x) - ora_dilog(-1 - y);
}

/* aux.hpp:132-148 : Li2(1+x) - Li2(1+y), x,y < 0 */
static double d1p_big(double v)
{
    const double l = ora_log(-v);
    return (-1 - 3 * l) / (9. * CU(v)) + (-1 - l) / v - SQ(l) / 2. + (1 + 2 * l) / (4. * SQ(v))
           + (1 + 4 * l) / (16. * SQ(SQ(v)));
}
static double d1p_small(double v)
{
    const double l = ora_log(-v);
    return v * (1 - l) + (SQ(v) * (-1 + 2 * l)) / 4. + (CU(v) * (1 - 3 * l)) / 9.
           + (SQ(SQ(v)) * (-1 + 4 * l)) / 16.;
}
double ora_dilog1pdiff(double x, double y)
{
    if (-x > 1e2 && -y > 1e2) return d1p_big(x) - d1p_big(y);
    if (-x < 1e-2 && -y < 1e-2) return d1p_small(x) - d1p_small(y);
    return ora_dilog(1 + x) - ora_dilog(1 + y);
}

/* aux.hpp:150-166 : Li2(1/(1-x)) - Li2(1/(1-y)), x,y < 0 */
static double d1o_big(double v)
{
    return -25 / (48. * SQ(SQ(v))) - 11 / (18. * CU(v)) - 3 / (4. * SQ(v)) - 1 / v;
}
static double d1o_small(double v)
{
    const double l = ora_log(-v);
    return (SQ(SQ(v)) * (-19 - 12 * l)) / 48. + (CU(v) * (-7 - 6 * l)) / 18.
           + (SQ(v) * (-1 - 2 * l)) / 4. + v * (1 - l);
}
double ora_dilog1over1mdiff(double x, double y)
{
    if (-x > 1e2 && -y > 1e2) return d1o_big(x) - d1o_big(y);
    if (-x < 1e-2 && -y < 1e-2) return d1o_small(x) - d1o_small(y);
    return ora_dilog(1 / (1 - x)) - ora_dilog(1 / (1 - y));
}

/*
 * aux.hpp:12-50 -- lightest neutrino mass from the mass sum.
 * The reference squares  mSum = m + sqrt(m^2+a) + sqrt(m^2+b)  twice into a
 * quartic, solves it with gsl_poly_complex_solve and returns the first root
 * that is real, >= 0 and passes the two "un-squaring" constraints
 * (aux.hpp:38-46).  Those constraints select exactly the roots of the
 * un-squared equation, which is strictly increasing in m, so the selected
 * root is unique: we find it by bisection of the un-squared equation to full
 * precision (GSL's QR root carries ~1e-14 relative noise instead).
 * Degenerate edge: at the minimal mass sum (test.py) the root is m = 0, where
 * GSL returns rounding noise and m = 0 exactly would make the tables NaN
 * (nuSIprop.hpp:791, m^2/(2*0)*0); we return ORA_ML_FLOOR = 1e-12 eV there.
 * Returns 0, or -2 when no spectrum exists (the reference prints and exits).
 */
#define ORA_ML_FLOOR 1e-12
static double mass_sum(double m, double dmqSL, double dmqAT)
{
    if (dmqAT > 0) return m + sqrt(SQ(m) + dmqSL) + sqrt(SQ(m) + dmqAT);
    const double m2 = sqrt(SQ(m) - dmqAT);
    return m + m2 + sqrt(SQ(m2) - dmqSL);
}
int ora_getmL(double mSum, double dmqSL, double dmqAT, double *mL)
{
    const double f0 = mass_sum(0.0, dmqSL, dmqAT) - mSum;
    double ml;
    if (f0 >= 0) {
        if (f0 > 64 * 2.220446049250313e-16 * mSum) return -2;
        ml = ORA_ML_FLOOR;
    } else {
        double lo = 0.0, hi = mSum;
        for (int it = 0; it < 2000; ++it) {
            const double mid = 0.5 * (lo + hi);
            if (mid <= lo || mid >= hi) break;
            if (mass_sum(mid, dmqSL, dmqAT) - mSum > 0) hi = mid; else lo = mid;
        }
        ml = (fabs(mass_sum(hi, dmqSL, dmqAT) - mSum) < fabs(mass_sum(lo, dmqSL, dmqAT) - mSum)) ? hi : lo;
        if (ml <= 0) ml = ORA_ML_FLOOR;
    }
    const int ok1 = (mSum - ml > 1.0e-7);
    const int ok2 = (dmqAT > 0) ? (SQ(mSum) - dmqAT - dmqSL - SQ(ml) - 2 * ml * mSum > 1.0e-7)
                                : (SQ(mSum) + 2 * dmqAT + dmqSL - SQ(ml) - 2 * ml * mSum > 1.0e-7);
    if (!(ok1 && ok2)) return -2;
    *mL = ml;
    return 0;
}
