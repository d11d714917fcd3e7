/*
 * nuSIprop CPU oracle -- TEST INFRASTRUCTURE ONLY (see nusi_oracle.h).
 *
 * Restates nuSIprop::calculate_flux (nuSIprop.hpp) in plain C99: same
 * formulas, same branch thresholds (Taylor switches, "x<0" quadrature
 * fallbacks, |t+1|<1e-7 nudges), same loop orders and the same quirks
 * (shadowed alpha_tu fallback, zmax overwrite, stale norm_total in the
 * energy check).  Sub-expressions that the reference repeats verbatim are
 * hoisted into locals; additions keep the reference's left-to-right order.
 * The functions feeding the tables (log/log1p/exp/atan/atan2/atanh, Li2,
 * Li3) and the complex arithmetic (ora_cplx.h) use a fixed operation
 * sequence shared with the GPU (ora_libm.c): the reference's closed forms
 * cancel catastrophically at small |t|, s', so bit-exact table parity needs
 * identical arithmetic.  Host-level set-up (grid, cosmology, normalisation)
 * uses glibc, as the product's host code does.
 */
#define _GNU_SOURCE
#include <complex.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nusi_oracle.h"
#include "ora_aux.h"
#include "ora_specfun.h"
#include "ora_spline.h"
#include "ora_libm.h"
#include "ora_cplx.h"

#define SQ(a) ((a) * (a))
#define CU(a) ((a) * (a) * (a))
#define CH(S, bit) ((S)->chan & (bit))

struct ora_state {
    ora_params p;
    int N, Nz, T;
    double *Emin, *Emax, *Enu, *z;
    double zmax_eff;                    /* member zmax after the overwrite, nuSIprop.hpp:128 */
    double U2m[3][3];                   /* |U_fk|^2 (only the moduli are used) */
    double mn[3];
    double norm_total;
    int have_pp;
    ora_spline spl_at, spl_a;
    int err;
    int warn;
    int chan;                           /* ORA_CH_* mask of the channels summed (test hook; all by default) */
};

static const double E0 = 1e14;          /* nuSIprop.hpp:549 */
static const int N_INTEG_Z = 100;       /* nuSIprop.hpp:550 */

/* ----------------------------------------------------------------------------
 * cosmology and source  (nuSIprop.hpp:573-662)
 * ------------------------------------------------------------------------- */
static double nd_of(double z) { return 4.3528e-13 * CU(1 + z); }
static double H_of(double z) { return 1.5e-33 * pow(0.692 + 0.308 * CU(1 + z), 0.5); }
static double sfr_of(double z)
{
    return pow(pow(1 + z, -3.4 * 10) + pow((1 + z) / 5161, 0.3 * 10) + pow((1 + z) / 9.06, 3.5 * 10), -1. / 10.);
}
static double rsn_of(double z)
{
    const double msun = 1.989 * 56.1;
    return sfr_of(z) * 0.01 / msun;
}
/* Fermi-Dirac (T = 6 MeV) antiderivative, nuSIprop.hpp:638-646 */
static double lum_int(double z, double E)
{
    const double Etot = 3 * 6.24, T = 6e6;
    const double y = -E * (1 + z) / T;
    const double ey = ora_exp(y);
    const double pref = (Etot * 120 / (6 * 7 * pow(M_PI, 4) * pow(T, 2)));   /* host libm constant */
    return pref * (-E * E * (1 + z) * ora_log(ey + 1) / T + 2 * E * ora_li2(-ey) + 2 * T * ora_li3(-ey) / (1 + z));
}
double ora_Lum(const ora_state *S, double z, double Em, double Ep)
{
    if (S->p.source == 1) {   /* power law, nuSIprop.hpp:656 */
        const double si = S->p.si;
        return S->norm_total / 3.0 * sfr_of(z) * (Ep * ora_pow(Ep / E0 * (1 + z), -si) - Em * ora_pow(Em / E0 * (1 + z), -si)) / (1 - si);
    }
    return (lum_int(z, Ep) - lum_int(z, Em)) * rsn_of(z);   /* DSNB, nuSIprop.hpp:659-662 */
}

/* nuSIprop.hpp:666-692 */
static double flux_FS_E0(const ora_state *S)
{
    double res = 0;
    const double z_min = 0, z_max = S->zmax_eff, si = S->p.si;
    for (int f = 0; f < N_INTEG_Z; f++) {
        const double a = z_min + f * (z_max - z_min) / N_INTEG_Z;
        const double b = z_min + (f + 1.0) * (z_max - z_min) / N_INTEG_Z;
        double zz[3];
        for (int q = 0; q < 3; ++q) zz[q] = (b - a) / 2. * ora_gl_x[q] + (b + a) / 2.;
        res += (b - a) / 2. * (ora_gl_w[0] * pow(1 + zz[0], -si) * sfr_of(zz[0]) / H_of(zz[0])
                               + ora_gl_w[1] * pow(1 + zz[1], -si) * sfr_of(zz[1]) / H_of(zz[1])
                               + ora_gl_w[2] * pow(1 + zz[2], -si) * sfr_of(zz[2]) / H_of(zz[2]));
    }
    return res;
}

/* nuSIprop.hpp:731-744 (power law, used by the energy check only) */
static double lum_times_E(const ora_state *S, double z, double Em, double Ep)
{
    const double si = S->p.si;
    if (fabs(si - 2) < 1e-5)
        return S->norm_total * sfr_of(z) * pow(E0 / (1 + z), si) * (log(Ep / Em) + (2 - si) / 2.0 * (SQ(log(Ep)) - SQ(log(Em))));
    return S->norm_total * sfr_of(z) * pow(E0 / (1 + z), si) * (pow(Ep, 2 - si) - pow(Em, 2 - si)) / (2 - si);
}
/* nuSIprop.hpp:694-729 */
static double energy_FS(const ora_state *S)
{
    double res = 0;
    const double z_min = 0, z_max = S->zmax_eff;
    const double lo = pow(10, S->p.lEmin), hi = pow(10, S->p.lEmax);
    for (int f = 0; f < N_INTEG_Z; f++) {
        const double a = z_min + f * (z_max - z_min) / N_INTEG_Z;
        const double b = z_min + (f + 1.0) * (z_max - z_min) / N_INTEG_Z;
        double zz[3];
        for (int q = 0; q < 3; ++q) zz[q] = (b - a) / 2. * ora_gl_x[q] + (b + a) / 2.;
        res += (b - a) / 2. * (ora_gl_w[0] * lum_times_E(S, zz[0], lo, hi) / H_of(zz[0])
                               + ora_gl_w[1] * lum_times_E(S, zz[1], lo, hi) / H_of(zz[1])
                               + ora_gl_w[2] * lum_times_E(S, zz[2], lo, hi) / H_of(zz[2]));
    }
    return res;
}

/* ----------------------------------------------------------------------------
 * interaction integrals  (nuSIprop.hpp:748-1520)
 * ------------------------------------------------------------------------- */
static double width_of(const ora_state *S)   /* nuSIprop.hpp:748-757 */
{
    const double g = S->p.g, mphi = S->p.mphi;
    if (S->p.majorana) return SQ(g) * mphi / (16.0 * M_PI);
    return SQ(g) * mphi / (8.0 * M_PI);
}
static double u2(const ora_state *S, int k) { return S->U2m[S->p.flav][k]; }

/* 3-point Gauss-Legendre over [a,b] of f(z) */
typedef double (*ora_f1)(double);
static double gl3(double a, double b, ora_f1 f)
{
    double z[3];
    for (int q = 0; q < 3; ++q) z[q] = (b - a) / 2. * ora_gl_x[q] + (b + a) / 2.;
    return ora_gl_w[0] * f(z[0]) + ora_gl_w[1] * f(z[1]) + ora_gl_w[2] * f(z[2]);
}
static double f_Gtu_nores(double z) { return (z + 2) / (z * (z + 1)) - 2 / SQ(z) * ora_log1p(z); }          /* :809 */
static double f_Gtu_int(double z) { return 1 / z - 2 * (1 + z) / (SQ(z) * (2 + z)) * ora_log1p(z); }         /* :833 */
static double f_Gpp(double z)                                                                              /* :900 */
{
    const double r = sqrt(z * (z - 4));
    return (SQ(z) - 4 * z + 6) / (SQ(z) * (z - 2)) * ora_log(SQ((r + z - 2) / (r - z + 2))) - 6 * r / SQ(z);
}

/* the double-scalar analytic absorption piece, nuSIprop.hpp:885 (a = max(s-,4)) */
double ora_Gpp_bracket(double a, double b)
{
    const double ra4 = sqrt(-4 + a), ra = sqrt(a), rb4 = sqrt(-4 + b), rb = sqrt(b);
    const double qa = sqrt((-4 + a) * a), qb = sqrt((-4 + b) * b);
    return 12 * sqrt((-4 + a) / a) - 12 * sqrt((-4 + b) / b)
           - 2 * ora_log(SQ(ra4 - ra) / 4.) * ora_log(SQ(-2 + a + qa) / 4.)
           - ((6 + a * ora_log((-2 + a) * a)) * ora_log(SQ(-2 + a + qa) / SQ(2 - a + qa))) / a
           - 24 * (sqrt((-4 + a) / a) - sqrt((-4 + b) / b) - ora_log(ra4 + ra) + ora_log(rb4 + rb))
           + 2 * ora_log(SQ(rb4 - rb) / 4.) * ora_log(SQ(-2 + b + qb) / 4.)
           + ((6 + b * ora_log((-2 + b) * b)) * ora_log(SQ(-2 + b + qb) / SQ(2 - b + qb))) / b
           + 8 * ora_dilogdiff(4 / SQ(ra4 + ra), 4 / SQ(rb4 + rb))
           + 2 * ora_dilogdiff(4 / SQ(-2 + a + qa), 4 / SQ(-2 + b + qb));
}

double ora_Gamma(ora_state *S, double Em, double Ep)       /* nuSIprop.hpp:759-922 */
{
    const double g = S->p.g, mphi = S->p.mphi;
    const double Ga = width_of(S);
    const double g4 = SQ(SQ(g)), m2 = SQ(mphi);
    const double gr = Ga / mphi;
    double tot = 0;
    for (int j = 0; j < 3; ++j) {
        const double mj = S->mn[j], uj = u2(S, j);
        const double sp = 2 * mj * Ep / m2, sm = 2 * mj * Em / m2;
        const double cs = m2 / (m2 + SQ(Ga));
        const double lg = Ga * (ora_log1p(cs * sp * (sp - 2)) - ora_log1p(cs * sm * (sm - 2)));
        double Gs;
        if (sp < 1e-5)
            Gs = g4 / (32 * M_PI * m2 * Ga) *
                 (2 * mphi * ((gr * (1 + SQ(gr) + 2 * sm)) / SQ(1 + SQ(gr)) * (sp - sm) + gr / SQ(1 + SQ(gr)) * SQ(sp - sm)) + lg);
        else
            Gs = g4 / (32 * M_PI * m2 * Ga) * (2 * mphi * ora_atandiff(mphi * (sp - 1) / Ga, mphi * (sm - 1) / Ga) + lg);
        Gs *= uj;
        const double wgt = m2 / (2 * mj);
        if (CH(S, ORA_CH_S)) tot += wgt * Gs;
        if (!S->p.non_resonant) continue;

        const double L1p = ora_log1p(sp), L1m = ora_log1p(sm);
        /* t + u channels */
        double Gtu0 = g4 / (16 * M_PI * m2) * (2 * L1p / sp - 2 * L1m / sm + L1p - L1m);
        if (Gtu0 < 0) Gtu0 = g4 / (16 * M_PI * m2) * (sp - sm) / 2. * gl3(sm, sp, f_Gtu_nores);
        Gtu0 *= 2 * uj;
        if (CH(S, ORA_CH_T)) tot += wgt * Gtu0;

        /* t-u interference */
        double Gint = g4 / (32 * M_PI * m2 * sm * sp) *
                      (sm * L1p * (2 + 2 * sp + sp * ora_log(2 + sp)) - sp * L1m * (2 + 2 * sm + sm * ora_log(2 + sm))
                       + sm * sp * (ora_dilog1mdiff(sp, sm) + ora_dilogdiff(sp, sm)));
        if (Gint < 0) Gint = g4 / (16 * M_PI * m2) * (sp - sm) / 2. * gl3(sm, sp, f_Gtu_int);
        Gint *= S->p.majorana ? uj : 0.5 * uj;
        if (CH(S, ORA_CH_TU)) tot += wgt * Gint;

        /* s-t interference */
        /* z1 = I(1+s)/(2I+gr), z2 = conj(z1)  (nuSIprop.hpp:846-849) */
        const zc den = zmk(gr, 2.0);
        const zc z1p = zdiv(zmk(0.0, 1 + sp), den), z1m = zdiv(zmk(0.0, 1 + sm), den);
        const zc z2p = zconj(z1p), z2m = zconj(z1m);
        zc d1, d2;
        if (sp < 1e-5) {   /* nuSIprop.hpp:855-860 */
            const zc ipg = zmk(gr, 1.0), mipg = zmk(gr, -1.0);   /* I+gr, -I+gr */
            const zc l1 = zlog(zdiv(ipg, den)), l2 = zlog(zdiv(mipg, zmk(gr, -2.0)));
            d1 = zadd(zsub(zadd(zscale(SQ(sm), zsub(zdiv(zmk(-0.0, -0.5), ipg), zdivr(l1, 2.))), zscale(sm, l1)), zscale(sp, l1)),
                      zdivr(zscale(SQ(sp), zadd(zdiv(zmk(0.0, 1.0), ipg), l1)), 2.));
            d2 = zadd(zsub(zadd(zscale(SQ(sm), zsub(zdiv(zmk(0.0, 0.5), mipg), zdivr(l2, 2.))), zscale(sm, l2)), zscale(sp, l2)),
                      zdivr(zscale(SQ(sp), zadd(zdiv(zmk(-0.0, -1.0), mipg), l2)), 2.));
        } else {
            d1 = ora_dilogdiff_c(z1p, z1m);
            d2 = ora_dilogdiff_c(z2p, z2m);
        }
        const double Lgp = ora_log1p(SQ(-1 + sp) / SQ(gr)), Lgm = ora_log1p(SQ(-1 + sm) / SQ(gr));
        double Gst = -g4 / (32 * M_PI * m2 * (1 + SQ(gr))) *
                     (d1.r + d2.r + gr * (d2.i - d1.i) + 2 * gr * zarg(zrsub(1, z2p)) * L1p
                      - 2 * gr * zarg(zrsub(1, z2m)) * L1m +ora_log1p(4 / SQ(gr)) * (L1m - L1p) + Lgp * L1p - Lgm * L1m
                      + (1 + SQ(gr)) * (Lgm - Lgp) + 2 * ora_dilogdiff(sp, sm));
        Gst *= uj;
        if (CH(S, ORA_CH_ST)) tot += wgt * Gst;
        const double Gsu = S->p.majorana ? Gst : 0;
        if (CH(S, ORA_CH_SU)) tot += wgt * Gsu;

        /* double scalar production */
        double Gpp = 0;
        if (sp > 4 && S->p.phiphi) {
            const double a = (sm > 4) ? sm : 4.0;
            Gpp = g4 / (128. * M_PI * m2) * ora_Gpp_bracket(a, sp);
            if (Gpp < 0) {
                const double aa = (sm < 4) ? 4 : sm;
                Gpp = g4 / (64 * M_PI * m2) * (sp - aa) / 2. * gl3(aa, sp, f_Gpp);
            }
            Gpp *= uj;
            if (S->p.majorana) Gpp *= 2;
        }
        if (CH(S, ORA_CH_PP)) tot += wgt * Gpp;

        if (Gs < 0 || Gtu0 < 0 || Gint < 0 || (Gs + Gtu0 + Gst + Gsu) < 0) S->warn |= 1;
    }
    return tot;
}

/* 3x3 Gauss-Legendre over the triangle-ish region y in [tp,tm], x in [-y,-tp] (nuSIprop.hpp:987-1003) */
typedef double (*ora_f2)(double, double);
static double gl33_tri(double tp, double tm, ora_f2 F)
{
    const double ay = tp, by = tm;
    double acc = 0;
    for (int i = 0; i < 3; ++i) {
        const double y = (by - ay) / 2. * ora_gl_x[i] + (by + ay) / 2.;
        const double ax = -y, bx = -tp;
        for (int j = 0; j < 3; ++j) {
            const double x = (bx - ax) / 2. * ora_gl_x[j] + (bx + ax) / 2.;
            acc += 1. / 4. * (by - ay) * (bx - ax) * ora_gl_w[i] * ora_gl_w[j] * F(y, x);
        }
    }
    return acc;
}
/* rectangle y in [tp,tm], x in [Sm,Sp] (nuSIprop.hpp:1288-1301) */
static double gl33_rect(double tp, double tm, double Sm, double Sp, ora_f2 F)
{
    double acc = 0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const double y = (tm - tp) / 2. * ora_gl_x[i] + (tm + tp) / 2.;
            const double x = (Sp - Sm) / 2. * ora_gl_x[j] + (Sp + Sm) / 2.;
            acc += ora_gl_w[i] * ora_gl_w[j] * F(y, x);
        }
    return acc * (1. / 4. * (tm - tp) * (Sp - Sm));
}
static double F_t_maj(double y, double x) { return SQ(y / x) / SQ(y - 1) + SQ((-x - y) / x) / SQ((-x - y) - 1); }
static double F_t_dir(double y, double x) { return SQ(y / x) / SQ(y - 1); }
static double F_tu(double y, double x) { return 2 * y * (-y - x) / SQ(x) / ((y - 1) * (-y - x - 1)); }

static int pp_lookup(ora_state *S, const ora_spline *s, const double *x, double *out)
{
    if (!S->have_pp) { S->err = -3; *out = 0; return -3; }
    const int r = ora_spline_eval(s, x, out);
    if (r) { S->err = r; *out = 0; }
    return r;
}

double ora_alphaTilde(ora_state *S, double Em, double Ep)   /* nuSIprop.hpp:924-1235 */
{
    const double g = S->p.g, mphi = S->p.mphi;
    const double Ga = width_of(S);
    const double g4 = SQ(SQ(g)), m2 = SQ(mphi), m4 = SQ(SQ(mphi));
    const double gr = Ga / mphi;
    const int maj = S->p.majorana;
    double tot = 0;
    for (int k = 0; k < 3; ++k) {
        const double mk = S->mn[k], uk = u2(S, k);
        double tp = -2 * mk * Ep / m2, tm = -2 * mk * Em / m2;
        if (fabs(tm + 1) < 1e-7) tm += tm * 1e-6;
        if (fabs(tp + 1) < 1e-7) tp += tp * 1e-6;
        const double wgt = m4 / (2 * mk);

        /* s channel */
        const double cs = m2 / (m2 + SQ(Ga));
        const double lg = Ga * (ora_log1p(cs * tp * (tp + 2)) - ora_log1p(cs * tm * (tm + 2)));
        double as;
        if (fabs(tp) < 1e-5)
            as = g4 / (16 * M_PI * Ga * m4) *
                 (2 * mphi * (1 + tm) * (-((gr * (1 + SQ(gr) - 2 * tm) * (-tm + tp)) / SQ(1 + SQ(gr))) + (gr * SQ(-tm + tp)) / SQ(1 + SQ(gr))) + lg);
        else
            as = g4 / (16 * M_PI * Ga * m4) * (2 * mphi * (1 + tm) * ora_atandiff(mphi * (1 + tm) / Ga, mphi * (1 + tp) / Ga) + lg);
        as *= uk;
        if (!maj) as /= 2.;
        if (CH(S, ORA_CH_S)) tot += wgt * as;
        if (!S->p.non_resonant) continue;

        const double Lmt = ora_log1p(-tm), Lmp = ora_log1p(-tp), Ld = ora_log1p(tm - tp);
        const double brk = (-2 + tm) * (tm - tp) - (-1 + tm) * (-2 + tp) * (Lmt - Lmp);
        /* t channel */
        double at;
        if (maj) {
            at = g4 * (1 / (16 * m4 * M_PI * (-1 + tm) * tp) * brk
                       + 1 / (16 * m4 * M_PI * SQ(1 + tm) * tp) *
                             ((1 + tm) * (2 + tm) * (tm - tp) + (-2 * SQ(1 + tm) + tp + 2 * tm * tp) * Ld - SQ(tm) * tp * ora_log(tm / tp)));
            if (at < 0) at = gl33_tri(tp, tm, F_t_maj) * (g4 / (16 * M_PI * m4));
        } else {
            at = 3. / 2. * g4 / (32 * m4 * M_PI * (-1 + tm) * tp) * brk;
            if (at < 0) at = gl33_tri(tp, tm, F_t_dir) * (3. / 2. * g4 / (32 * M_PI * m4));
        }
        at *= uk;
        if (CH(S, ORA_CH_T)) tot += wgt * at;

        /* u channel */
        double au;
        if (maj) au = at;
        else {
            au = 1. / 2. * g4 / (32 * m4 * M_PI * (-1 + tm) * tp) * brk;
            if (au < 0) au = gl33_tri(tp, tm, F_t_dir) * (1. / 2. * g4 / (32 * M_PI * m4));
            au *= uk;
        }
        if (CH(S, ORA_CH_U)) tot += wgt * au;

        /* t-u interference */
        double atu;
        if (maj) {
            double combi;
            if (-tp < 1e-2 && -tm < 1e-2) {
                const double d = tp / tm, lt = ora_log(-tp);
                combi = -(((-1 + d) * tp * ora_log(-2 * tp)) / d)
                        - ((-1 + d) * SQ(tp) * (-2 + d + d * 0.6931471805599453 + ora_log(-2 / tp) - d * lt)) / (2. * SQ(d))
                        + (CU(tp) * (8 - 30 * d + 21 * SQ(d) + CU(d) - 8 * CU(d) * 0.6931471805599453 + 5.545177444479562 + 8 * lt - 8 * CU(d) * lt)) / (24. * CU(d))
                        + (SQ(SQ(tp)) * (-32 + 56 * d - 51 * SQ(d) + 30 * CU(d) - 3 * SQ(SQ(d)) + 8.317766166719343 - SQ(SQ(d)) * 8.317766166719343
                                         - 12 * lt + 12 * SQ(SQ(d)) * lt)) / (48. * SQ(SQ(d)));
            } else if (-tp > 1e2 && -tm > 1e2) {
                const double d = tp / tm, lq = ora_log((-1 + d) / d), lt = ora_log(-tp);
                combi = (-2 * (-1 + d) * lq) / tp - (2 * (-1 + ora_log(-(d / ((-1 + d) * tp))))) / SQ(tp)
                        + (-6 + 4 * d + SQ(d) - 2 * CU(d) - 8 * lq + 8 * d * lq + 2 * CU(d) * lq - 2 * SQ(SQ(d)) * lq - 6 * lt + 6 * d * lt) / (3. * (-1 + d) * CU(tp))
                        + (8 - 12 * d + 3 * SQ(d) + 12 * lq - 24 * d * lq + 12 * SQ(d) * lq + 12 * lt - 24 * d * lt + 12 * SQ(d) * lt) / (3. * SQ(-1 + d) * SQ(SQ(tp)));
            } else
                combi = ora_dilog(1 + 1 / (-2 + tp)) - ora_dilog((-1 + tm) / (-2 + tp)) + ora_dilog(1 + (1 + tm - tp) / tp) - ora_dilog(1 + 1 / tp);

            atu = g4 / (32 * M_PI * m4 * (1 + tm) * tp) *
                  (2 * (2 * (1 + tm) * (tm - tp) - 2 * (1 + tm) * tp * ora_atanh(1 / (1 - tp)) * ora_atanh((tm - tp) / (-2 + tm + tp))
                        + tm * tp * (-Lmt + Lmp) + (1 + tm) * (Lmt - Lmp - Ld) + tp * (-Lmt + Lmp + Ld) - tm * tp * ora_log(tm / tp))
                   + (1 + tm) * tp * ((-SQ(Lmt) + SQ(Lmp)) / 2. + ora_dilog1over1mdiff(tp, tm))
                   - (1 + tm) * tp * (ora_dilog1pdiff(tm, tp) + combi));
            if (atu < 0) atu = gl33_tri(tp, tm, F_tu) * (g4 / (16 * M_PI * m4));
        } else
            atu = 0;
        atu *= uk;
        if (CH(S, ORA_CH_TU)) tot += wgt * atu;

        /* s-t interference */
        /* nuSIprop.hpp:1137-1144 */
        const zc den = zmk(gr, 2.0);          /* 2I + gr   */
        const zc ipg = zmk(gr, 1.0);          /* I + gr    */
        const zc dtm = zmk(2 + tm, -gr);      /* 2 - I gr + tm */
        zc d78, d51, d26, d43;
        if (-tp < 1e-5) {   /* nuSIprop.hpp:1151-1167 */
            const double d = tp / tm;
            const zc ltm = zlog(zre(tm)), ltp = zlog(zre(tp)), ld = zlog(zre(d));
            const zc lq = zlog(zrsub(1.0, zdiv(zmk(0.0, 1.0), den))), lr = zlog(zdiv(ipg, den));
            d78 = zsub(zadd(zscale(tm, zaddr(ltm, -1.0)), zdivr(zscale(SQ(tm), zaddr(zscale(2, ltm), -1.0)), 4.)),
                       zadd(zscale(tp, zaddr(ltp, -1.0)), zdivr(zscale(SQ(tp), zaddr(zscale(2, ltp), -1.0)), 4.)));
            d51 = zadd(zscale(-tm + tp, lq),
                       zdiv(zscale(-SQ(tm) + SQ(tp), zadd(zmul(zmk(0.0, 1.0), zaddr(lq, 1.0)), zscale(gr, lq))), zscale(2., ipg)));
            {
                const zc a1 = zsub(zadd(zrsub(-1.0 + d, ld), ltp), zscale(d, ltp));
                zc b2 = zaddr(zscale(2, ld), -1.0 + SQ(d));          /* -1 + d^2 + 2 ld */
                b2 = zsub(b2, zscale(2, ltp));
                b2 = zadd(b2, zscale(4 * d, ltp));
                b2 = zsub(b2, zscale(2 * SQ(d), ltp));
                zc b3 = zrsub(7 - 9 * d + 2 * CU(d), zscale(6, ld));  /* 7 - 9d + 2d^3 - 6 ld */
                b3 = zadd(b3, zscale(6, ltp));
                b3 = zsub(b3, zscale(18 * d, ltp));
                b3 = zadd(b3, zscale(18 * SQ(d), ltp));
                b3 = zsub(b3, zscale(6 * CU(d), ltp));
                d26 = zadd(zadd(zdivr(zscale(tp, a1), d), zdivr(zscale(SQ(tp), b2), 4. * SQ(d))),
                           zdivr(zscale(CU(tp), b3), 18. * CU(d)));
            }
            d43 = zadd(zdivr(zscale((-1 + d) * tp, lr), d),
                       zdivr(zscale((-1 + d) * SQ(tp),
                                    zadd(zmul(zmk(0.0, 1.0), zsub(zrdiv(1 + d, ipg), zrdiv(2, den))), zscale(-1 + d, lr))),
                             2. * SQ(d)));
        } else {
            const zc z1 = zdiv(zmk(0.0, 1 - tm), den);     /* (-I(-1+tm))/(2I+gr) */
            const double z2 = 1 / (1 + tm);
            const zc z3 = zrdiv(1, dtm);
            const zc z4 = zrdiv(1 + tm - tp, dtm);
            const zc z5 = zdiv(zmk(0.0, 1 - tp), den);
            const double z6 = 1 - tp / (1 + tm);
            d78 = ora_dilogdiff_c(zre(1 - tm), zre(1 - tp));
            d51 = ora_dilogdiff_c(z5, z1);
            d26 = ora_dilogdiff_c(zre(z2), zre(z6));
            d43 = ora_dilogdiff_c(z4, z3);
        }
        const double Lgp = ora_log1p(SQ(1 + tp) / SQ(gr)), Lgm = ora_log1p(SQ(1 + tm) / SQ(gr));
        const double Am = zarg(zmk(-1 - tm, gr)), Ap = zarg(zmk(-1 - tp, gr));          /* carg(-1 + I gr - t) */
        const double Bm = zarg(zdiv(zmk(gr, 1 + tm), den)), Bp = zarg(zdiv(zmk(gr, 1 + tp), den));
        double ast;
        if (maj)
            ast = g4 / (32 * M_PI * (1 + SQ(gr)) * m4) *
                  (2 * M_PI * Am - 2 * M_PI * Ap + 2 * gr * (d51.i + d26.i + d43.i)
                   - 2 * (d51.r + d26.r + d43.r + d78.r) - Bm * (2 * M_PI + 2 * gr * Lmt)
                   + Bp * (2 * M_PI + 2 * gr * Lmp) + (Am - Ap) * (4 * gr * tm + 2 * gr * Lmt)
                   + 2 * gr * (zarg_real(1 + tm) - zarg(dtm) + zarg(zmk(1 + tp, -gr))) * Ld
                   + ora_log(4 + SQ(gr)) * (Lmp - Lmt) + ora_log(SQ(gr) + SQ(2 + tm)) * Ld - 2 * Lmt * ora_log(-tp)
                   - 2 * gr * M_PI * (ora_log(SQ(tp)) + Ld) + 2 * gr * M_PI * ora_log(SQ(tp)) + 4 * tm * ora_log(tm / tp)
                   + (-Lmp + Lmt - Ld) * (Lgp + 2 * ora_log(gr)) - Ld * ora_log1p(SQ(tm) + 2 * tm)
                   + 2 * (SQ(gr) + tm) * (Lgp - Lgm) + 2 * (ora_log(-tp) * (Lmp + Ld) + (Lgp - Lgm)));
        else
            ast = g4 / (32 * M_PI * (1 + SQ(gr)) * m4) *
                  (gr * d51.i - 2 * (d51.r + d78.r) + 2 * Bm * (-M_PI - gr * Lmt)
                   + 2 * Am * (M_PI + gr * tm + gr * Lmt) - 2 * Ap * (M_PI + gr * tm + gr * Lmt)
                   + 2 * Bp * (M_PI + gr * Lmp) - 2 * Lmt * ora_log(-tp) + 2 * tm * ora_log(tm / tp) + 2 * Lmp * ora_log(-tp)
                   + (Lmp - Lmt) * (ora_log(4 + SQ(gr)) - 2 * ora_log(gr) - Lgp) + (1 + tm + SQ(gr)) * (Lgp - Lgm));
        ast *= uk;
        if (CH(S, ORA_CH_ST)) tot += wgt * ast;
        const double asu = maj ? ast : 0;
        if (CH(S, ORA_CH_SU)) tot += wgt * asu;

        /* double scalar production */
        double app = 0;
        if (-tp > 4 && S->p.phiphi) {
            if (-tp < 1e4) {
                const double xx[2] = {-tp, ora_log10(tp / tm)};
                double v;
                pp_lookup(S, &S->spl_at, xx, &v);
                app = g4 / m4 * v;
            } else
                app = g4 / m4 *
                      (6 * tm * ora_log(-tm) - tp * SQ(ora_log(-tm)) + 2 * (-8 * tm + 8 * tp + 4 * tp * ora_log(-tm) + ora_log(tm - tp) * (tm - tp - tp * ora_log(tm / tp)))
                       - 2 * (2 * tm + 5 * tp) * ora_log(-tp) + tp * SQ(ora_log(-tp)) - 2 * tp * ora_dilog(1 - tm / tp)) / (128. * M_PI * tp);
            app *= uk;
            if (maj) app *= 2;
            app *= 2;
            if (maj) app *= 2;
        }
        if (CH(S, ORA_CH_PP)) tot += wgt * app;

        const double nrm = SQ(SQ(g / mphi));
        if (as < 0 || at < 0 || au < 0 || atu / nrm < -1e-11 || (ast + at + as) / nrm < -1e-11 || (asu + au + as) / nrm < -1e-11)
            S->warn |= 2;
    }
    return tot;
}

static int g_ref_order;
/* The s-t interference's g-dependent pieces (nuSIprop.hpp:1440-1459), dt = 2 + t - i gr, a = 1 + S + t,
 * c = 2 + t:  Li2(w), w = a / dt = a (c + i gr) / (c^2 + gr^2), by the Taylor series about the real point
 * x0 = a / c at d = w - x0 = i (gr / c) w when |d| <= 2.5e-3 min(|x0|, |1 - x0|), else the general complex
 * dilog; and arg(-(-1 + i gr + S) / dt) = arg(S - 1 + i gr) + arg(c + i gr) - pi, each argument written as
 * f pi + s with s the small angle.  The GPU forms them the same way (nusi_physics.hpp alpha_member_*). */
static void member_dc_ref(double S, double t, double gr, double *re, double *im);
static void member_dc(double S, double t, double gr, double *re, double *im)
{
    if (g_ref_order) {
        member_dc_ref(S, t, gr, re, im);
        return;
    }
    const double a = 1 + S + t, c = 2 + t;
    const double x0 = a / c;
    const double ax = fabs(x0), a1 = fabs(1.0 - x0);
    ora_li2t T;
    double m = 0.0;
    if (c != 0.0 && a1 > 0.0 && ax < 1e300) {
        ora_li2_taylor_coeffs(x0, &T);
        m = ORA_LI2T_RATIO * (ax < a1 ? ax : a1);
    }
    const double inv = 1.0 / (c * c + gr * gr), q = gr / c;
    const double wr = (a * c) * inv, wi = (a * gr) * inv;
    const double dr = -(q * wi), di = q * wr;
    if (dr * dr + di * di <= m * m) ora_li2_taylor_eval(&T, dr, di, 1.0, re, im);
    else ora_complex_dilog_xy(wr, wi, re, im);
}
/* Reference-order arithmetic (ora_set_reference_order, test infrastructure): the s-t interference's
 * member dilogs are the general complex dilogarithm of the reference's quotient z = (1+S+t)/(2 - i gr + t)
 * (C99 complex division, nuSIprop.hpp:1432-1438 -> gsl_sf_complex_dilog_xy_e, :1444-1451) and its arguments
 * carg(-((-1 + i gr + S)/(2 - i gr + t))) (:1456), instead of member_dc's Taylor evaluation and member_arg's sum of
 * edge arguments; every complex dilogarithm skips the near-axis Taylor path.  Measures how far the
 * shared-algorithm tables sit from the reference's own operation order (tests/test_oracle_reference_order.py). */
void ora_set_reference_order(int level)
{
    g_ref_order = level != 0;
    ora_cdilog_set_general(level);
}
static void member_dc_ref(double S, double t, double gr, double *re, double *im)
{
    const zc z = zrdiv(1 + S + t, zmk(2 + t, -gr));
    ora_complex_dilog_xy(z.r, z.i, re, im);
}
static double member_arg_ref(double S, double t, double gr)
{
    return zarg(zneg(zdiv(zmk(-1 + S, gr), zmk(2 + t, -gr))));
}
static double member_arg(double S, double t, double gr)
{
    if (g_ref_order) return member_arg_ref(S, t, gr);
    const double c = 2 + t;
    double sS, fS, sT, fT;
    if (S < 1.0) { sS = -ora_atan2(gr, 1.0 - S); fS = 1.0; } else { sS = ora_atan2(gr, S - 1.0); fS = 0.0; }
    if (c < 0.0) { sT = -ora_atan2(gr, -c); fT = 1.0; } else { sT = ora_atan2(gr, c); fT = 0.0; }
    return (sS + sT) + (fS + fT - 1.0) * M_PI;
}

double ora_alpha(ora_state *S, double Em, double Ep, double Emp, double Epp)   /* nuSIprop.hpp:1237-1520 */
{
    const double g = S->p.g, mphi = S->p.mphi;
    const double Ga = width_of(S);
    const double g4 = SQ(SQ(g)), m2 = SQ(mphi), m4 = SQ(SQ(mphi));
    const double gr = Ga / mphi;
    const int maj = S->p.majorana;
    double tot = 0;
    for (int k = 0; k < 3; ++k) {
        const double mk = S->mn[k], uk = u2(S, k);
        double tp = -2 * mk * Ep / m2, tm = -2 * mk * Em / m2;
        const double Sp = 2 * mk * Epp / m2, Sm = 2 * mk * Emp / m2;
        if (fabs(tm + 1) < 1e-7) tm += tm * 1e-6;
        if (fabs(tp + 1) < 1e-7) tp += tp * 1e-6;
        const double wgt = m4 / (2 * mk);

        /* s channel */
        double as;
        if (Sp < 1e-5)
            as = g4 / (8 * M_PI * Ga * CU(mphi)) * (tm - tp) *
                 ((gr * (1 + SQ(gr) + 2 * Sm)) / SQ(1 + SQ(gr)) * (Sp - Sm) + gr / SQ(1 + SQ(gr)) * SQ(Sp - Sm));
        else
            as = g4 / (8 * M_PI * Ga * CU(mphi)) * (tm - tp) * ora_atandiff(mphi * (Sp - 1) / Ga, mphi * (Sm - 1) / Ga);
        as *= uk;
        if (!maj) as /= 2.;
        if (CH(S, ORA_CH_S)) tot += wgt * as;
        if (!S->p.non_resonant) continue;

        const double Lmt = ora_log1p(-tm), Lmp = ora_log1p(-tp);
        const double lSm = ora_log(Sm), lSp = ora_log(Sp);
        const double Lmm = ora_log1p(Sm + tm), Lpm = ora_log1p(Sp + tm), Lmq = ora_log1p(Sm + tp), Lpq = ora_log1p(Sp + tp);
        /* t channel */
        double at;
        if (maj) {
            const double LA = ora_log(((1 + Sm + tm) * (-1 + tp)) / ((-1 + tm) * (1 + Sm + tp)));
            const double LB = ora_log(((1 + Sp + tm) * (-1 + tp)) / ((-1 + tm) * (1 + Sp + tp)));
            const double SS = Sm * Sp;
            const double inner = SS * (-tm + tp) * lSm + SS * (tm - tp) * lSp - SS * Lmm - SS * tp * Lmm + SS * Lpm + SS * tp * Lpm
                                 - Sp * LA - Sp * tm * LA - Sp * tp * LA - Sp * tm * tp * LA
                                 + SS * ora_log(1 + Sm + tp) + SS * tm * Lmq
                                 + Sm * LB + Sm * tm * LB + Sm * tp * LB + Sm * tm * tp * LB
                                 - SS * ora_log(1 + Sp + tp) - SS * tm * Lpq;
            at = g4 / (Sm * Sp * 16 * M_PI * m4) *
                 (-((Sm - Sp) * (3 + 2 * tm * (-1 + tp) - 2 * tp) * (tm - tp)) / ((-1 + tm) * (-1 + tp))
                  + 2 * inner / ((1 + tm) * (1 + tp))
                  - ((SS * ora_log((Sm * (1 + Sp + tm)) / (Sp * (1 + Sm + tm)))) / SQ(1 + tm)
                     + (((Sm - Sp) * (tm - tp) * (1 + tp)) / (1 + tm) - SS * ora_log((Sm * (1 + Sp + tp)) / (Sp * (1 + Sm + tp)))) / SQ(1 + tp)));
            if (at < 0) at = gl33_rect(tp, tm, Sm, Sp, F_t_maj) * (g4 / (16 * M_PI * m4));
        } else {
            const double brk = -((tm - tp) * (2 + tm * (-1 + tp) - tp)) - 2 * (-1 + tm) * (-1 + tp) * (Lmt - Lmp);
            at = 3. / 2. * g4 / (32 * M_PI * m4 * Sm * Sp * (-1 + tm) * (-1 + tp)) * (Sm - Sp) * brk;
            if (at < 0) at = gl33_rect(tp, tm, Sm, Sp, F_t_dir) * (3. / 2. * g4 / (32 * M_PI * m4));
        }
        at *= uk;
        if (CH(S, ORA_CH_T)) tot += wgt * at;

        /* u channel */
        double au;
        if (maj) au = at;
        else {
            const double brk = -((tm - tp) * (2 + tm * (-1 + tp) - tp)) - 2 * (-1 + tm) * (-1 + tp) * (Lmt - Lmp);
            au = 1. / 2. * g4 / (32 * M_PI * m4 * Sm * Sp * (-1 + tm) * (-1 + tp)) * (Sm - Sp) * brk;
            if (au < 0) au = gl33_rect(tp, tm, Sm, Sp, F_t_dir) * (1. / 2. * g4 / (32 * M_PI * m4));
            au *= uk;
        }
        if (CH(S, ORA_CH_U)) tot += wgt * au;

        /* t-u interference */
        double atu;
        if (maj) {
            double Fp, Fm;
            if (tp < -1) Fp = ora_dilog((1 + Sm + tp) / Sm) - ora_dilog((1 + Sp + tp) / Sp);
            else Fp = -ora_dilog(Sm / (1 + Sm + tp)) + ora_dilog(Sp / (1 + Sp + tp))
                      - 0.5 * (SQ(ora_log((1 + Sm + tp) / Sm)) - SQ(ora_log((1 + Sp + tp) / Sp)));
            if (tm < -1) Fm = -ora_dilog((1 + Sm + tm) / Sm) + ora_dilog((1 + Sp + tm) / Sp);
            else Fm = ora_dilog(Sm / (1 + Sm + tm)) - ora_dilog(Sp / (1 + Sp + tm))
                      + 0.5 * (SQ(ora_log((1 + Sm + tm) / Sm)) - SQ(ora_log((1 + Sp + tm) / Sp)));
            const double lap = (tp > -1) ? ora_log1p(tp) : ora_log(-1 - tp);
            const double lam = (tm > -1) ? ora_log1p(tm) : ora_log(-1 - tm);
            const double SS = Sm * Sp, P = (1 + tm) * (1 + tp);
            const double l2m = ora_log((2 + Sm) / Sm), l2p = ora_log((2 + Sp) / Sp);
            atu = g4 / (32 * M_PI * m4 * Sm * Sp * (1 + tm) * (1 + tp)) *
                  (-4 * (Sm - Sp) * (1 + tm) * (tm - tp) * (1 + tp)
                   + 2 * SS * tp * (ora_log(Sm / Sp) - Lmm + Lpm)
                   + 2 * Sp * (1 + tm) * (1 + tp) * (Lmt - Lmm - Lmp + Lmq)
                   - 2 * Sm * (1 + tm) * (1 + tp) * (Lmt - Lpm - Lmp + Lpq)
                   + 2 * SS * (-Lmm + Lpm + Lmq - Lpq)
                   + SS * (1 + tm) * (1 + tp) * (l2m * (lSp + Lmq) - l2p * (lSm + Lpq) + Lmp * (ora_log(Sm / Sp) - Lmq + Lpq))
                   + SS * (1 + tm) * (1 + tp) * ((lSp + Lmm) * (ora_log(Sm / (2 + Sm)) + Lmt - lam) + (lSm + Lpm) * (l2p - Lmt + lam))
                   + SS * (ora_log(Sp / Sm) + Lmq - Lpq) * (2 * tm + P * lap)
                   + SS * (1 + tm) * (1 + tp) * (ora_dilog((1 + Sm + tm) / (2 + Sm)) - ora_dilog((1 + Sp + tm) / (2 + Sp))
                                                 - ora_dilog((1 + Sm + tp) / (2 + Sm)) + ora_dilog((1 + Sp + tp) / (2 + Sp)))
                   + SS * (1 + tm) * (1 + tp) * (Fp + Fm));
            /* nuSIprop.hpp:1401-1418: the quadrature fallback writes a shadowing
             * local, so a negative alpha_tu is kept as is. */
        } else
            atu = 0.;
        atu *= uk;
        if (CH(S, ORA_CH_TU)) tot += wgt * atu;

        /* s-t interference: 8 GSL complex dilogs (nuSIprop.hpp:1431-1451) */
        const double z1 = (1 + Sm + tm) / (1 + tm);
        const double z3 = (1 + Sp + tm) / (1 + tm);
        const double z5 = (1 + Sm + tp) / (1 + tp);
        const double z7 = (1 + Sp + tp) / (1 + tp);
        double R[9], J[9];
        ora_complex_dilog_xy(z1, 0, &R[1], &J[1]);
        member_dc(Sm, tm, gr, &R[2], &J[2]);   /* (1+Sm+tm)/(2 - I gr + tm) */
        ora_complex_dilog_xy(z3, 0, &R[3], &J[3]);
        member_dc(Sp, tm, gr, &R[4], &J[4]);
        ora_complex_dilog_xy(z5, 0, &R[5], &J[5]);
        member_dc(Sm, tp, gr, &R[6], &J[6]);
        ora_complex_dilog_xy(z7, 0, &R[7], &J[7]);
        member_dc(Sp, tp, gr, &R[8], &J[8]);
        const double Lsm = ora_log1p(SQ(-1 + Sm) / SQ(gr)), Lsp = ora_log1p(SQ(-1 + Sp) / SQ(gr));
        double ast;
        if (maj) {
            const double cm = zarg_real(-(1 / (1 + tm))), cp = zarg_real(-(1 / (1 + tp)));
            const zc nm_ = zmk(-1 + Sm, gr), np_ = zmk(-1 + Sp, gr);      /* -1 + I gr + S */
            const double L2m = ora_log1p(SQ(2 + tm) / SQ(gr)), L2p = ora_log1p(SQ(2 + tp) / SQ(gr));
            const double am = ora_log(fabs(1 + tm)), ap = ora_log(fabs(1 + tp));
            ast = g4 / (32 * M_PI * (1 + SQ(gr)) * m4) *
                  (2 * gr * (J[1] - J[2] - J[3] + J[4] - J[5] + J[6] + J[7] - J[8])
                   - 2 * (R[1] - R[2] - R[3] + R[4] - R[5] + R[6] + R[7] - R[8])
                   + 2 * gr * (cm - member_arg(Sm, tm, gr)) * Lmm
                   - 2 * gr * (cm - member_arg(Sp, tm, gr)) * Lpm
                   + 2 * gr * (cp - member_arg(Sp, tp, gr)) * Lpq
                   - 2 * gr * (cp - member_arg(Sm, tp, gr)) * Lmq
                   + 2 * (gr * zarg(nm_) - gr * zarg(np_) + Lsp / 2. - Lsm / 2. + lSm - lSp) * (2 * (tm - tp) + (Lmt - Lmp))
                   + Lmm * (Lsm - L2m - 2 * (lSm - am)) - Lpm * (Lsp - L2m - 2 * (lSp - am))
                   - Lmq * (Lsm - L2p - 2 * (lSm - ap)) + Lpq * (Lsp - L2p - 2 * (lSp - ap)));
        } else
            ast = g4 / (32 * M_PI * (1 + SQ(gr)) * m4) *
                  ((2 * gr * zarg(zmk(-1 + Sm, gr)) - 2 * gr * zarg(zmk(-1 + Sp, gr)) + 2 * lSm - 2 * lSp + Lsp - Lsm) * (tm - tp + Lmt - Lmp));
        ast *= uk;
        if (CH(S, ORA_CH_ST)) tot += wgt * ast;
        const double asu = maj ? ast : 0.;
        if (CH(S, ORA_CH_SU)) tot += wgt * asu;

        /* double scalar production */
        double app = 0;
        if (Sm > 4 && S->p.phiphi) {
            if (Sm < 1e4) {
                const double d = Sp / Sm;
                const double xx[3] = {Sm, ora_log(-Sm / tm) / ora_log(d) * 1.0001, ora_log10(d)};
                double v;
                pp_lookup(S, &S->spl_a, xx, &v);
                app = g4 / m4 * fabs(v);
            } else if (tm < -1) {
                const double l1m = ora_log(-1 - tm), l0m = ora_log(-tm), l1p = ora_log(-1 - tp), l0p = ora_log(-tp);
                app = g4 / m4 *
                      ((-Sm + Sp) * ((tm - tp) * (Sp * (-2 + tm + tp) + Sm * (-2 - 24 * Sp + tm + tp))
                                     + 4 * (-(Sp * (1 + tm)) + Sm * (-1 + 2 * Sp + (-1 + Sp) * tm)) * l1m
                                     + 2 * (3 * Sp + Sm * (3 + 4 * Sp)) * tm * l0m
                                     + 4 * (Sp + Sp * tp + Sm * (1 + tp - Sp * (2 + tp))) * l1p
                                     - 2 * (3 * Sp + Sm * (3 + 4 * Sp)) * tp * l0p)
                       + 2 * SQ(Sm) * lSp * ((3 + 2 * Sp) * (tm - tp) + 2 * SQ(Sp) * ((-1 - tm) * l1m + tm * l0m + (1 + tp) * l1p - tp * l0p))
                       + 2 * SQ(Sp) * lSm * ((-3 - 2 * Sm) * (tm - tp) + 2 * SQ(Sm) * ((1 + tm) * l1m - tm * l0m - (1 + tp) * l1p + tp * l0p)))
                      / (256. * M_PI * SQ(Sm) * SQ(Sp));
            } else if (tp < -1) {
                const double l1p = ora_log(-1 - tp), l0p = ora_log(-tp);
                app = g4 / m4 *
                      ((2 * SQ(Sm) * lSp * ((1 + tp) * (-3 - 2 * Sp + 2 * SQ(Sp) * l1p) - 2 * SQ(Sp) * tp * l0p)
                        + (Sm - Sp) * ((1 + tp) * (-3 * (Sm + Sp + 8 * Sm * Sp) + (Sm + Sp) * tp)
                                       + 4 * (-(Sp * (1 + tp)) + Sm * (-1 + 2 * Sp + (-1 + Sp) * tp)) * l1p
                                       + 2 * (3 * Sp + Sm * (3 + 4 * Sp)) * tp * l0p)
                        + 2 * SQ(Sp) * lSm * ((3 + 2 * Sm) * (1 + tp) + 2 * SQ(Sm) * (-((1 + tp) * l1p) + tp * l0p)))
                           / (256. * M_PI * SQ(Sm) * SQ(Sp))
                       + (-1 - tm) * (-6 * Sm + 6 * Sp - 2 * (-2 + Sm) * Sp * lSm + Sm * Sp * SQ(lSm) + 2 * Sm * (-2 + Sp) * lSp - Sm * Sp * SQ(lSp))
                             / (128. * M_PI * Sm * Sp));
            } else
                app = g4 / m4 * (tp - tm) *
                      (-6 * Sm + 6 * Sp - 2 * (-2 + Sm) * Sp * lSm + Sm * Sp * SQ(lSm) + 2 * Sm * (-2 + Sp) * lSp - Sm * Sp * SQ(lSp))
                      / (128. * M_PI * Sm * Sp);
            app *= uk;
            if (maj) app *= 2;
            app *= 2;
            if (maj) app *= 2;
        }
        if (CH(S, ORA_CH_PP)) tot += wgt * app;

        const double nrm = SQ(SQ(g / mphi));
        if (as < 0 || at / nrm < -1e-11 || au / nrm < -1e-11 || atu / nrm < -1e-11 || (ast + as + at) / nrm < -1e-11)
            S->warn |= 4;
    }
    return tot;
}

/* ----------------------------------------------------------------------------
 * object: constructor (nuSIprop.hpp:61-171), evolve (176-337)
 * ------------------------------------------------------------------------- */
static void build_grid(ora_state *S)
{
    const int N = S->p.N_bins_E;
    const double lo = S->p.lEmin, hi = S->p.lEmax;
    for (int i = 0; i < N; ++i) {
        S->Emin[i] = pow(10, lo + (hi - lo) * (i * 1.0) / N);
        S->Enu[i] = pow(10, lo + (hi - lo) * (i + 0.5) / N);
        S->Emax[i] = pow(10, lo + (hi - lo) * (i + 1.0) / N);
    }
}

/* nuSIprop.hpp:130-163.  The reference keeps std::complex<double> U and uses
 * only std::norm(U); the entries are formed here with the same real
 * operations (real*complex component-wise, s13/del by Smith's division) so
 * that the product's host code, which does the same, gets identical bits. */
static void build_pmns(ora_state *S)
{
    double t12, t13, t23, dcp;
    if (S->p.normal_ordering) { t12 = 33.44 * (M_PI / 180); t13 = 8.57 * (M_PI / 180); t23 = 49.0 * (M_PI / 180); dcp = 195.0 * (M_PI / 180); }
    else { t12 = 33.45 * (M_PI / 180); t13 = 8.61 * (M_PI / 180); t23 = 49.3 * (M_PI / 180); dcp = 286.0 * (M_PI / 180); }
    const double c12 = cos(t12), c13 = cos(t13), c23 = cos(t23);
    const double s12 = sin(t12), s13 = sin(t13), s23 = sin(t23);
    const zc del = zmk(cos(dcp), sin(dcp));
    zc U[3][3];
    U[0][0] = zre(c12 * c13);
    U[0][1] = zre(s12 * c13);
    U[0][2] = zrdiv(s13 * 1.0, del);
    U[1][0] = zrsub(-s12 * c23, zscale(c12 * s23 * s13, del));
    U[1][1] = zrsub(c12 * c23, zscale(s12 * s23 * s13, del));
    U[1][2] = zre(s23 * c13);
    U[2][0] = zrsub(s12 * s23, zscale(c12 * c23 * s13, del));
    U[2][1] = zrsub(-c12 * s23, zscale(s12 * c23 * s13, del));
    U[2][2] = zre(c23 * c13);
    for (int f = 0; f < 3; ++f)
        for (int k = 0; k < 3; ++k) S->U2m[f][k] = U[f][k].r * U[f][k].r + U[f][k].i * U[f][k].i;
}

ora_state *ora_create(const ora_params *p, int *err)
{
    ora_state *S = (ora_state *)calloc(1, sizeof(ora_state));
    S->p = *p;
    const int N = p->N_bins_E;
    if (N < 2 || p->flav < 0 || p->flav > 2 || !(p->lEmax > p->lEmin)) { free(S); if (err) *err = -1; return NULL; }
    S->N = N;
    S->Emin = (double *)malloc(sizeof(double) * (size_t)N);
    S->Emax = (double *)malloc(sizeof(double) * (size_t)N);
    S->Enu = (double *)malloc(sizeof(double) * (size_t)N);
    build_grid(S);
    S->Nz = (int)(log((1 + p->zmax) / (1 + 0)) / log(S->Emax[0] / S->Emin[0]) + 2);
    S->z = (double *)malloc(sizeof(double) * (size_t)S->Nz);
    for (int i = 0; i < S->Nz; ++i) S->z[i] = (1 + 0) * pow(S->Emax[0] / S->Emin[0], i) - 1;
    S->zmax_eff = S->z[S->Nz - 1];
    S->T = N + S->Nz - 2;
    build_pmns(S);
    S->norm_total = 0;   /* uninitialised in the reference until the first evolve() */
    S->chan = ORA_CH_ALL;
    if (err) *err = 0;
    return S;
}

void ora_destroy(ora_state *S)
{
    if (!S) return;
    if (S->have_pp) { ora_spline_free(&S->spl_at); ora_spline_free(&S->spl_a); }
    free(S->Emin); free(S->Emax); free(S->Enu); free(S->z);
    free(S);
}

int ora_load_phiphi(ora_state *S, const char *at_path, const char *a_path)
{
    /* nuSIprop.hpp:166-170 : dims {5000,100} and {1000,1000,100}, x0 logarithmic */
    const int n2[2] = {5000, 100}, n3[3] = {1000, 1000, 100};
    const int lg2[3] = {1, 0, 0}, lg3[4] = {1, 0, 0, 0};
    int r = ora_spline_load(&S->spl_at, 2, n2, at_path, 0, lg2);
    if (!r) r = ora_spline_load(&S->spl_a, 3, n3, a_path, 0, lg3);
    S->have_pp = (r == 0);
    return r;
}

/* test hook: same, with caller-chosen node counts (synthetic small tables) */
int ora_load_phiphi_dims(ora_state *S, const char *at_path, const int *n2, const char *a_path, const int *n3)
{
    const int lg2[3] = {1, 0, 0}, lg3[4] = {1, 0, 0, 0};
    int r = ora_spline_load(&S->spl_at, 2, n2, at_path, 0, lg2);
    if (!r) r = ora_spline_load(&S->spl_a, 3, n3, a_path, 0, lg3);
    S->have_pp = (r == 0);
    return r;
}

int ora_set_params(ora_state *S, double mphi, double g, double mntot, double si, double norm)
{
    S->p.mphi = mphi; S->p.g = g; S->p.mntot = mntot; S->p.si = si; S->p.norm = norm;
    return 0;
}

int ora_N(const ora_state *S) { return S->N; }
int ora_Nz(const ora_state *S) { return S->Nz; }
int ora_T(const ora_state *S) { return S->T; }
double ora_zmax(const ora_state *S) { return S->zmax_eff; }
int ora_warnings(const ora_state *S) { return S->warn; }
void ora_grid(const ora_state *S, double *Emin, double *Emax, double *Enu, double *z)
{
    memcpy(Emin, S->Emin, sizeof(double) * (size_t)S->N);
    memcpy(Emax, S->Emax, sizeof(double) * (size_t)S->N);
    memcpy(Enu, S->Enu, sizeof(double) * (size_t)S->N);
    memcpy(z, S->z, sizeof(double) * (size_t)S->Nz);
}
void ora_mixing(const ora_state *S, double *U2)
{
    for (int f = 0; f < 3; ++f)
        for (int k = 0; k < 3; ++k) U2[3 * f + k] = S->U2m[f][k];
}

int ora_prepare(ora_state *S)   /* nuSIprop.hpp:184-205 */
{
    const double dmq21 = 7.42e-5;
    const double dmqAT = S->p.normal_ordering ? 2.514e-3 : -2.497e-3;
    double mL;
    if (ora_getmL(S->p.mntot, dmq21, dmqAT, &mL)) return -2;
    if (S->p.normal_ordering) {
        S->mn[0] = mL;
        S->mn[1] = sqrt(dmq21 + SQ(mL));
        S->mn[2] = sqrt(dmqAT + SQ(mL));
    } else {
        S->mn[2] = mL;
        S->mn[1] = sqrt(SQ(mL) - dmqAT);
        S->mn[0] = sqrt(SQ(S->mn[1]) - dmq21);
    }
    S->norm_total = S->p.norm / flux_FS_E0(S);
    return 0;
}
void ora_masses(const ora_state *S, double *mn3, double *norm_total)
{
    for (int k = 0; k < 3; ++k) mn3[k] = S->mn[k];
    *norm_total = S->norm_total;
}

static void edges(const ora_state *S, int n, double *lo, double *hi)   /* nuSIprop.hpp:224-233 */
{
    const int N = S->N;
    if (n < N) { *lo = S->Emin[n]; *hi = S->Emax[n]; }
    else { *lo = S->Emin[N - 1] * (1 + S->z[n - N + 1]); *hi = S->Emax[N - 1] * (1 + S->z[n - N + 1]); }
}

int ora_tables(ora_state *S, double *Gam, double *aT, double *al)   /* nuSIprop.hpp:217-253 */
{
    const int T = S->T;
    S->err = 0;
    if (S->p.phiphi && S->p.non_resonant && !S->have_pp) return -3;
    for (int n = 0; n < T; ++n) {
        double lo, hi;
        edges(S, n, &lo, &hi);
        Gam[n] = ora_Gamma(S, lo, hi);
        aT[n] = ora_alphaTilde(S, lo, hi);
        for (int m = n + 1; m < T; ++m) {
            double lo2, hi2;
            edges(S, m, &lo2, &hi2);
            al[(size_t)n * T + m] = ora_alpha(S, lo, hi, lo2, hi2);
        }
    }
    return S->err;
}

/* gsl_linalg_LU_decomp + gsl_linalg_LU_solve on 3x3 (partial pivoting, Doolittle) */
static void lu3_solve(double A[3][3], const double b[3], double x[3])
{
    int perm[3] = {0, 1, 2};
    for (int j = 0; j < 2; ++j) {
        double amax = fabs(A[j][j]);
        int ip = j;
        for (int i = j + 1; i < 3; ++i) if (fabs(A[i][j]) > amax) { amax = fabs(A[i][j]); ip = i; }
        if (ip != j) {
            for (int c = 0; c < 3; ++c) { const double t = A[j][c]; A[j][c] = A[ip][c]; A[ip][c] = t; }
            const int t = perm[j]; perm[j] = perm[ip]; perm[ip] = t;
        }
        const double ajj = A[j][j];
        if (ajj != 0.0)
            for (int i = j + 1; i < 3; ++i) {
                const double aij = A[i][j] / ajj;
                A[i][j] = aij;
                for (int c = j + 1; c < 3; ++c) A[i][c] = A[i][c] - aij * A[j][c];
            }
    }
    for (int i = 0; i < 3; ++i) x[i] = b[perm[i]];
    for (int i = 0; i < 3; ++i) { double t = x[i]; for (int c = 0; c < i; ++c) t -= A[i][c] * x[c]; x[i] = t; }
    for (int i = 2; i >= 0; --i) { double t = x[i]; for (int c = i + 1; c < 3; ++c) t -= A[i][c] * x[c]; x[i] = t / A[i][i]; }
}

int ora_cascade(ora_state *S, const double *Gam, const double *aT, const double *al, double *flux, double *flux_fla)
{
    const int N = S->N, Nz = S->Nz, T = S->T;
    const double *z = S->z, *Emin = S->Emin, *Emax = S->Emax;
    double uu[3];
    for (int k = 0; k < 3; ++k) uu[k] = u2(S, k);
    double *F[3] = {flux, flux + N, flux + 2 * N};
    for (int k = 0; k < 3; ++k) for (int b = 0; b < N; ++b) F[k][b] = 0;
    double *awo = (double *)calloc((size_t)N, sizeof(double));
    const double dlogz = log(1 + z[1]) - log(1 + z[0]);
    for (int i = Nz - 1; i > 0; --i) {
        const double H = H_of(z[i - 1]);
        const double sfac = nd_of(z[i - 1]) / SQ(1 + z[i - 1]);
        const double c = (1 + z[i - 1]) * dlogz / H;
        double acc[3] = {0, 0, 0};
        for (int j = N; j > 0; --j) {
            const double Gwo = sfac * Gam[j + i - 2];
            const double aTwo = sfac * aT[j + i - 2];
            if (S->p.non_resonant)
                for (int m = j; m < N; ++m) awo[m] = sfac * al[(size_t)(j + i - 2) * T + (m + i - 1)];
            else if (j != N) {
                awo[j] = sfac * al[(size_t)(j + i - 2) * T + (j + i - 1)];
                for (int l = 0; l < 3; ++l) acc[l] += F[l][j] * awo[j] / (Emax[j] - Emin[j]) / (Emax[j - 1] - Emin[j - 1]);
            }
            const double dEb = Emax[j - 1] - Emin[j - 1];
            const double lum = ora_Lum(S, z[i], Emin[j - 1], Emax[j - 1]);
            double M[3][3], v[3], x[3];
            for (int k = 0; k < 3; ++k) {
                double src = c * lum;
                if (!S->p.non_resonant && j != N)
                    for (int l = 0; l < 3; ++l) src += c * acc[l] * uu[k] * uu[l] * dEb;
                else
                    for (int m = j; m < N; ++m)
                        for (int l = 0; l < 3; ++l) src += c * F[l][m] * awo[m] * uu[k] * uu[l] / (Emax[m] - Emin[m]);
                const double Znr = F[k][j - 1] + src;
                const double Zdr = 1.0 + c * (Gwo * uu[k] - aTwo * SQ(uu[k])) / dEb;
                v[k] = Znr / Zdr;
                for (int l = 0; l < 3; ++l) M[k][l] = (k == l) ? 1.0 : (aTwo * uu[k] * uu[l] / dEb) / Zdr;
            }
            lu3_solve(M, v, x);
            for (int k = 0; k < 3; ++k) F[k][j - 1] = x[k];
        }
    }
    free(awo);
    for (int b = 0; b < N; ++b)
        for (int k = 0; k < 3; ++k) F[k][b] /= (Emax[b] - Emin[b]);
    double U2[9];
    ora_mixing(S, U2);
    for (int b = 0; b < N; ++b)
        for (int f = 0; f < 3; ++f)
            flux_fla[f * N + b] = U2[3 * f + 0] * F[0][b] + U2[3 * f + 1] * F[1][b] + U2[3 * f + 2] * F[2][b];
    return 0;
}

int ora_evolve(ora_state *S, double *flux, double *flux_fla)
{
    int r = ora_prepare(S);
    if (r) return r;
    const size_t T = (size_t)S->T;
    double *Gam = (double *)malloc(sizeof(double) * T);
    double *aT = (double *)malloc(sizeof(double) * T);
    double *al = (double *)calloc(T * T, sizeof(double));
    r = ora_tables(S, Gam, aT, al);
    if (!r) r = ora_cascade(S, Gam, aT, al, flux, flux_fla);
    free(Gam); free(aT); free(al);
    return r;
}

double ora_check_energy_conservation(ora_state *S, double *flux, double *flux_fla)   /* nuSIprop.hpp:339-357 */
{
    const double E_FS = energy_FS(S);   /* uses the previous evolve()'s norm_total */
    if (ora_evolve(S, flux, flux_fla)) return NAN;
    double E_int = 0;
    const int N = S->N;
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < 3; ++k) E_int += (log(S->Emax[i]) - log(S->Emin[i])) * SQ(S->Enu[i]) * flux[k * N + i];
    return (E_int - E_FS) / E_FS;
}

/* test hooks: sum only the ORA_CH_* channels in Gamma / alphaTilde / alpha (quadrature and
 * additivity KATs, tests/test_oracle_quadrature.py) */
void ora_set_channels(ora_state *S, int mask) { S->chan = mask; }
