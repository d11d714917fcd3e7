// nuSIprop MI355X -- interaction integrals and source term, one table entry per call.
//
// Device restatement of calculate_flux's private physics (nuSIprop.hpp):
//   scalar_width   748-757      gamma_entry       759-922   (absorption Gamma)
//   alphat_entry   924-1235     (same-bin regeneration alphaTilde)
//   alpha_entry    1237-1520    (inter-bin regeneration alpha)
//   Lum / Lum_int / RSN / SFR / H / n_nu  573-662 (DSNB source and the
//   commented-out power-law source of :656, selected by Point::source)
// Same formulas, thresholds (Taylor switches, x<0 quadrature fallbacks,
// |t+1|<1e-7 nudges) and quirks (shadowed alpha_tu fallback :1406) as the
// reference; repeated sub-expressions are hoisted.  The double-scalar (phi-phi)
// spline lookups (:1199, :1483) go through a SplineSet (nusi_spline.hpp).
#pragma once

#include "nusi_math.hpp"
#include "nusi_spline.hpp"

// The three-mass loops (j/k = 0..2) are kept rolled by default: unrolled, the
// alpha kernel is ~225 KB of code (instruction-cache thrashing) and 300+
// VGPRs.  -DNUSI_MASS_UNROLLED restores full unrolling (A/B builds).
#ifdef NUSI_MASS_UNROLLED
#define NUSI_MASS_LOOP
#else
#define NUSI_MASS_LOOP _Pragma("unroll 1")
#endif

namespace nusi {

// Per-parameter-point constants, built on the host (nusi_capi.cpp) from the
// reference's constructor/evolve() set-up (nuSIprop.hpp:130-163, 184-205).
struct Point {
    double mphi, g, mntot, si, norm;
    double norm_total;   // norm / flux_FS_E0()  (nuSIprop.hpp:205)
    double Ga;           // scalar_width()       (nuSIprop.hpp:748-757)
    double mn[3];        // masses               (nuSIprop.hpp:191-203)
    double u[3];         // |U_flav,k|^2
    double U2[9];        // |U_fk|^2, row-major, for the flavour basis
    int majorana, non_resonant, phiphi, source;
    int tslot;           // Stage-A table slot of this point (points that differ only in si / norm /
                         // source share their tables: nuSIprop.hpp:217-253 read none of them)
    // alpha()'s entry-independent factors (point_derive), each the exact subexpression the
    // reference evaluates per entry (nuSIprop.hpp:1243-1275, 1430, 1505)
    double a_wgt[3];     // m_phi^4 / (2 m_k)
    double a_s;          // g^4 / (8 pi Ga m_phi^3)
    double a_st;         // g^4 / (32 pi (1 + gr^2) m_phi^4)
    double a_nrm;        // (g / m_phi)^4
    double a_gr;         // Ga / m_phi
};
NUSI_FN void point_derive(Point& P)
{
    const double g = P.g, mphi = P.mphi, Ga = P.Ga;
    const double g4 = (g * g) * (g * g), m4 = (mphi * mphi) * (mphi * mphi);
    const double gr = Ga / mphi, gr2 = gr * gr;
    for (int k = 0; k < 3; ++k) P.a_wgt[k] = m4 / (2 * P.mn[k]);
    P.a_s = g4 / (8 * kPi * Ga * (mphi * mphi * mphi));
    P.a_st = g4 / (32 * kPi * (1 + gr2) * m4);
    P.a_nrm = (g / mphi) * (g / mphi) * ((g / mphi) * (g / mphi));
    P.a_gr = gr;
}

enum { kWarnGamma = 1, kWarnAlphaTilde = 2, kWarnAlpha = 4, kWarnSplineOOB = 8 };

// ---------------------------------------------------------------------------
// cosmology and source (nuSIprop.hpp:573-662)
// ---------------------------------------------------------------------------
NUSI_FN double lum_int_dsnb(double z, double E)
{
    const double T = 6e6;
    const double ey = nm::exp(-E * (1 + z) / T);
    const double pref = 1.5252316492673872e-14;  // Etot*120/(6*7*pow(M_PI,4)*pow(Tnue,2)), as libm evaluates it
    return pref * (-E * E * (1 + z) * nm::log(ey + 1) / T + 2 * E * li2(-ey) + 2 * T * li3(-ey) / (1 + z));
}
// integral of the source over [Em,Ep] at redshift z (nuSIprop.hpp:656 / 659-662);
// sfr_z = get_SFR(z) (nuSIprop.hpp:591-605), a grid quantity computed on the host
NUSI_FN double lum(const Point& P, double z, double sfr_z, double Em, double Ep)
{
    if (P.source == 1) {
        const double E0 = 1e14, si = P.si;
        return P.norm_total / 3.0 * sfr_z * (Ep * nm::pow(Ep / E0 * (1 + z), -si) - Em * nm::pow(Em / E0 * (1 + z), -si)) / (1 - si);
    }
    const double rsn = sfr_z * 0.01 / (1.989 * 56.1);
    return (lum_int_dsnb(z, Ep) - lum_int_dsnb(z, Em)) * rsn;
}

// ---------------------------------------------------------------------------
// quadrature fallbacks
// ---------------------------------------------------------------------------
NUSI_FN double gl3_Gtu_nores(double a, double b)  // nuSIprop.hpp:805-809
{
    double s = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const double z = (b - a) / 2. * kGLx[q] + (b + a) / 2.;
        s += kGLw[q] * ((z + 2) / (z * (z + 1)) - 2 / (z * z) * nm::log1p(z));
    }
    return s;
}
NUSI_FN double gl3_Gtu_int(double a, double b)  // nuSIprop.hpp:829-833
{
    double s = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const double z = (b - a) / 2. * kGLx[q] + (b + a) / 2.;
        s += kGLw[q] * (1 / z - 2 * (1 + z) / ((z * z) * (2 + z)) * nm::log1p(z));
    }
    return s;
}
NUSI_FN double gl3_Gpp(double a, double b)  // nuSIprop.hpp:895-900
{
    double s = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const double z = (b - a) / 2. * kGLx[q] + (b + a) / 2.;
        const double r = sqrt(z * (z - 4));
        const double qq = (r + z - 2) / (r - z + 2);
        s += kGLw[q] * ((z * z - 4 * z + 6) / ((z * z) * (z - 2)) * nm::log(qq * qq) - 6 * r / (z * z));
    }
    return s;
}
// kind: 0 = Majorana t (two terms), 1 = Dirac t/u, 2 = t-u interference
NUSI_FN double Fkernel(int kind, double y, double x)
{
    if (kind == 0) {
        const double a = y / x, b = (-x - y) / x, c = (-x - y) - 1;
        return (a * a) / ((y - 1) * (y - 1)) + (b * b) / (c * c);
    }
    if (kind == 1) {
        const double a = y / x;
        return (a * a) / ((y - 1) * (y - 1));
    }
    return 2 * y * (-y - x) / (x * x) / ((y - 1) * (-y - x - 1));
}
// y in [tp,tm], x in [-y,-tp] (nuSIprop.hpp:987-1003)
NUSI_FN_OUT double gl33_tri(int kind, double tp, double tm)   // cold: fallback only
{
    double acc = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double y = (tm - tp) / 2. * kGLx[i] + (tm + tp) / 2.;
        const double ax = -y, bx = -tp;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double x = (bx - ax) / 2. * kGLx[j] + (bx + ax) / 2.;
            acc += 1. / 4. * (tm - tp) * (bx - ax) * kGLw[i] * kGLw[j] * Fkernel(kind, y, x);
        }
    }
    return acc;
}
// y in [tp,tm], x in [Sm,Sp] (nuSIprop.hpp:1288-1301)
NUSI_FN_OUT double gl33_rect(int kind, double tp, double tm, double Sm, double Sp)   // cold: fallback only
{
    double acc = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double y = (tm - tp) / 2. * kGLx[i] + (tm + tp) / 2.;
            const double x = (Sp - Sm) / 2. * kGLx[j] + (Sp + Sm) / 2.;
            acc += kGLw[i] * kGLw[j] * Fkernel(kind, y, x);
        }
    return acc * (1. / 4. * (tm - tp) * (Sp - Sm));
}

template <bool kRef = false>
NUSI_FN double gpp_analytic(double a, double b)  // nuSIprop.hpp:885 with a = max(s-,4)
{
    const double ra4 = sqrt(-4 + a), ra = sqrt(a), rb4 = sqrt(-4 + b), rb = sqrt(b);
    const double qa = sqrt((-4 + a) * a), qb = sqrt((-4 + b) * b);
    const double A1 = ra4 - ra, A2 = -2 + a + qa, A3 = 2 - a + qa, A4 = ra4 + ra;
    const double B1 = rb4 - rb, B2 = -2 + b + qb, B3 = 2 - b + qb, B4 = rb4 + rb;
    return 12 * sqrt((-4 + a) / a) - 12 * sqrt((-4 + b) / b)
           - 2 * nm::log(A1 * A1 / 4.) * nm::log(A2 * A2 / 4.)
           - ((6 + a * nm::log((-2 + a) * a)) * nm::log(A2 * A2 / (A3 * A3))) / a
           - 24 * (sqrt((-4 + a) / a) - sqrt((-4 + b) / b) - nm::log(A4) + nm::log(B4))
           + 2 * nm::log(B1 * B1 / 4.) * nm::log(B2 * B2 / 4.)
           + ((6 + b * nm::log((-2 + b) * b)) * nm::log(B2 * B2 / (B3 * B3))) / b
           + 8 * dilogdiff<kRef>(4 / (A4 * A4), 4 / (B4 * B4))
           + 2 * dilogdiff<kRef>(4 / (A2 * A2), 4 / (B2 * B2));
}

// ---------------------------------------------------------------------------
// Gamma(Em, Ep)  -- nuSIprop.hpp:759-922
// ---------------------------------------------------------------------------
// The entries sum their channels' terms over the mass states into one accumulator, in the reference's order
// (channel by channel within a state, state after state).  The per-state bodies (gamma_k, alphat_k) hand each term
// wgt * X to a sink with its channel slot and the unscaled X: SumSink accumulates as the reference does (gamma_entry,
// alphat_entry: the per-entry paths and the host checks); k_gamma_alphat runs each (mass state, part) on a wave of its
// own -- kPart 0: every channel but the s-t / s-u interference, 1: those two (the complex dilogarithms), -1: all --
// stores the terms by slot and sums them on one wave in slot order, state after state: the same additions of the same
// values, so the same bits.  The warnings, which read several channels, are formed from the unscaled values
// (gamma_warn, alphat_warn) by whoever holds them all.
struct SumSink {
    double tot = 0;
    NUSI_FN void put(int, double x, double) { tot += x; }
};
constexpr int kGammaSlots = 6;    // s, t+u, t-u (int), s-t, s-u, phi-phi
constexpr int kAlphatSlots = 7;   // s, t, u, t-u, s-t, s-u, phi-phi
NUSI_FN int gamma_warn(double Gs, double Gtu0, double Gint, double Gst, double Gsu)
{
    return (Gs < 0 || Gtu0 < 0 || Gint < 0 || (Gs + Gtu0 + Gst + Gsu) < 0) ? kWarnGamma : 0;
}
NUSI_FN int alphat_warn(double as, double at, double au, double atu, double ast, double asu, double nrm)
{
    return (as < 0 || at < 0 || au < 0 || atu / nrm < -1e-11 || (ast + at + as) / nrm < -1e-11 || (asu + au + as) / nrm < -1e-11)
               ? kWarnAlphaTilde : 0;
}
// Gamma's dilogarithms of one bin edge (E, s = 2 m_j E / m_phi^2): li2(-s), li2(-1 - s) and Li2 of
// z = i (1 + s) / (gr + 2 i) (and, in the shared-algorithm order, of conj z) -- the edge-shared path of
// k_gamma_alphat evaluates them once per edge for the two bins it bounds (the *_pre forms, nusi_math.hpp)
struct GammaEdgeVals { double ls, l1s; cd cz, czc; };
struct GammaEdgePair { GammaEdgeVals lo, hi; };
constexpr unsigned kGeLs = 1, kGeL1s = 2, kGeCz = 4;
template <bool kRef>
NUSI_FN void gamma_edge_vals(const Point& P, int j, double E, unsigned need, GammaEdgeVals& v)
{
    const double mphi = P.mphi, Ga = P.Ga, m2 = mphi * mphi, gr = Ga / mphi;
    const double s = 2 * P.mn[j] * E / m2;   // gamma_k's sp / sm
    if (need & kGeLs) v.ls = li2_t<kRef>(-s);
    if (need & kGeL1s) v.l1s = li2_t<kRef>(-1 - s);
    if (need & kGeCz) {
        const cd z = C(0.0, 1 + s) / C(gr, 2.0);
        v.cz = cli2_t<kRef>(z);
        if (!kRef) v.czc = cli2_t<kRef>(conj(z));
    }
}
// the edge values gamma_k<kRef, kPart> reads for bin (Em, Ep): the middle branches of its differences
template <int kPart>
NUSI_FN unsigned gamma_edge_need(const Point& P, int j, double Em, double Ep)
{
    if (!P.non_resonant) return 0;
    const double mphi = P.mphi, Ga = P.Ga, m2 = mphi * mphi, gr = Ga / mphi, mj = P.mn[j];
    const double sp = 2 * mj * Ep / m2, sm = 2 * mj * Em / m2;
    unsigned m = dilogdiff_mid(sp, sm) ? kGeLs : 0u;   // Gint and Gst
    if (kPart != 1 && dilog1mdiff_mid(sp, sm)) m |= kGeL1s;
    if (kPart != 0 && !(sp < 1e-5)) {
        const cd den = C(gr, 2.0);
        if (dilogdiff_c_mid(C(0.0, 1 + sp) / den, C(0.0, 1 + sm) / den)) m |= kGeCz;
    }
    return m;
}
template <bool kRef, int kPart, class Sink>   // kRef: NUSI_OPT_REFERENCE_ORDER (GSL's dilogarithms, nusi_gsl.hpp)
NUSI_FN void gamma_k(const Point& P, int j, double Em, double Ep, Sink& tot, int& warn, const GammaEdgePair* ge = nullptr)
{
    const double g = P.g, mphi = P.mphi, Ga = P.Ga;
    const double g4 = (g * g) * (g * g), m2 = mphi * mphi;
    const double gr = Ga / mphi, gr2 = gr * gr;
    {
        const double mj = P.mn[j], uj = P.u[j];
        const double sp = 2 * mj * Ep / m2, sm = 2 * mj * Em / m2;
        const double cs = m2 / (m2 + Ga * Ga);
        const double lg = Ga * (nm::log1p(cs * sp * (sp - 2)) - nm::log1p(cs * sm * (sm - 2)));
        const double wgt = m2 / (2 * mj);
        double Gs = 0, Gtu0 = 0, Gint = 0, Gst = 0, Gsu = 0;
        if (kPart != 1) {
            if (sp < 1e-5)
                Gs = g4 / (32 * kPi * m2 * Ga) *
                     (2 * mphi * ((gr * (1 + gr2 + 2 * sm)) / ((1 + gr2) * (1 + gr2)) * (sp - sm) + gr / ((1 + gr2) * (1 + gr2)) * ((sp - sm) * (sp - sm))) + lg);
            else
                Gs = g4 / (32 * kPi * m2 * Ga) * (2 * mphi * atandiff(mphi * (sp - 1) / Ga, mphi * (sm - 1) / Ga) + lg);
            Gs *= uj;
            tot.put(0, wgt * Gs, Gs);
        }
        if (!P.non_resonant) return;

        const double L1p = nm::log1p(sp), L1m = nm::log1p(sm);
        if (kPart != 1) {
            Gtu0 = g4 / (16 * kPi * m2) * (2 * L1p / sp - 2 * L1m / sm + L1p - L1m);
            if (Gtu0 < 0) Gtu0 = g4 / (16 * kPi * m2) * (sp - sm) / 2. * gl3_Gtu_nores(sm, sp);
            Gtu0 *= 2 * uj;
            tot.put(1, wgt * Gtu0, Gtu0);

            Gint = g4 / (32 * kPi * m2 * sm * sp) *
                   (sm * L1p * (2 + 2 * sp + sp * nm::log(2 + sp)) - sp * L1m * (2 + 2 * sm + sm * nm::log(2 + sm))
                    + sm * sp * (ge ? dilog1mdiff_pre(sp, sm, ge->hi.l1s, ge->lo.l1s) + dilogdiff_pre(sp, sm, ge->hi.ls, ge->lo.ls)
                                    : dilog1mdiff<kRef>(sp, sm) + dilogdiff<kRef>(sp, sm)));
            if (Gint < 0) Gint = g4 / (16 * kPi * m2) * (sp - sm) / 2. * gl3_Gtu_int(sm, sp);
            Gint *= P.majorana ? uj : 0.5 * uj;
            tot.put(2, wgt * Gint, Gint);
        }

        if (kPart != 0) {   // s-t interference
        const cd den = C(gr, 2.0);                    // 2*I + gr
        const cd z1p = C(0.0, 1 + sp) / den, z1m = C(0.0, 1 + sm) / den;
        const cd z2p = conj(z1p), z2m = conj(z1m);
        cd d1, d2;
        if (sp < 1e-5) {
            const cd l1 = clog(C(gr, 1.0) / den), l2 = clog(C(gr, -1.0) / C(gr, -2.0));
            d1 = (sm * sm) * (C(-0.0, -0.5) / C(gr, 1.0) - l1 / 2.) + sm * l1 - sp * l1 + ((sp * sp) * (kI / C(gr, 1.0) + l1)) / 2.;
            d2 = (sm * sm) * (C(0.0, 0.5) / C(gr, -1.0) - l2 / 2.) + sm * l2 - sp * l2 + ((sp * sp) * (C(-0.0, -1.0) / C(gr, -1.0) + l2)) / 2.;
        } else {
            d1 = ge ? dilogdiff_c_pre(z1p, z1m, ge->hi.cz, ge->lo.cz) : dilogdiff_c<kRef>(z1p, z1m);
            // (kRef) GSL's complex dilogarithm is odd in y operation by operation (every y-dependent quantity is
            // negated exactly, atan2 and Clausen are odd, the series' rotation and sums negate, the modulus terms do
            // not change), and so is li2_asym: Li2(conj z) = conj Li2(z) bit for bit, and d2 = conj(d1) is the
            // reference's own value at half the cost (the tables stay bit-identical to the oracle, which calls both)
            d2 = kRef ? conj(d1) : ge ? dilogdiff_c_pre(z2p, z2m, ge->hi.czc, ge->lo.czc) : dilogdiff_c<kRef>(z2p, z2m);
        }
        const double Lgp = nm::log1p(((-1 + sp) * (-1 + sp)) / gr2), Lgm = nm::log1p(((-1 + sm) * (-1 + sm)) / gr2);
        Gst = -g4 / (32 * kPi * m2 * (1 + gr2)) *
              (d1.r + d2.r + gr * (d2.i - d1.i) + 2 * gr * carg(1.0 - z2p) * L1p - 2 * gr * carg(1.0 - z2m) * L1m
               + nm::log1p(4 / gr2) * (L1m - L1p) + Lgp * L1p - Lgm * L1m + (1 + gr2) * (Lgm - Lgp)
               + 2 * (ge ? dilogdiff_pre(sp, sm, ge->hi.ls, ge->lo.ls) : dilogdiff<kRef>(sp, sm)));
        Gst *= uj;
        tot.put(3, wgt * Gst, Gst);
        Gsu = P.majorana ? Gst : 0;
        tot.put(4, wgt * Gsu, Gsu);
        }

        if (kPart != 1) {
            double Gpp = 0;
            if (sp > 4 && P.phiphi) {
                const double a = (sm > 4) ? sm : 4.0;
                Gpp = g4 / (128. * kPi * m2) * gpp_analytic<kRef>(a, sp);
                if (Gpp < 0) Gpp = g4 / (64 * kPi * m2) * (sp - a) / 2. * gl3_Gpp(a, sp);
                Gpp *= uj;
                if (P.majorana) Gpp *= 2;
            }
            tot.put(5, wgt * Gpp, Gpp);
        }
        if (kPart == -1) warn |= gamma_warn(Gs, Gtu0, Gint, Gst, Gsu);
    }
}
template <bool kRef = false>
NUSI_FN double gamma_entry(const Point& P, double Em, double Ep, int& warn)
{
    SumSink tot;
    NUSI_MASS_LOOP
    for (int j = 0; j < 3; ++j) gamma_k<kRef, -1>(P, j, Em, Ep, tot, warn);
    return tot.tot;
}

// ---------------------------------------------------------------------------
// alphaTilde(Em, Ep)  -- nuSIprop.hpp:924-1235
// ---------------------------------------------------------------------------
// alphaTilde's dilogarithms of one bin edge (t = -2 m_k E / m_phi^2 with alphat_k's |t + 1| < 1e-7 nudge): Li2 of
// 1 - t (real axis) and of i (1 - t) / (gr + 2 i), li2(1 / (1 - t)) and li2(1 + t) (k_gamma_alphat's edge-shared path)
struct AlphatEdgeVals { cd e78, e51; double e1o, e1p; };
struct AlphatEdgePair { AlphatEdgeVals lo, hi; };
constexpr unsigned kAe78 = 1, kAe51 = 2, kAe1o = 4, kAe1p = 8;
NUSI_FN double alphat_t(double mk, double E, double m2)
{
    double t = -2 * mk * E / m2;
    if (fabs(t + 1) < 1e-7) t += t * 1e-6;
    return t;
}
template <bool kRef>
NUSI_FN void alphat_edge_vals(const Point& P, int k, double E, unsigned need, AlphatEdgeVals& v)
{
    const double mphi = P.mphi, Ga = P.Ga, m2 = mphi * mphi, gr = Ga / mphi;
    const double t = alphat_t(P.mn[k], E, m2);
    if (need & kAe78) v.e78 = cli2_t<kRef>(C(1 - t));
    if (need & kAe51) v.e51 = cli2_t<kRef>(C(0.0, 1 - t) / C(gr, 2.0));
    if (need & kAe1o) v.e1o = li2_t<kRef>(1 / (1 - t));
    if (need & kAe1p) v.e1p = li2_t<kRef>(1 + t);
}
template <int kPart>
NUSI_FN unsigned alphat_edge_need(const Point& P, int k, double Em, double Ep)
{
    if (!P.non_resonant) return 0;
    const double mphi = P.mphi, Ga = P.Ga, m2 = mphi * mphi, gr = Ga / mphi;
    const double tp = alphat_t(P.mn[k], Ep, m2), tm = alphat_t(P.mn[k], Em, m2);
    unsigned m = 0;
    if (kPart != 1 && P.majorana) {
        if (dilog1over1mdiff_mid(tp, tm)) m |= kAe1o;
        if (dilog1pdiff_mid(tm, tp)) m |= kAe1p;
    }
    if (kPart != 0 && !(-tp < 1e-5)) {
        const cd den = C(gr, 2.0);
        if (dilogdiff_c_mid(C(1 - tm), C(1 - tp))) m |= kAe78;
        if (dilogdiff_c_mid(C(0.0, 1 - tp) / den, C(0.0, 1 - tm) / den)) m |= kAe51;
    }
    return m;
}
// alphaTilde's dilogarithms of one bin that are not edge values: the s-t interference's d26 = Li2(z2) - Li2(z6) and
// d43 = Li2(z4) - Li2(z3) (their four gsl_sf_complex_dilog_xy_e values) and the t-u combination's four gsl_sf_dilog
// values (k_ga_dilogs evaluates them one per work-item for calls of few tables)
struct AlphatBinVals { cd d26a, d26b, d43a, d43b; double c1, c2, c3, c4; };
template <bool kRef, int kPart, class Sink>   // kRef: NUSI_OPT_REFERENCE_ORDER (GSL's dilogarithms, nusi_gsl.hpp)
NUSI_FN void alphat_k(const Point& P, const SplineSet& spl, int k, double Em, double Ep, Sink& tot, int& warn,
                      const AlphatEdgePair* ae = nullptr, const AlphatBinVals* bv = nullptr)
{
    const double g = P.g, mphi = P.mphi, Ga = P.Ga;
    const double g4 = (g * g) * (g * g), m2 = mphi * mphi, m4 = (mphi * mphi) * (mphi * mphi);
    const double gr = Ga / mphi, gr2 = gr * gr;
    const bool maj = P.majorana;
    {
        const double mk = P.mn[k], uk = P.u[k];
        double tp = -2 * mk * Ep / m2, tm = -2 * mk * Em / m2;
        if (fabs(tm + 1) < 1e-7) tm += tm * 1e-6;
        if (fabs(tp + 1) < 1e-7) tp += tp * 1e-6;
        const double wgt = m4 / (2 * mk);

        const double cs = m2 / (m2 + Ga * Ga);
        const double lg = Ga * (nm::log1p(cs * tp * (tp + 2)) - nm::log1p(cs * tm * (tm + 2)));
        double as = 0, at = 0, au = 0, atu = 0, ast = 0, asu = 0;
        if (kPart != 1) {
            if (fabs(tp) < 1e-5)
                as = g4 / (16 * kPi * Ga * m4) *
                     (2 * mphi * (1 + tm) * (-((gr * (1 + gr2 - 2 * tm) * (-tm + tp)) / ((1 + gr2) * (1 + gr2))) + (gr * ((-tm + tp) * (-tm + tp))) / ((1 + gr2) * (1 + gr2))) + lg);
            else
                as = g4 / (16 * kPi * Ga * m4) * (2 * mphi * (1 + tm) * atandiff(mphi * (1 + tm) / Ga, mphi * (1 + tp) / Ga) + lg);
            as *= uk;
            if (!maj) as /= 2.;
            tot.put(0, wgt * as, as);
        }
        if (!P.non_resonant) return;

        const double Lmt = nm::log1p(-tm), Lmp = nm::log1p(-tp), Ld = nm::log1p(tm - tp);
        const double brk = (-2 + tm) * (tm - tp) - (-1 + tm) * (-2 + tp) * (Lmt - Lmp);
        if (kPart != 1) {
        if (maj) {
            at = g4 * (1 / (16 * m4 * kPi * (-1 + tm) * tp) * brk
                       + 1 / (16 * m4 * kPi * ((1 + tm) * (1 + tm)) * tp) *
                             ((1 + tm) * (2 + tm) * (tm - tp) + (-2 * ((1 + tm) * (1 + tm)) + tp + 2 * tm * tp) * Ld - (tm * tm) * tp * nm::log(tm / tp)));
            if (at < 0) at = gl33_tri(0, tp, tm) * (g4 / (16 * kPi * m4));
        } else {
            at = 3. / 2. * g4 / (32 * m4 * kPi * (-1 + tm) * tp) * brk;
            if (at < 0) at = gl33_tri(1, tp, tm) * (3. / 2. * g4 / (32 * kPi * m4));
        }
        at *= uk;
        tot.put(1, wgt * at, at);

        if (maj) au = at;
        else {
            au = 1. / 2. * g4 / (32 * m4 * kPi * (-1 + tm) * tp) * brk;
            if (au < 0) au = gl33_tri(1, tp, tm) * (1. / 2. * g4 / (32 * kPi * m4));
            au *= uk;
        }
        tot.put(2, wgt * au, au);

        if (maj) {
            double combi;
            if (-tp < 1e-2 && -tm < 1e-2) {
                // log(2), log(256), log(4096) as the reference's libm calls return them
                const double d = tp / tm, lt = nm::log(-tp);
                const double ln2 = 0.6931471805599453, ln256 = 5.545177444479562, ln4096 = 8.317766166719343;
                const double d2 = d * d, d3 = d * d * d, d4 = (d * d) * (d * d);
                combi = -(((-1 + d) * tp * nm::log(-2 * tp)) / d)
                        - ((-1 + d) * (tp * tp) * (-2 + d + d * ln2 + nm::log(-2 / tp) - d * lt)) / (2. * d2)
                        + ((tp * tp * tp) * (8 - 30 * d + 21 * d2 + d3 - 8 * d3 * ln2 + ln256 + 8 * lt - 8 * d3 * lt)) / (24. * d3)
                        + (((tp * tp) * (tp * tp)) * (-32 + 56 * d - 51 * d2 + 30 * d3 - 3 * d4 + ln4096 - d4 * ln4096 - 12 * lt + 12 * d4 * lt)) / (48. * d4);
            } else if (-tp > 1e2 && -tm > 1e2) {
                const double d = tp / tm, lq = nm::log((-1 + d) / d), lt = nm::log(-tp);
                const double d2 = d * d, d3 = d * d * d, d4 = (d * d) * (d * d);
                combi = (-2 * (-1 + d) * lq) / tp - (2 * (-1 + nm::log(-(d / ((-1 + d) * tp))))) / (tp * tp)
                        + (-6 + 4 * d + d2 - 2 * d3 - 8 * lq + 8 * d * lq + 2 * d3 * lq - 2 * d4 * lq - 6 * lt + 6 * d * lt) / (3. * (-1 + d) * (tp * tp * tp))
                        + (8 - 12 * d + 3 * d2 + 12 * lq - 24 * d * lq + 12 * d2 * lq + 12 * lt - 24 * d * lt + 12 * d2 * lt) / (3. * ((-1 + d) * (-1 + d)) * ((tp * tp) * (tp * tp)));
            } else if (bv)
                combi = bv->c1 - bv->c2 + bv->c3 - bv->c4;   // (the same four values, the same left-to-right sum)
            else
                combi = li2_t<kRef>(1 + 1 / (-2 + tp)) - li2_t<kRef>((-1 + tm) / (-2 + tp)) + li2_t<kRef>(1 + (1 + tm - tp) / tp) - li2_t<kRef>(1 + 1 / tp);
            atu = g4 / (32 * kPi * m4 * (1 + tm) * tp) *
                  (2 * (2 * (1 + tm) * (tm - tp) - 2 * (1 + tm) * tp * nm::atanh(1 / (1 - tp)) * nm::atanh((tm - tp) / (-2 + tm + tp))
                        + tm * tp * (-Lmt + Lmp) + (1 + tm) * (Lmt - Lmp - Ld) + tp * (-Lmt + Lmp + Ld) - tm * tp * nm::log(tm / tp))
                   + (1 + tm) * tp * ((-(Lmt * Lmt) + Lmp * Lmp) / 2.
                                      + (ae ? dilog1over1mdiff_pre(tp, tm, ae->hi.e1o, ae->lo.e1o) : dilog1over1mdiff<kRef>(tp, tm)))
                   - (1 + tm) * tp * ((ae ? dilog1pdiff_pre(tm, tp, ae->lo.e1p, ae->hi.e1p) : dilog1pdiff<kRef>(tm, tp)) + combi));
            if (atu < 0) atu = gl33_tri(2, tp, tm) * (g4 / (16 * kPi * m4));
        }
        atu *= uk;
        tot.put(3, wgt * atu, atu);
        }

        if (kPart != 0) {   // s-t interference
        const cd den = C(gr, 2.0);                  // 2*I + gr
        const cd dt_m = C(2 + tm, -gr);             // 2 - I*gr + tm
        cd d78, d51, d26, d43;
        if (-tp < 1e-5) {
            const double d = tp / tm;
            const cd ltm = clog_real(tm), ltp = clog_real(tp), ld = clog_real(d);
            const cd lq = clog(1.0 - kI / den), lr = clog(C(gr, 1.0) / den);
            d78 = tm * (-1.0 + ltm) + ((tm * tm) * (-1.0 + 2 * ltm)) / 4. - (tp * (-1.0 + ltp) + ((tp * tp) * (-1.0 + 2 * ltp)) / 4.);
            d51 = (-tm + tp) * lq + ((-(tm * tm) + tp * tp) * (kI * (1.0 + lq) + lq * gr)) / (2. * C(gr, 1.0));
            d26 = (tp * (-1.0 + d - ld + ltp - d * ltp)) / d
                  + ((tp * tp) * (-1.0 + d * d + 2 * ld - 2 * ltp + 4 * d * ltp - 2 * (d * d) * ltp)) / (4. * (d * d))
                  + ((tp * tp * tp) * (7 - 9 * d + 2 * (d * d * d) - 6 * ld + 6 * ltp - 18 * d * ltp + 18 * (d * d) * ltp - 6 * (d * d * d) * ltp)) / (18. * (d * d * d));
            d43 = ((-1 + d) * tp * lr) / d + ((-1 + d) * (tp * tp) * (kI * ((1 + d) / C(gr, 1.0) - 2 / den) + (-1 + d) * lr)) / (2. * (d * d));
        } else {
            const cd z1 = C(0.0, 1 - tm) / den;      // (-I*(-1+tm))/(2I+gr)
            const double z2 = 1 / (1 + tm);
            const cd z3 = 1 / dt_m;
            const cd z4 = (1 + tm - tp) / dt_m;
            const cd z5 = C(0.0, 1 - tp) / den;
            const double z6 = 1 - tp / (1 + tm);
            d78 = ae ? dilogdiff_c_pre(C(1 - tm), C(1 - tp), ae->lo.e78, ae->hi.e78) : dilogdiff_c<kRef>(C(1 - tm), C(1 - tp));
            d51 = ae ? dilogdiff_c_pre(z5, z1, ae->hi.e51, ae->lo.e51) : dilogdiff_c<kRef>(z5, z1);
            d26 = bv ? dilogdiff_c_pre(C(z2), C(z6), bv->d26a, bv->d26b) : dilogdiff_c<kRef>(C(z2), C(z6));
            d43 = bv ? dilogdiff_c_pre(z4, z3, bv->d43a, bv->d43b) : dilogdiff_c<kRef>(z4, z3);
        }
        const double Lgp = nm::log1p(((1 + tp) * (1 + tp)) / gr2), Lgm = nm::log1p(((1 + tm) * (1 + tm)) / gr2);
        const double Am = carg(C(-1 - tm, gr)), Ap = carg(C(-1 - tp, gr));
        const double Bm = carg(C(gr, 1 + tm) / den), Bp = carg(C(gr, 1 + tp) / den);
        if (maj)
            ast = g4 / (32 * kPi * (1 + gr2) * m4) *
                  (2 * kPi * Am - 2 * kPi * Ap + 2 * gr * (d51.i + d26.i + d43.i) - 2 * (d51.r + d26.r + d43.r + d78.r)
                   - Bm * (2 * kPi + 2 * gr * Lmt) + Bp * (2 * kPi + 2 * gr * Lmp) + (Am - Ap) * (4 * gr * tm + 2 * gr * Lmt)
                   + 2 * gr * (carg_real(1 + tm) - carg(dt_m) + carg(C(1 + tp, -gr))) * Ld
                   + nm::log(4 + gr2) * (Lmp - Lmt) + nm::log(gr2 + (2 + tm) * (2 + tm)) * Ld - 2 * Lmt * nm::log(-tp)
                   - 2 * gr * kPi * (nm::log(tp * tp) + Ld) + 2 * gr * kPi * nm::log(tp * tp) + 4 * tm * nm::log(tm / tp)
                   + (-Lmp + Lmt - Ld) * (Lgp + 2 * nm::log(gr)) - Ld * nm::log1p(tm * tm + 2 * tm)
                   + 2 * (gr2 + tm) * (Lgp - Lgm) + 2 * (nm::log(-tp) * (Lmp + Ld) + (Lgp - Lgm)));
        else
            ast = g4 / (32 * kPi * (1 + gr2) * m4) *
                  (gr * d51.i - 2 * (d51.r + d78.r) + 2 * Bm * (-kPi - gr * Lmt) + 2 * Am * (kPi + gr * tm + gr * Lmt)
                   - 2 * Ap * (kPi + gr * tm + gr * Lmt) + 2 * Bp * (kPi + gr * Lmp) - 2 * Lmt * nm::log(-tp)
                   + 2 * tm * nm::log(tm / tp) + 2 * Lmp * nm::log(-tp) + (Lmp - Lmt) * (nm::log(4 + gr2) - 2 * nm::log(gr) - Lgp)
                   + (1 + tm + gr2) * (Lgp - Lgm));
        ast *= uk;
        tot.put(4, wgt * ast, ast);
        asu = maj ? ast : 0;
        tot.put(5, wgt * asu, asu);
        }

        if (kPart != 1) {
        double app = 0;
        if (-tp > 4 && P.phiphi) {
            if (-tp < 1e4) {
                const double xx[2] = {-tp, nm::log10(tp / tm)};
                double v = 0;
                if (!spl.at.eval<2>(xx, v)) warn |= kWarnSplineOOB;
                app = g4 / m4 * v;
            } else {
                const double lm = nm::log(-tm), lp = nm::log(-tp);
                app = g4 / m4 *
                      (6 * tm * lm - tp * (lm * lm) + 2 * (-8 * tm + 8 * tp + 4 * tp * lm + nm::log(tm - tp) * (tm - tp - tp * nm::log(tm / tp)))
                       - 2 * (2 * tm + 5 * tp) * lp + tp * (lp * lp) - 2 * tp * li2_t<kRef>(1 - tm / tp)) / (128. * kPi * tp);
            }
            app *= uk;
            if (maj) app *= 2;
            app *= 2;
            if (maj) app *= 2;
        }
        tot.put(6, wgt * app, app);
        }

        if (kPart == -1) warn |= alphat_warn(as, at, au, atu, ast, asu, P.a_nrm);
    }
}
template <bool kRef = false>
NUSI_FN double alphat_entry(const Point& P, const SplineSet& spl, double Em, double Ep, int& warn)
{
    SumSink tot;
    NUSI_MASS_LOOP
    for (int k = 0; k < 3; ++k) alphat_k<kRef, -1>(P, spl, k, Em, Ep, tot, warn);
    return tot.tot;
}

// Calls of few tables in the reference order (k_ga_dilogs): every GSL dilogarithm Gamma and alphaTilde read for
// (point, mass state k, bin [Em, Ep]) -- the edge values at both edges (gamma_edge_vals, alphat_edge_vals) and
// alphaTilde's bin values (AlphatBinVals) -- one slot per work-item, the same functions on the same arguments as
// gamma_k / alphat_k would call them (so the same bits), into kGaPreFields fields per (point, k, bin):
//   0 ls, 1 l1s, 2-3 cz at Em | 4 ls, 5 l1s, 6-7 cz at Ep | 8-9 e78, 10-11 e51, 12 e1o, 13 e1p at Em | 14-19 at Ep |
//   20-21 d26a, 22-23 d26b, 24-25 d43a, 26-27 d43b, 28-31 c1 .. c4
// Values no branch of the bin reads are evaluated too (and not read).  v[0], v[1] at field *f (v[1]: complex only);
// returns the count.
constexpr int kGaPreSlots = 22, kGaPreFields = 32;
NUSI_FN int ga_pre_slot(const Point& P, int k, double Em, double Ep, int slot, double* v, int* f)
{
    if (slot < 6) {   // Gamma's edge values (reference order: no conj z value)
        const int side = slot / 3, which = slot - 3 * side;
        GammaEdgeVals e{};
        gamma_edge_vals<true>(P, k, side ? Ep : Em, which == 0 ? kGeLs : which == 1 ? kGeL1s : kGeCz, e);
        *f = 4 * side + which;
        if (which == 0) { v[0] = e.ls; return 1; }
        if (which == 1) { v[0] = e.l1s; return 1; }
        v[0] = e.cz.r; v[1] = e.cz.i;
        return 2;
    }
    if (slot < 14) {   // alphaTilde's edge values
        const int side = (slot - 6) / 4, which = slot - 6 - 4 * side;
        AlphatEdgeVals e{};
        alphat_edge_vals<true>(P, k, side ? Ep : Em, which == 0 ? kAe78 : which == 1 ? kAe51 : which == 2 ? kAe1o : kAe1p, e);
        const int f0 = 8 + 6 * side;
        if (which == 0) { *f = f0; v[0] = e.e78.r; v[1] = e.e78.i; return 2; }
        if (which == 1) { *f = f0 + 2; v[0] = e.e51.r; v[1] = e.e51.i; return 2; }
        *f = f0 + 2 + which;
        v[0] = which == 2 ? e.e1o : e.e1p;
        return 1;
    }
    // alphaTilde's bin values: tm, tp, z2 .. z6 and the combination's arguments as alphat_k forms them
    const double mphi = P.mphi, Ga = P.Ga, m2 = mphi * mphi, gr = Ga / mphi, mk = P.mn[k];
    double tp = -2 * mk * Ep / m2, tm = -2 * mk * Em / m2;
    if (fabs(tm + 1) < 1e-7) tm += tm * 1e-6;
    if (fabs(tp + 1) < 1e-7) tp += tp * 1e-6;
    const int b = slot - 14;
    if (b < 4) {
        const cd dt_m = C(2 + tm, -gr);
        cd z;
        if (b == 0) z = C(1 / (1 + tm));
        else if (b == 1) z = C(1 - tp / (1 + tm));
        else if (b == 2) z = (1 + tm - tp) / dt_m;
        else z = 1 / dt_m;
        const cd d = cli2_t<true>(z);
        *f = 20 + 2 * b;
        v[0] = d.r; v[1] = d.i;
        return 2;
    }
    const double x = b == 4 ? 1 + 1 / (-2 + tp) : b == 5 ? (-1 + tm) / (-2 + tp) : b == 6 ? 1 + (1 + tm - tp) / tp : 1 + 1 / tp;
    *f = 28 + (b - 4);
    v[0] = li2_t<true>(x);
    return 1;
}
// the fields of (point, k, bin n) -> the pairs and bin values gamma_k / alphat_k take (fb: field 0 of (point, k),
// fields T doubles apart)
NUSI_FN void ga_pre_load(const double* fb, int T, int n, GammaEdgePair& ge, AlphatEdgePair& ae, AlphatBinVals& bv)
{
    const double* x = fb + n;
    auto F = [&](int i) { return x[(size_t)i * T]; };
    ge.lo.ls = F(0); ge.lo.l1s = F(1); ge.lo.cz = C(F(2), F(3));
    ge.hi.ls = F(4); ge.hi.l1s = F(5); ge.hi.cz = C(F(6), F(7));
    ae.lo.e78 = C(F(8), F(9)); ae.lo.e51 = C(F(10), F(11)); ae.lo.e1o = F(12); ae.lo.e1p = F(13);
    ae.hi.e78 = C(F(14), F(15)); ae.hi.e51 = C(F(16), F(17)); ae.hi.e1o = F(18); ae.hi.e1p = F(19);
    bv.d26a = C(F(20), F(21)); bv.d26b = C(F(22), F(23)); bv.d43a = C(F(24), F(25)); bv.d43b = C(F(26), F(27));
    bv.c1 = F(28); bv.c2 = F(29); bv.c3 = F(30); bv.c4 = F(31);
}

// ---------------------------------------------------------------------------
// alpha(Em, Ep, Em', Ep')  -- nuSIprop.hpp:1237-1520
//
// The entry for bins n (t edges tm, tp) and m (S' edges Sm, Sp) is a fixed
// combination of transcendental "leaves" that depend on ONE edge or on ONE
// (S' edge, t edge) corner only.  Neighbouring bins share edges, so the tile
// kernel (k_alpha_tile) evaluates each leaf once per edge / corner and the
// entries of a tile combine them; the per-entry path evaluates them inline.
// Both go through alpha_k<Leaves>() -- one expression text -- and the leaves
// are pure functions of the same fp64 arguments, so the two paths (and the
// oracle, which computes them inline in the reference's order) agree bit for
// bit.
// ---------------------------------------------------------------------------
NUSI_FN double alpha_t(double mk, double E, double m2)   // :1262-1266, incl. the |t+1| < 1e-7 nudge
{
    double t = -2 * mk * E / m2;
    if (fabs(t + 1) < 1e-7) t += t * 1e-6;
    return t;
}
NUSI_FN double alpha_S(double mk, double E, double m2) { return 2 * mk * E / m2; }   // :1263-1264

// corner (S', t) leaves
struct AlphaCorner {
    double L;          // log1p(S + t)
    double LL;         // log(1 + S + t)
    double TU1, TU2;   // t < -1: li2((1+S+t)/S), 0 ; else li2(S/(1+S+t)), log((1+S+t)/S)   (:1375-1398)
    double G;          // li2((1+S+t)/(2+S))
    double Drr, Dri;   // cli2((1+S+t)/(1+t) + 0i)                                          (:1444-1451)
    double Dcr, Dci;   // cli2((1+S+t)/(2 - i gr + t))
    double A;          // arg(-(-1 + i gr + S)/(2 - i gr + t))
};
// the corner leaves' own elementary functions: inline by default (-DNUSI_CORNER_CALL_LIBM: calls)
#ifdef NUSI_CORNER_CALL_LIBM
#define NUSI_CLOG nm::log
#define NUSI_CLOG1P nm::log1p
#define NUSI_CARG carg
#else
#define NUSI_CLOG nm::log_i
#define NUSI_CLOG1P nm::log1p_i
#define NUSI_CARG carg_i
#endif
// The leaves split into those of (S', t) alone ("shared": every point with the same m_phi and
// masses has them, bit for bit) and those that also read gr = Gamma_phi / m_phi ("member").  kRef:
// NUSI_OPT_REFERENCE_ORDER (GSL's dilogarithms)
template <bool kRef = false>
NUSI_FN void alpha_corner_shared(double S, double t, AlphaCorner& c)
{
    c.L = NUSI_CLOG1P(S + t);
    c.LL = NUSI_CLOG(1 + S + t);
    if (t < -1) {
        c.TU1 = li2_t<kRef>((1 + S + t) / S);
        c.TU2 = 0.0;
    } else {
        c.TU1 = li2_t<kRef>(S / (1 + S + t));
        c.TU2 = NUSI_CLOG((1 + S + t) / S);
    }
    c.G = li2_t<kRef>((1 + S + t) / (2 + S));
    const cd Dr = cli2_real_t<kRef>((1 + S + t) / (1 + t));
    c.Drr = Dr.r;
    c.Dri = Dr.i;
}
// The member leaves of the s-t interference (nuSIprop.hpp:1444-1451, 1456-1459), dt = 2 + t - i gr:
//   Dc = Li2(w), w = (1 + S + t) / dt = a (c + i gr) / (c^2 + gr^2), a = 1 + S + t, c = 2 + t;
//   A  = arg(-(-1 + i gr + S) / dt) = arg(S - 1 + i gr) + arg(c + i gr) - pi   (both arguments lie in
//        (0, pi), and Im(-(S - 1 + i gr)(c + i gr)) = -gr a < 0 puts A in (-pi, 0): no wrap).
// w lies within gr / |c| (relative) of the real point x0 = a / c, which does not depend on gr: the Taylor
// coefficients of Li2 about x0 are formed once per corner for every point of a batch (alpha_member_shared),
// and a point only evaluates them at d = w - x0 = i (gr / c) w (li2_taylor_eval); a w outside the
// expansion's radius takes the general cli2.  Each argument is written as f pi + s with s the small angle
// where the argument is near 0 or pi (edge leaves), so A = (sS + sT) + (fS + fT - 1) pi keeps full
// relative accuracy where it is small.  The oracle forms them the same way (nusi_oracle.c member_*).
struct MemberShared {
    Li2Taylor T;
    double m;   // kLi2AxisRatio min(|x0|, |1 - x0|): the radius used (0: no expansion)
};
NUSI_FN void alpha_member_shared(double S, double t, MemberShared& M)
{
    const double a = 1 + S + t, c = 2 + t;
    const double x0 = a / c;
    const double ax = fabs(x0), a1 = fabs(1.0 - x0);
    if (c != 0.0 && a1 > 0.0 && ax < 1e300) {
        li2_taylor_coeffs(x0, M.T);
        M.m = kLi2AxisRatio * (ax < a1 ? ax : a1);
    } else {
        for (int n = 0; n <= kLi2AxisTerms; ++n) M.T.c[n] = 0.0;
        M.T.r = M.T.b0 = 0.0;
        M.m = 0.0;
    }
}
// member t-edge leaves of coupling gr: inv = 1 / (c^2 + gr^2), q = gr / c, arg(c + i gr) = fT pi + sT
struct MemberTEdge { double inv, q, sT, fT; };
NUSI_FN MemberTEdge alpha_member_tedge(double t, double gr)
{
    const double c = 2 + t;
    MemberTEdge e;
    e.inv = 1.0 / (c * c + gr * gr);
    e.q = gr / c;
    if (c < 0.0) { e.sT = -nm::atan2_i(gr, -c); e.fT = 1.0; }
    else { e.sT = nm::atan2_i(gr, c); e.fT = 0.0; }
    return e;
}
// member S'-edge leaves: arg(S - 1 + i gr) = fS pi + sS
NUSI_FN void alpha_member_sarg(double S, double gr, double& sS, double& fS)
{
    if (S < 1.0) { sS = -nm::atan2_i(gr, 1.0 - S); fS = 1.0; }
    else { sS = nm::atan2_i(gr, S - 1.0); fS = 0.0; }
}
// Dc and A of corner (S, t) for coupling gr from the shared coefficients and the edge leaves
NUSI_FN void alpha_member_corner(const MemberShared& M, double S, double t, double gr, const MemberTEdge& e, double sS,
                                 double fS, double& Dcr, double& Dci, double& A)
{
    const double a = 1 + S + t, c = 2 + t;
    const double wr = (a * c) * e.inv, wi = (a * gr) * e.inv;
    const double dr = -(e.q * wi), di = e.q * wr;
    const cd Dc = (dr * dr + di * di <= M.m * M.m) ? li2_taylor_eval(M.T, dr, di, 1.0) : cli2(wr, wi);
    Dcr = Dc.r;
    Dci = Dc.i;
    A = (sS + e.sT) + (fS + e.fT - 1.0) * kPi;
}
// NUSI_OPT_REFERENCE_ORDER: the member leaves in the reference's own operation order -- Dc =
// gsl_sf_complex_dilog_xy_e of its quotient z = (1 + S + t) / (2 - i gr + t) (C99 complex division,
// nuSIprop.hpp:1432-1438, 1444-1451), by GSL's algorithm (gsl_cli2), and A = carg(-((-1 + i gr + S) / (2 - i gr + t)))
// (:1456); no Taylor expansion about the real point and no sum of edge arguments.  The oracle's
// member_dc_ref / member_arg_ref (ora_set_reference_order(1)).
#ifndef NUSI_REFO_STUB   // timing A/B only: 1 = the member corners without the dilogarithm (Dc = z), 2 = nothing
#define NUSI_REFO_STUB 0
#endif
NUSI_FN cd alpha_member_ref_dc(double S, double t, double gr)
{
    const cd z = (1 + S + t) / C(2 + t, -gr);
    return NUSI_REFO_STUB == 1 ? z : gsl_cli2(z.r, z.i);
}
// the same, with GSL's call inline (k_alpha_mcorner's single call site)
NUSI_FN cd alpha_member_ref_dc_inl(double S, double t, double gr)
{
    const cd z = (1 + S + t) / C(2 + t, -gr);
    return NUSI_REFO_STUB == 1 ? z : gsl_cli2_inl(z.r, z.i);
}
NUSI_FN double alpha_member_ref_arg(double S, double t, double gr)
{
    return carg_i(-(C(-1 + S, gr) / C(2 + t, -gr)));   // (atan2 inline)
}
NUSI_FN void alpha_member_ref(double S, double t, double gr, double& Dcr, double& Dci, double& A)
{
    if (NUSI_REFO_STUB == 2) { Dcr = Dci = A = 0.0; return; }
    const cd Dc = alpha_member_ref_dc(S, t, gr);
    Dcr = Dc.r;
    Dci = Dc.i;
    A = alpha_member_ref_arg(S, t, gr);
}
template <bool kRef = false>
NUSI_FN void alpha_corner_member(double S, double t, double gr, AlphaCorner& c)
{
    if (kRef) {
        alpha_member_ref(S, t, gr, c.Dcr, c.Dci, c.A);
        return;
    }
    MemberShared M;
    alpha_member_shared(S, t, M);
    const MemberTEdge e = alpha_member_tedge(t, gr);
    double sS, fS;
    alpha_member_sarg(S, gr, sS, fS);
    alpha_member_corner(M, S, t, gr, e, sS, fS, c.Dcr, c.Dci, c.A);
}
template <bool kRef = false>
NUSI_FN void alpha_corner(double S, double t, double gr, AlphaCorner& c)
{
    alpha_corner_shared<kRef>(S, t, c);
    alpha_corner_member<kRef>(S, t, gr, c);
}
// t-edge leaves (L2 is the member leaf)
struct AlphaTEdge { double Lm1, la, cm, L2, am; };
NUSI_FN void alpha_tedge_shared(double t, AlphaTEdge& e)
{
    e.Lm1 = nm::log1p(-t);
    e.la = (t > -1) ? nm::log1p(t) : nm::log(-1 - t);
    e.cm = carg_real(-(1 / (1 + t)));
    e.am = nm::log(fabs(1 + t));
}
NUSI_FN double alpha_tedge_L2(double t, double gr2) { return nm::log1p(((2 + t) * (2 + t)) / gr2); }
NUSI_FN void alpha_tedge(double t, double gr2, AlphaTEdge& e)
{
    alpha_tedge_shared(t, e);
    e.L2 = alpha_tedge_L2(t, gr2);
}
// S'-edge leaves (Ls, cS are member leaves)
struct AlphaSEdge { double lS, l2, Ls, cS, lS2; };
NUSI_FN void alpha_sedge_shared(double S, AlphaSEdge& e)
{
    e.lS = nm::log(S);
    e.l2 = nm::log((2 + S) / S);
    e.lS2 = nm::log(S / (2 + S));
}
NUSI_FN void alpha_sedge_member(double S, double gr, double gr2, AlphaSEdge& e)
{
    e.Ls = nm::log1p(((-1 + S) * (-1 + S)) / gr2);
    e.cS = carg(C(-1 + S, gr));
}
NUSI_FN void alpha_sedge(double S, double gr, double gr2, AlphaSEdge& e)
{
    alpha_sedge_shared(S, e);
    alpha_sedge_member(S, gr, gr2, e);
}
// mixed leaves of the Majorana t channel (nuSIprop.hpp:1284): each of its four logarithms
// depends on one S' edge and the n bin (xlog) or on the m bin and one t edge (ylog)
NUSI_FN double alpha_xlog(double S, double tm, double tp) { return nm::log(((1 + S + tm) * (-1 + tp)) / ((-1 + tm) * (1 + S + tp))); }
NUSI_FN double alpha_ylog(double Sm, double Sp, double t) { return nm::log((Sm * (1 + Sp + t)) / (Sp * (1 + Sm + t))); }
// m-bin leaves
struct AlphaMBin { double lr, lr2, atd; };
NUSI_FN double alpha_mbin_atd(double Sm, double Sp, double mphi, double Ga)   // the member leaf
{
    return (Sp < 1e-5) ? 0.0 : atandiff(mphi * (Sp - 1) / Ga, mphi * (Sm - 1) / Ga);
}
NUSI_FN void alpha_mbin(double Sm, double Sp, double mphi, double Ga, AlphaMBin& b)
{
    b.lr = nm::log(Sm / Sp);
    b.lr2 = nm::log(Sp / Sm);
    b.atd = alpha_mbin_atd(Sm, Sp, mphi, Ga);
}

// shared edge-block fields: t edges Lm1 la cm am t, S' edges lS l2 lS2 S, m bins lr lr2
constexpr int kCornerFields = 10, kTEdgeFields = 5, kSEdgeFields = 4, kMBinFields = 2;
constexpr int kTEdgeVal = 4, kSEdgeVal = 3;   // edge field holding t resp. S' itself (alpha_t / alpha_S)

// leaves evaluated on the spot (per-entry path, host checks); kRef: NUSI_OPT_REFERENCE_ORDER
template <bool kRef = false>
struct DirectLeavesT {
    double gr, gr2, mphi, Ga;
    NUSI_FN double tval(int, double mk, double E, double m2) const { return alpha_t(mk, E, m2); }
    NUSI_FN double Sval(int, double mk, double E, double m2) const { return alpha_S(mk, E, m2); }
    NUSI_FN AlphaCorner corner(int, int, double S, double t) const { AlphaCorner c; alpha_corner<kRef>(S, t, gr, c); return c; }
    NUSI_FN AlphaTEdge tedge(int, double t) const { AlphaTEdge e; alpha_tedge(t, gr2, e); return e; }
    NUSI_FN AlphaSEdge sedge(int, double S) const { AlphaSEdge e; alpha_sedge(S, gr, gr2, e); return e; }
    NUSI_FN AlphaMBin mbin(double Sm, double Sp) const { AlphaMBin b; alpha_mbin(Sm, Sp, mphi, Ga, b); return b; }
    NUSI_FN double xlog(int, double S, double tm, double tp) const { return alpha_xlog(S, tm, tp); }
    NUSI_FN double ylog(int, double Sm, double Sp, double t) const { return alpha_ylog(Sm, Sp, t); }
};
using DirectLeaves = DirectLeavesT<false>;

// leaves read from a tile's precomputed arrays (structure of arrays):
//   cor[v * cc + s * ct + t]  (v = shared field of AlphaCorner, cc = cs * ct),
//   corm[v * cc + s * ct + t] (v = member field Dcr, Dci, A of this point),
//   ted[v * ct + t], sed[v * cs + s], mbv[v * kAlphaTile + j] (shared edge / m-bin fields),
//   tedm[t] = L2, sedm[s] = Ls, sedm[cs + s] = cS, mbm[j] = atd (this point's member fields),
//   xl[s * kAlphaTile + n bin], yl[m bin * ct + t]
#ifndef NUSI_ALPHA_TILE   // A/B: bins per alpha tile side (the edges of a core tile side are kAlphaTile + 1 <= 17)
#define NUSI_ALPHA_TILE 15
#endif
constexpr int kAlphaTile = NUSI_ALPHA_TILE;
constexpr int kCornerShared = 7, kCornerMember = 3;   // L LL TU1 TU2 G Drr Dri | Dcr Dci A
struct TileLeaves {
    const double *cor, *corm, *ted, *sed, *mbv, *tedm, *sedm, *mbm, *xl, *yl;
    int cc, ct, cs, mb, nb;
    int sidx[2], tidx[2];   // slots of (Sm, Sp) and (tm, tp)
    NUSI_FN AlphaCorner corner(int si, int ti, double, double) const
    {
        const int o = sidx[si] * ct + tidx[ti];
        const double *c = cor + o, *d = corm + o;
        return AlphaCorner{c[0], c[cc], c[2 * cc], c[3 * cc], c[4 * cc], c[5 * cc], c[6 * cc], d[0], d[cc], d[2 * cc]};
    }
    NUSI_FN AlphaTEdge tedge(int ti, double) const
    {
        const double* e = ted + tidx[ti];
        return AlphaTEdge{e[0], e[ct], e[2 * ct], tedm[tidx[ti]], e[3 * ct]};
    }
    NUSI_FN AlphaSEdge sedge(int si, double) const
    {
        const double* e = sed + sidx[si];
        return AlphaSEdge{e[0], e[cs], sedm[sidx[si]], sedm[cs + sidx[si]], e[2 * cs]};
    }
    NUSI_FN AlphaMBin mbin(double, double) const
    {
        return AlphaMBin{mbv[mb], mbv[kAlphaTile + mb], mbm[mb]};
    }
    NUSI_FN double tval(int ti, double, double, double) const { return ted[kTEdgeVal * ct + tidx[ti]]; }
    NUSI_FN double Sval(int si, double, double, double) const { return sed[kSEdgeVal * cs + sidx[si]]; }
    NUSI_FN double xlog(int si, double, double, double) const { return xl[sidx[si] * kAlphaTile + nb]; }
    NUSI_FN double ylog(int ti, double, double, double) const { return yl[mb * ct + tidx[ti]]; }
};
// per-k leaf block of the corner phase for G points: shared corners, G member corner blocks, then
// xlog [cs][kAlphaTile], then ylog [kAlphaTile][ct]
NUSI_FN int alpha_tile_corner_block(int cs, int ct, int G)
{
    return (kCornerShared + kCornerMember * G) * cs * ct + kAlphaTile * (cs + ct);
}

// Unique edge energies of bins b0 .. b0+kAlphaTile-1 (< T): E[0..count), il/ih = slot of each bin's
// lower/upper edge.  Bins of the first N share edges bitwise (Emax[n] == Emin[n+1], same pow()
// argument); the redshift-extended bins do not (nuSIprop.hpp:217-252).
NUSI_FN int alpha_edge_list(const double* lo, const double* hi, int b0, int T, double* E, int* il, int* ih)
{
    int c = 0;
    for (int j = 0; j < kAlphaTile && b0 + j < T; ++j) {
        const double l = lo[b0 + j], h = hi[b0 + j];
        if (c > 0 && l == E[c - 1]) il[j] = c - 1;
        else { E[c] = l; il[j] = c++; }
        E[c] = h;
        ih[j] = c++;
    }
    return c;
}

// Tile precomputation jobs (k_alpha_tile; emulated on the host by tests/hostcheck).
// Edge-leaf block of mass state k: [5][ct] t edges, [4][cs] S' edges, [2][kAlphaTile] m bins (the
// shared fields), then after the 3 blocks the member blocks of (k, point m): [ct] L2, [cs] Ls,
// [cs] cS, [kAlphaTile] atd.
NUSI_FN int alpha_tile_edge_stride(int cs, int ct) { return kTEdgeFields * ct + kSEdgeFields * cs + kMBinFields * kAlphaTile; }
NUSI_FN int alpha_tile_member_stride(int cs, int ct) { return ct + 2 * cs + kAlphaTile; }
NUSI_FN int alpha_tile_edge_doubles(int cs, int ct, int G)
{
    return 3 * (alpha_tile_edge_stride(cs, ct) + G * alpha_tile_member_stride(cs, ct));
}
NUSI_FN double* alpha_tile_member_block(double* edg, int cs, int ct, int G, int k, int m)
{
    return edg + 3 * alpha_tile_edge_stride(cs, ct) + (k * G + m) * alpha_tile_member_stride(cs, ct);
}
// job in [0, 3 (ct + cs + kAlphaTile)): the shared edge / m-bin leaves of one mass state (P: any
// point of the tile's batch -- they read m_phi and the masses only)
// job j in [0, ct + cs + kAlphaTile) of mass state k into that state's edge block edgk
NUSI_FN void alpha_tile_edge_job_k(const Point& P, int k, int j, const double* tE, int ct, const double* sE, int cs,
                                   const double* lo, const double* hi, int m0, int T, double* edgk)
{
    const double mphi = P.mphi, m2 = mphi * mphi;
    const double mk = P.mn[k];
    double* ted = edgk;
    double* sed = ted + kTEdgeFields * ct;
    double* mbv = sed + kSEdgeFields * cs;
    if (j < ct) {
        const double t = alpha_t(mk, tE[j], m2);
        ted[kTEdgeVal * ct + j] = t;
        if (!P.non_resonant) return;
        AlphaTEdge e;
        alpha_tedge_shared(t, e);
        ted[j] = e.Lm1; ted[ct + j] = e.la; ted[2 * ct + j] = e.cm; ted[3 * ct + j] = e.am;
    } else if (j < ct + cs) {
        const int q = j - ct;
        const double S = alpha_S(mk, sE[q], m2);
        sed[kSEdgeVal * cs + q] = S;
        if (!P.non_resonant) return;
        AlphaSEdge e;
        alpha_sedge_shared(S, e);
        sed[q] = e.lS; sed[cs + q] = e.l2; sed[2 * cs + q] = e.lS2;
    } else {
        const int q = j - ct - cs;
        if (m0 + q >= T) return;
        const double Sm = alpha_S(mk, lo[m0 + q], m2), Sp = alpha_S(mk, hi[m0 + q], m2);
        mbv[q] = nm::log(Sm / Sp);
        mbv[kAlphaTile + q] = nm::log(Sp / Sm);
    }
}
NUSI_FN void alpha_tile_edge_job(const Point& P, int job, const double* tE, int ct, const double* sE, int cs,
                                 const double* lo, const double* hi, int m0, int T, double* edg)
{
    const int per = ct + cs + kAlphaTile;
    const int k = job / per;
    alpha_tile_edge_job_k(P, k, job - k * per, tE, ct, sE, cs, lo, hi, m0, T, edg + k * alpha_tile_edge_stride(cs, ct));
}
// job in [0, 3 (ct + cs + kAlphaTile)): the member edge / m-bin leaves of point P (slot m of the
// batch); t and S' are recomputed (the same expression), so no barrier orders it after the shared jobs
NUSI_FN void alpha_tile_edge_member_job(const Point& P, int m, int G, int job, const double* tE, int ct,
                                        const double* sE, int cs, const double* lo, const double* hi, int m0, int T,
                                        double* edg)
{
    const double mphi = P.mphi, Ga = P.Ga, m2 = mphi * mphi, gr = P.a_gr, gr2 = gr * gr;
    const int per = ct + cs + kAlphaTile;
    const int k = job / per, j = job - k * per;
    const double mk = P.mn[k];
    double* mbk = alpha_tile_member_block(edg, cs, ct, G, k, m);
    if (j < ct) {
        if (!P.non_resonant) return;
        mbk[j] = alpha_tedge_L2(alpha_t(mk, tE[j], m2), gr2);
    } else if (j < ct + cs) {
        if (!P.non_resonant) return;
        const int q = j - ct;
        AlphaSEdge e;
        alpha_sedge_member(alpha_S(mk, sE[q], m2), gr, gr2, e);
        mbk[ct + q] = e.Ls;
        mbk[ct + cs + q] = e.cS;
    } else {
        const int q = j - ct - cs;
        if (m0 + q >= T) return;
        mbk[ct + 2 * cs + q] = alpha_mbin_atd(alpha_S(mk, lo[m0 + q], m2), alpha_S(mk, hi[m0 + q], m2), mphi, Ga);
    }
}
// job j in [0, cs ct): the shared leaves of corner (S' slot j / ct, t slot j % ct) of mass state k;
// edgk = the edge block of mass state k (its t and S' values)
template <bool kRef = false>
NUSI_FN void alpha_tile_corner_job(int j, const double* edgk, int ct, int cs, double* cor)
{
    const int cc = cs * ct;
    const int si = j / ct, ti = j - si * ct;
    AlphaCorner c;
    alpha_corner_shared<kRef>(edgk[kTEdgeFields * ct + kSEdgeVal * cs + si], edgk[kTEdgeVal * ct + ti], c);
    cor[j] = c.L; cor[cc + j] = c.LL; cor[2 * cc + j] = c.TU1; cor[3 * cc + j] = c.TU2; cor[4 * cc + j] = c.G;
    cor[5 * cc + j] = c.Drr; cor[6 * cc + j] = c.Dri;
}
// job j in [0, cs ct): the member leaves of corner j for point P (slot m of the batch)
template <bool kRef = false>
NUSI_FN void alpha_tile_corner_member_job(const Point& P, int m, int j, const double* edgk, int ct, int cs, double* cor)
{
    const int cc = cs * ct;
    const int si = j / ct, ti = j - si * ct;
    AlphaCorner c;
    alpha_corner_member<kRef>(edgk[kTEdgeFields * ct + kSEdgeVal * cs + si], edgk[kTEdgeVal * ct + ti], P.a_gr, c);
    double* d = cor + (kCornerShared + kCornerMember * m) * cc;
    d[j] = c.Dcr; d[cc + j] = c.Dci; d[2 * cc + j] = c.A;
}
// job j in [0, kAlphaTile (cs + ct)): the xlog leaf (S' slot, n bin) or the ylog leaf (m bin, t slot)
// of mass state k (shared), into the block after the corners; bins past the table are skipped
NUSI_FN void alpha_tile_mixed_job(int j, const double* edgk, int ct, int cs, int G, const int* tl, const int* th,
                                  const int* sl, const int* sh, int n0, int m0, int T, int Tm, double* cor)
{
    const double* tv = edgk + kTEdgeVal * ct;                           // t of each t slot
    const double* sv = edgk + kTEdgeFields * ct + kSEdgeVal * cs;       // S' of each S' slot
    double* xl = cor + (kCornerShared + kCornerMember * G) * cs * ct;
    double* yl = xl + kAlphaTile * cs;
    if (j < kAlphaTile * cs) {
        const int s = j / kAlphaTile, ln = j - s * kAlphaTile;
        if (n0 + ln >= T) return;
        xl[j] = alpha_xlog(sv[s], tv[tl[ln]], tv[th[ln]]);
    } else {
        const int q = j - kAlphaTile * cs, lm = q / ct, t = q - lm * ct;
        if (m0 + lm >= Tm) return;   // Tm: end of the tile's m bins
        yl[q] = alpha_ylog(sv[sl[lm]], sv[sh[lm]], tv[t]);
    }
}
// leaves of entry (n0 + ln, m0 + lm) of a tile for mass state k and batch point m (of G)
NUSI_FN TileLeaves alpha_tile_leaves(const double* cor, const double* edg, int k, int m, int G, int cs, int ct, int lm,
                                     const int* sl, const int* sh, const int* tl, const int* th, int ln)
{
    TileLeaves lv;
    lv.cc = cs * ct;
    lv.cor = cor;
    lv.corm = cor + (kCornerShared + kCornerMember * m) * lv.cc;
    lv.ct = ct;
    lv.cs = cs;
    lv.mb = lm;
    lv.nb = ln;
    lv.xl = cor + (kCornerShared + kCornerMember * G) * lv.cc;
    lv.yl = lv.xl + kAlphaTile * cs;
    lv.sidx[0] = sl[lm];
    lv.sidx[1] = sh[lm];
    lv.tidx[0] = tl[ln];
    lv.tidx[1] = th[ln];
    lv.ted = edg + k * alpha_tile_edge_stride(cs, ct);
    lv.sed = lv.ted + kTEdgeFields * ct;
    lv.mbv = lv.sed + kSEdgeFields * cs;
    const double* mbk = alpha_tile_member_block(const_cast<double*>(edg), cs, ct, G, k, m);
    lv.tedm = mbk;
    lv.sedm = mbk + ct;
    lv.mbm = mbk + ct + 2 * cs;
    return lv;
}

// phi-phi double-scalar production term of alpha (nuSIprop.hpp:1477-1503), split as
//   alpha_pp = ((g^4 / m_phi^4 * f1) * f2) / den  (then * |U_fk|^2 and the Majorana / 2-neutrino factors),
// the reference's association in each branch: f1 = |spline(S'-, ln(-S'-/t-)/ln d * 1.0001, log10 d)| below
// S'- = 1e4 (f2 = den = 1), else its large-s expansion (branch 1: f1 = numerator, den = 256 pi S-^2 S+^2;
// branch 2: f1 = the whole bracket; branch 3: f1 = t+ - t-, f2 = bracket, den = 128 pi S- S+).  The term
// reads neither g nor Gamma_phi, so the points of a batch (same m_phi and masses) share it.  Out of line:
// only the phiphi configuration reaches it, and inlined it would cost every entry registers.  The
// out-of-range warning comes back in the result (oob), not through a reference: a caller's warning word
// whose address escaped into a call would live in scratch, stored and reloaded every entry.
struct PPTerm { double f1, f2, den; int oob = 0; };
NUSI_FN_OUT PPTerm alpha_phiphi_core(const SplineSet& spl, double Sm, double Sp, double tm, double tp, double lSm,
                                     double lSp)
{
    if (Sm < 1e4) {
        const double d = Sp / Sm;
        const double xx[3] = {Sm, nm::log(-Sm / tm) / nm::log(d) * 1.0001, nm::log10(d)};
        double v = 0;
        const bool in = spl.a.eval<3>(xx, v);
        return PPTerm{fabs(v), 1.0, 1.0, in ? 0 : kWarnSplineOOB};
    }
    if (tm < -1) {
        const double l1m = nm::log(-1 - tm), l0m = nm::log(-tm), l1p = nm::log(-1 - tp), l0p = nm::log(-tp);
        return PPTerm{((-Sm + Sp) * ((tm - tp) * (Sp * (-2 + tm + tp) + Sm * (-2 - 24 * Sp + tm + tp))
                              + 4 * (-(Sp * (1 + tm)) + Sm * (-1 + 2 * Sp + (-1 + Sp) * tm)) * l1m
                              + 2 * (3 * Sp + Sm * (3 + 4 * Sp)) * tm * l0m
                              + 4 * (Sp + Sp * tp + Sm * (1 + tp - Sp * (2 + tp))) * l1p
                              - 2 * (3 * Sp + Sm * (3 + 4 * Sp)) * tp * l0p)
                + 2 * (Sm * Sm) * lSp * ((3 + 2 * Sp) * (tm - tp) + 2 * (Sp * Sp) * ((-1 - tm) * l1m + tm * l0m + (1 + tp) * l1p - tp * l0p))
                + 2 * (Sp * Sp) * lSm * ((-3 - 2 * Sm) * (tm - tp) + 2 * (Sm * Sm) * ((1 + tm) * l1m - tm * l0m - (1 + tp) * l1p + tp * l0p))),
                      1.0, 256. * kPi * (Sm * Sm) * (Sp * Sp)};
    }
    if (tp < -1) {
        const double l1p = nm::log(-1 - tp), l0p = nm::log(-tp);
        return PPTerm{(2 * (Sm * Sm) * lSp * ((1 + tp) * (-3 - 2 * Sp + 2 * (Sp * Sp) * l1p) - 2 * (Sp * Sp) * tp * l0p)
                + (Sm - Sp) * ((1 + tp) * (-3 * (Sm + Sp + 8 * Sm * Sp) + (Sm + Sp) * tp)
                               + 4 * (-(Sp * (1 + tp)) + Sm * (-1 + 2 * Sp + (-1 + Sp) * tp)) * l1p
                               + 2 * (3 * Sp + Sm * (3 + 4 * Sp)) * tp * l0p)
                + 2 * (Sp * Sp) * lSm * ((3 + 2 * Sm) * (1 + tp) + 2 * (Sm * Sm) * (-((1 + tp) * l1p) + tp * l0p)))
                   / (256. * kPi * (Sm * Sm) * (Sp * Sp))
               + (-1 - tm) * (-6 * Sm + 6 * Sp - 2 * (-2 + Sm) * Sp * lSm + Sm * Sp * (lSm * lSm) + 2 * Sm * (-2 + Sp) * lSp - Sm * Sp * (lSp * lSp))
                     / (128. * kPi * Sm * Sp), 1.0, 1.0};
    }
    return PPTerm{tp - tm,
                  -6 * Sm + 6 * Sp - 2 * (-2 + Sm) * Sp * lSm + Sm * Sp * (lSm * lSm) + 2 * Sm * (-2 + Sp) * lSp - Sm * Sp * (lSp * lSp),
                  128. * kPi * Sm * Sp};
}
// alpha_pp of point P from its term (the reference's association: ((g^4/m^4 * f1) * f2) / den; f2 = den = 1
// are exact)
NUSI_FN double alpha_phiphi_scale(const Point& P, double uk, const PPTerm& X)
{
    const double g = P.g, mphi = P.mphi;
    const double g4 = (g * g) * (g * g), m4 = (mphi * mphi) * (mphi * mphi);
    double app = ((g4 / m4 * X.f1) * X.f2) / X.den;
    app *= uk;
    if (P.majorana) app *= 2;
    app *= 2;
    if (P.majorana) app *= 2;
    return app;
}

// Leaves of the big-batch tile kernel (k_alpha_batch): the shared corner fields live in separate blocks
// (L, Drr, Dri persist for every mass state through the batch loop; LL, TU1, TU2, G and the mixed logs
// only while the batch's shared brackets are formed), so each field has its own base pointer.  kRefA
// (NUSI_OPT_REFERENCE_ORDER): A is a corner field of its own, marg[o] (the batch kernel's per-point A block).
// The big-batch kernel's corner blocks (P3, X, mem) keep their fields kCC doubles apart, a compile-time stride, so that
// every field of a corner is one LDS load at an immediate offset from the same address.
constexpr int kCC = (kAlphaTile + 1) * (kAlphaTile + 1);
template <bool kRefA = false>
struct SplitLeavesT {
    const double* cf[kCornerShared];   // L LL TU1 TU2 G Drr Dri, each [cc]
    const double *corm, *ted, *sed, *mbv, *tedm, *sedm, *mbm, *xl, *yl;
    const double* marg;                // sT [ct] | fT [ct] | sS [cs] | fS [cs]: A from the edge arguments (kRefA: A [cc])
    int cc, ct, cs, mb, nb;
    int sidx[2], tidx[2];
    NUSI_FN AlphaCorner corner(int si, int ti, double, double) const
    {
        const int o = sidx[si] * ct + tidx[ti];
        const int a = sidx[si], b = tidx[ti];
        // A = arg(S - 1 + i gr) + arg(c + i gr) - pi, the expression of alpha_member_corner
        const double A = kRefA ? marg[o] : (marg[2 * ct + a] + marg[b]) + (marg[2 * ct + cs + a] + marg[ct + b] - 1.0) * kPi;
        return AlphaCorner{cf[0][o], cf[1][o], cf[2][o], cf[3][o], cf[4][o], cf[5][o], cf[6][o],
                           corm[o], corm[kCC + o], A};
    }
    NUSI_FN AlphaTEdge tedge(int ti, double) const
    {
        const double* e = ted + tidx[ti];
        return AlphaTEdge{e[0], e[ct], e[2 * ct], tedm[tidx[ti]], e[3 * ct]};
    }
    NUSI_FN AlphaSEdge sedge(int si, double) const
    {
        const double* e = sed + sidx[si];
        return AlphaSEdge{e[0], e[cs], sedm[sidx[si]], sedm[cs + sidx[si]], e[2 * cs]};
    }
    NUSI_FN AlphaMBin mbin(double, double) const { return AlphaMBin{mbv[mb], mbv[kAlphaTile + mb], mbm[mb]}; }
    NUSI_FN double tval(int ti, double, double, double) const { return ted[kTEdgeVal * ct + tidx[ti]]; }
    NUSI_FN double Sval(int si, double, double, double) const { return sed[kSEdgeVal * cs + sidx[si]]; }
    NUSI_FN double xlog(int si, double, double, double) const { return xl[sidx[si] * kAlphaTile + nb]; }
    NUSI_FN double ylog(int ti, double, double, double) const { return yl[mb * ct + tidx[ti]]; }
};
using SplitLeaves = SplitLeavesT<false>;
// shared corner leaves of corner j: L, Drr, Dri -> per[0..2][cc] (kept), LL, TU1, TU2, G -> tmp[0..3][cc]
template <bool kRef = false>
NUSI_FN void alpha_batch_corner_job(int j, const double* edgk, int ct, int cs, double* per, double* tmp)
{
    const int si = j / ct, ti = j - si * ct;
    AlphaCorner c;
    alpha_corner_shared<kRef>(edgk[kTEdgeFields * ct + kSEdgeVal * cs + si], edgk[kTEdgeVal * ct + ti], c);
    per[j] = c.L; per[kCC + j] = c.Drr; per[2 * kCC + j] = c.Dri;
    tmp[j] = c.LL; tmp[kCC + j] = c.TU1; tmp[2 * kCC + j] = c.TU2; tmp[3 * kCC + j] = c.G;
}
// The big-batch kernel's member blocks, per (point, mass state):
//   X    [10][cc]  shared across the batch: the Taylor coefficients of Li2 about x0 = (1+S+t)/(2+t) per corner
//                  (c_0..c_6, 1/x0, pi log x0, the radius bound m), alpha_batch_xshared_job
//   memb [5 ct + 4 cs + kAlphaTile]  the point's edge leaves: L2 [ct] | Ls [cs] | cS [cs] | atd [kAlphaTile] |
//                  inv [ct] | q [ct] | sT [ct] | fT [ct] | sS [cs] | fS [cs]   (the first four as TileLeaves reads them)
//   mem  [2][cc]   the point's corner leaves Dcr, Dci (A = sum of the edge arguments, formed where read)
constexpr int kXFields = kLi2AxisTerms + 4;
NUSI_FN int alpha_batch_memb_doubles(int cs, int ct) { return 5 * ct + 4 * cs + kAlphaTile; }
NUSI_FN void alpha_batch_xshared_job(int j, const double* edgk, int ct, int cs, double* X)
{
    const int si = j / ct, ti = j - si * ct;
    MemberShared M;
    alpha_member_shared(edgk[kTEdgeFields * ct + kSEdgeVal * cs + si], edgk[kTEdgeVal * ct + ti], M);
#pragma unroll
    for (int n = 0; n <= kLi2AxisTerms; ++n) X[n * kCC + j] = M.T.c[n];
    X[(kLi2AxisTerms + 1) * kCC + j] = M.T.r;
    X[(kLi2AxisTerms + 2) * kCC + j] = M.T.b0;
    X[(kLi2AxisTerms + 3) * kCC + j] = M.m;
}
// job in [0, ct + cs + kAlphaTile): the member edge / m-bin leaves of point P for mass state k
NUSI_FN void alpha_batch_medge_job(const Point& P, int k, int job, const double* tE, int ct, const double* sE, int cs,
                                   const double* lo, const double* hi, int m0, int Tm, double* memb)
{
    const double mphi = P.mphi, Ga = P.Ga, m2 = mphi * mphi, gr = P.a_gr, gr2 = gr * gr, mk = P.mn[k];
    double* ext = memb + ct + 2 * cs + kAlphaTile;   // inv | q | sT | fT | sS | fS
    if (job < ct) {
        if (!P.non_resonant) return;
        const double t = alpha_t(mk, tE[job], m2);
        memb[job] = alpha_tedge_L2(t, gr2);
        const MemberTEdge e = alpha_member_tedge(t, gr);
        ext[job] = e.inv; ext[ct + job] = e.q; ext[2 * ct + job] = e.sT; ext[3 * ct + job] = e.fT;
    } else if (job < ct + cs) {
        if (!P.non_resonant) return;
        const int q = job - ct;
        const double S = alpha_S(mk, sE[q], m2);
        AlphaSEdge e;
        alpha_sedge_member(S, gr, gr2, e);
        memb[ct + q] = e.Ls;
        memb[ct + cs + q] = e.cS;
        alpha_member_sarg(S, gr, ext[4 * ct + q], ext[4 * ct + cs + q]);
    } else {
        const int q = job - ct - cs;
        if (m0 + q >= Tm) return;
        memb[ct + 2 * cs + q] = alpha_mbin_atd(alpha_S(mk, lo[m0 + q], m2), alpha_S(mk, hi[m0 + q], m2), mphi, Ga);
    }
}
// The member edge leaves of a table point are functions of one bin edge energy (t side, S' side) or of
// one bin (atd), not of the tile: k_alpha_medge evaluates them once per (point, k, bin edge) into
// global memory -- layout per (point, k), with e = 2 b + (0: lo[b], 1: hi[b]):
//   L2 inv q sT fT [5][2T] | Ls cS sS fS [4][2T] | atd [T]
// -- and the batch kernel copies its tile's edges from there (alpha_batch_medge_copy), instead of every
// tile of a row re-evaluating the same edges.  Same functions, same arguments: the same bits as
// alpha_batch_medge_job.
constexpr int kMedFields = 19;   // doubles per bin per (point, k): 2 (5 + 4) + 1
NUSI_FN void alpha_medge_job(const Point& P, int k, int j, int T, const double* lo, const double* hi, double* med)
{
    const double mphi = P.mphi, Ga = P.Ga, m2 = mphi * mphi, gr = P.a_gr, gr2 = gr * gr, mk = P.mn[k];
    const int E2 = 2 * T;
    if (j < E2) {
        if (!P.non_resonant) return;
        const double t = alpha_t(mk, (j & 1) ? hi[j >> 1] : lo[j >> 1], m2);
        med[j] = alpha_tedge_L2(t, gr2);
        const MemberTEdge e = alpha_member_tedge(t, gr);
        med[E2 + j] = e.inv; med[2 * E2 + j] = e.q; med[3 * E2 + j] = e.sT; med[4 * E2 + j] = e.fT;
    } else if (j < 2 * E2) {
        if (!P.non_resonant) return;
        const int q = j - E2;
        const double S = alpha_S(mk, (q & 1) ? hi[q >> 1] : lo[q >> 1], m2);
        AlphaSEdge e;
        alpha_sedge_member(S, gr, gr2, e);
        double* ms = med + 5 * E2;
        ms[q] = e.Ls;
        ms[E2 + q] = e.cS;
        alpha_member_sarg(S, gr, ms[2 * E2 + q], ms[3 * E2 + q]);
    } else if (j < 2 * E2 + T) {
        const int b = j - 2 * E2;
        med[9 * E2 + b] = alpha_mbin_atd(alpha_S(mk, lo[b], m2), alpha_S(mk, hi[b], m2), mphi, Ga);
    }
}
// alpha_batch_medge_job's outputs, copied from k_alpha_medge's block med (point, k): medge_load reads
// job's values (tsrc / ssrc: the bin edge, 2 b + side, each slot of the tile's t / S' edge list was
// taken from), medge_store puts them where alpha_batch_medge_job would have written them.
struct MedVals { double v[5]; };
NUSI_FN void alpha_batch_medge_load(bool nonres, int job, const int* tsrc, int ct, const int* ssrc, int cs, int m0,
                                    int Tm, int T, const double* __restrict__ med, MedVals& o)
{
    const int E2 = 2 * T;
    if (job < ct) {
        if (!nonres) return;
        const int e = tsrc[job];
#pragma unroll
        for (int f = 0; f < 5; ++f) o.v[f] = med[f * E2 + e];
    } else if (job < ct + cs) {
        if (!nonres) return;
        const int e = ssrc[job - ct];
#pragma unroll
        for (int f = 0; f < 4; ++f) o.v[f] = med[(5 + f) * E2 + e];
    } else {
        const int q = job - ct - cs;
        if (m0 + q < Tm) o.v[0] = med[9 * E2 + m0 + q];
    }
}
NUSI_FN void alpha_batch_medge_store(bool nonres, int job, int ct, int cs, int m0, int Tm, const MedVals& o, double* memb)
{
    double* ext = memb + ct + 2 * cs + kAlphaTile;   // inv | q | sT | fT | sS | fS
    if (job < ct) {
        if (!nonres) return;
        memb[job] = o.v[0];
        ext[job] = o.v[1]; ext[ct + job] = o.v[2]; ext[2 * ct + job] = o.v[3]; ext[3 * ct + job] = o.v[4];
    } else if (job < ct + cs) {
        if (!nonres) return;
        const int q = job - ct;
        memb[ct + q] = o.v[0];
        memb[ct + cs + q] = o.v[1];
        ext[4 * ct + q] = o.v[2];
        ext[4 * ct + cs + q] = o.v[3];
    } else {
        const int q = job - ct - cs;
        if (m0 + q < Tm) memb[ct + 2 * cs + q] = o.v[0];
    }
}
// member corner leaves of corner j for point P -> mem[0..2][cc] (Dcr, Dci, A); edgk: the shared edge block of
// mass state k (its t and S' values)
NUSI_FN void alpha_batch_mcorner_job(const Point& P, int j, const double* edgk, int ct, int cs, const double* X,
                                     const double* memb, double* mem)
{
    const int si = j / ct, ti = j - si * ct;
    MemberShared M;
#pragma unroll
    for (int n = 0; n <= kLi2AxisTerms; ++n) M.T.c[n] = X[n * kCC + j];
    M.T.r = X[(kLi2AxisTerms + 1) * kCC + j];
    M.T.b0 = X[(kLi2AxisTerms + 2) * kCC + j];
    M.m = X[(kLi2AxisTerms + 3) * kCC + j];
    const double* ext = memb + ct + 2 * cs + kAlphaTile;
    const MemberTEdge e{ext[ti], ext[ct + ti], ext[2 * ct + ti], ext[3 * ct + ti]};
    double Dcr, Dci, A;
    alpha_member_corner(M, edgk[kTEdgeFields * ct + kSEdgeVal * cs + si], edgk[kTEdgeVal * ct + ti], P.a_gr, e,
                        ext[4 * ct + si], ext[4 * ct + cs + si], Dcr, Dci, A);
    mem[j] = Dcr; mem[kCC + j] = Dci;   // (A: SplitLeaves forms it from the edge arguments)
}
// NUSI_OPT_REFERENCE_ORDER: the S' and t of member corner c = us (us + 1) / 2 + ut (S' edge us, t edge ut <= us,
// energies ue[]) of mass state k for the tables of a batch whose first point is P (m_phi and the masses), by the
// functions the tile's edge block uses (alpha_tile_edge_job_k), so the values are those the batch kernel's own
// corners take; the member leaves are then alpha_member_ref_dc / _arg of (S', t, gr)
NUSI_FN void alpha_mcorner_st(const Point& P, int k, long long c, const double* ue, double& S, double& t)
{
    int us = (int)((sqrt(8.0 * (double)c + 1.0) - 1.0) * 0.5);
    while ((long long)us * (us + 1) / 2 > c) --us;
    while ((long long)(us + 1) * (us + 2) / 2 <= c) ++us;
    const int ut = (int)(c - (long long)us * (us + 1) / 2);
    const double m2 = P.mphi * P.mphi, mk = P.mn[k];
    S = alpha_S(mk, ue[us], m2);
    t = alpha_t(mk, ue[ut], m2);
}
// xlog / ylog leaves of mass state k into xl [cs][kAlphaTile], yl [kAlphaTile][ct] (alpha_tile_mixed_job's jobs)
NUSI_FN void alpha_batch_mixed_job(int j, const double* edgk, int ct, int cs, const int* tl, const int* th,
                                   const int* sl, const int* sh, int n0, int m0, int T, int Tm, double* xl, double* yl)
{
    const double* tv = edgk + kTEdgeVal * ct;
    const double* sv = edgk + kTEdgeFields * ct + kSEdgeVal * cs;
    if (j < kAlphaTile * cs) {
        const int s = j / kAlphaTile, ln = j - s * kAlphaTile;
        if (n0 + ln >= T) return;
        xl[j] = alpha_xlog(sv[s], tv[tl[ln]], tv[th[ln]]);
    } else {
        const int q = j - kAlphaTile * cs, lm = q / ct, t = q - lm * ct;
        if (m0 + lm >= Tm) return;
        yl[q] = alpha_ylog(sv[sl[lm]], sv[sh[lm]], tv[t]);
    }
}

// compiler fence between the phases of alpha_k (device: no scheduling or LDS-load reuse across it)
#ifdef __HIP_DEVICE_COMPILE__
#define NUSI_PHASE() do { __builtin_amdgcn_sched_barrier(0); __asm__ volatile("" ::: "memory"); } while (0)
#else
#define NUSI_PHASE() do { } while (0)
#endif
// The Majorana t (:1281-1333) and tu (:1370-1425) channels are g^4 / D * B with D and the bracket B
// functions of the (S', t) leaves alone: points of a batch (same m_phi, masses, flags) share them.
struct AlphaPre { double Dt, Bt, Dtu, Btu; };
template <class Lv>
NUSI_FN void alpha_bracket_t(const Lv& lv, double Sm, double Sp, double tm, double tp, double m4, double& D, double& B)
{
    const AlphaSEdge eSm = lv.sedge(0, Sm), eSp = lv.sedge(1, Sp);
    const double lSm = eSm.lS, lSp = eSp.lS;
    const double SS = Sm * Sp;
    const AlphaCorner cmm = lv.corner(0, 0, Sm, tm), cpm = lv.corner(1, 0, Sp, tm);
    const AlphaCorner cmq = lv.corner(0, 1, Sm, tp), cpq = lv.corner(1, 1, Sp, tp);
    const double Lmm = cmm.L, Lpm = cpm.L, Lmq = cmq.L, Lpq = cpq.L;
    const double LA = lv.xlog(0, Sm, tm, tp), LB = lv.xlog(1, Sp, tm, tp);
    const double inner = SS * (-tm + tp) * lSm + SS * (tm - tp) * lSp - SS * Lmm - SS * tp * Lmm + SS * Lpm + SS * tp * Lpm
                         - Sp * LA - Sp * tm * LA - Sp * tp * LA - Sp * tm * tp * LA
                         + SS * cmq.LL + SS * tm * Lmq
                         + Sm * LB + Sm * tm * LB + Sm * tp * LB + Sm * tm * tp * LB
                         - SS * cpq.LL - SS * tm * Lpq;
    D = Sm * Sp * 16 * kPi * m4;
    B = (-((Sm - Sp) * (3 + 2 * tm * (-1 + tp) - 2 * tp) * (tm - tp)) / ((-1 + tm) * (-1 + tp))
         + 2 * inner / ((1 + tm) * (1 + tp))
         - ((SS * lv.ylog(0, Sm, Sp, tm)) / ((1 + tm) * (1 + tm))
            + (((Sm - Sp) * (tm - tp) * (1 + tp)) / (1 + tm) - SS * lv.ylog(1, Sm, Sp, tp)) / ((1 + tp) * (1 + tp))));
}
template <class Lv>
NUSI_FN void alpha_bracket_tu(const Lv& lv, double Sm, double Sp, double tm, double tp, double m4, double& D, double& B)
{
    const double SS = Sm * Sp;
    const AlphaCorner cmm = lv.corner(0, 0, Sm, tm), cpm = lv.corner(1, 0, Sp, tm);
    const AlphaCorner cmq = lv.corner(0, 1, Sm, tp), cpq = lv.corner(1, 1, Sp, tp);
    const AlphaSEdge fSm = lv.sedge(0, Sm), fSp = lv.sedge(1, Sp);
    const AlphaTEdge fTm = lv.tedge(0, tm), fTp = lv.tedge(1, tp);
    const AlphaMBin mc = lv.mbin(Sm, Sp);
    const double Lmm = cmm.L, Lpm = cpm.L, Lmq = cmq.L, Lpq = cpq.L;
    double Fp, Fm;
    if (tp < -1) Fp = cmq.TU1 - cpq.TU1;
    else {
        const double a = cmq.TU2, b = cpq.TU2;
        Fp = -cmq.TU1 + cpq.TU1 - 0.5 * (a * a - b * b);
    }
    if (tm < -1) Fm = -cmm.TU1 + cpm.TU1;
    else {
        const double a = cmm.TU2, b = cpm.TU2;
        Fm = cmm.TU1 - cpm.TU1 + 0.5 * (a * a - b * b);
    }
    const double lap = fTp.la, lam = fTm.la;
    const double Pq = (1 + tm) * (1 + tp);
    const double l2m = fSm.l2, l2p = fSp.l2;
    const double SSP = SS * (1 + tm) * (1 + tp);
    const double lSm = fSm.lS, lSp = fSp.lS, Lmt = fTm.Lm1, Lmp = fTp.Lm1;
    D = 32 * kPi * m4 * Sm * Sp * (1 + tm) * (1 + tp);
    B = (-4 * (Sm - Sp) * (1 + tm) * (tm - tp) * (1 + tp)
         + 2 * SS * tp * (mc.lr - Lmm + Lpm)
         + 2 * Sp * (1 + tm) * (1 + tp) * (Lmt - Lmm - Lmp + Lmq)
         - 2 * Sm * (1 + tm) * (1 + tp) * (Lmt - Lpm - Lmp + Lpq)
         + 2 * SS * (-Lmm + Lpm + Lmq - Lpq)
         + SSP * (l2m * (lSp + Lmq) - l2p * (lSm + Lpq) + Lmp * (mc.lr - Lmq + Lpq))
         + SSP * ((lSp + Lmm) * (fSm.lS2 + Lmt - lam) + (lSm + Lpm) * (l2p - Lmt + lam))
         + SS * (mc.lr2 + Lmq - Lpq) * (2 * tm + Pq * lap)
         + SSP * (cmm.G - cpm.G - cmq.G + cpq.G)
         + SSP * (Fp + Fm));
}
// the shared brackets of entry (Em, Ep, Em', Ep') and mass state k (Majorana, non-resonant)
template <class Lv>
NUSI_FN void alpha_k_pre(const Point& P, int k, double Em, double Ep, double Emp, double Epp, const Lv& lv, AlphaPre& pre)
{
    const double mphi = P.mphi, m2 = mphi * mphi, m4 = (mphi * mphi) * (mphi * mphi), mk = P.mn[k];
    const double tp = lv.tval(1, mk, Ep, m2), tm = lv.tval(0, mk, Em, m2);
    const double Sp = lv.Sval(1, mk, Epp, m2), Sm = lv.Sval(0, mk, Emp, m2);
    alpha_bracket_t(lv, Sm, Sp, tm, tp, m4, pre.Dt, pre.Bt);
    alpha_bracket_tu(lv, Sm, Sp, tm, tp, m4, pre.Dtu, pre.Btu);
}
// the phi-phi term of entry (Em, Ep, Em', Ep') and mass state k (shared by a batch); zero term where the
// channel is closed (S'- <= 4)
template <class Lv>
NUSI_FN PPTerm alpha_k_pp(const Point& P, const SplineSet& spl, int k, double Em, double Ep, double Emp, double Epp,
                          const Lv& lv, int& warn)
{
    const double mphi = P.mphi, m2 = mphi * mphi, mk = P.mn[k];
    const double tp = lv.tval(1, mk, Ep, m2), tm = lv.tval(0, mk, Em, m2);
    const double Sp = lv.Sval(1, mk, Epp, m2), Sm = lv.Sval(0, mk, Emp, m2);
    if (!(Sm > 4 && P.phiphi)) return PPTerm{0.0, 1.0, 1.0};
    const AlphaSEdge eSm = lv.sedge(0, Sm), eSp = lv.sedge(1, Sp);
    const PPTerm X = alpha_phiphi_core(spl, Sm, Sp, tm, tp, eSm.lS, eSp.lS);
    warn |= X.oob;
    return X;
}

// one mass state k of alpha(Em, Ep, Em', Ep'): tot += wgt * (every channel); pre: the shared brackets
// of a batch (alpha_k_pre with another point of it), nullptr = evaluate them here.  kPhiPhi = false: the caller's
// points have no phi-phi channel, and the call of the out-of-line phi-phi term is compiled out (its register
// footprint otherwise shapes the caller's allocation around the call: C4 alpha 5.58 -> 5.94 ms with the unrolled
// spline evaluator)
// The terms alpha_k adds to its running sum, recorded in order instead (the k-split alpha path of calls of few
// tables: every mass state's workgroups run at once, and k_alpha_ksum adds the terms in the same order -- the same
// additions from the same 0.0, so the same bits)
struct TermRec {
    double v[7];
    int n = 0;
    NUSI_FN TermRec& operator+=(double x)
    {
        v[n++] = x;
        return *this;
    }
};
template <class Lv, bool kPhiPhi = true, class Acc = double>
NUSI_FN void alpha_k(const Point& P, const SplineSet& spl, int k, double Em, double Ep, double Emp, double Epp,
                     const Lv& lv, Acc& tot, int& warn, const AlphaPre* pre = nullptr, const PPTerm* ppt = nullptr)
{
    const double g = P.g, mphi = P.mphi;
    const double g4 = (g * g) * (g * g), m2 = mphi * mphi, m4 = (mphi * mphi) * (mphi * mphi);
    const double gr = P.a_gr, gr2 = gr * gr;
    const bool maj = P.majorana;
    const double mk = P.mn[k], uk = P.u[k];
    const double tp = lv.tval(1, mk, Ep, m2), tm = lv.tval(0, mk, Em, m2);
    const double Sp = lv.Sval(1, mk, Epp, m2), Sm = lv.Sval(0, mk, Emp, m2);
    const double wgt = P.a_wgt[k];
    const AlphaMBin mb = lv.mbin(Sm, Sp);

    double as;
    if (Sp < 1e-5)
        as = P.a_s * (tm - tp) *
             ((gr * (1 + gr2 + 2 * Sm)) / ((1 + gr2) * (1 + gr2)) * (Sp - Sm) + gr / ((1 + gr2) * (1 + gr2)) * ((Sp - Sm) * (Sp - Sm)));
    else
        as = P.a_s * (tm - tp) * mb.atd;
    as *= uk;
    if (!maj) as /= 2.;
    tot += wgt * as;
    if (!P.non_resonant) return;

    // The Majorana channels run as three phases (t/u, tu, st) that each fetch the leaves they use:
    // NUSI_PHASE stops the compiler from keeping all ~60 leaves of the entry live at once (which
    // spilled to scratch); the leaves and the expressions are unchanged.
    const AlphaTEdge eTm = lv.tedge(0, tm), eTp = lv.tedge(1, tp);
    const AlphaSEdge eSm = lv.sedge(0, Sm), eSp = lv.sedge(1, Sp);
    const double Lmt = eTm.Lm1, Lmp = eTp.Lm1;
    const double lSm = eSm.lS, lSp = eSp.lS;
    double at, au, atu = 0., ast;
    if (maj) {
        {
            double D, B;
            if (pre) { D = pre->Dt; B = pre->Bt; }
            else alpha_bracket_t(lv, Sm, Sp, tm, tp, m4, D, B);
            at = g4 / D * B;
            if (at < 0) at = gl33_rect(0, tp, tm, Sm, Sp) * (g4 / (16 * kPi * m4));
            at *= uk;
            tot += wgt * at;
            au = at;
            tot += wgt * au;
        }
        NUSI_PHASE();
        {
            double D, B;
            if (pre) { D = pre->Dtu; B = pre->Btu; }
            else alpha_bracket_tu(lv, Sm, Sp, tm, tp, m4, D, B);
            atu = g4 / D * B;
            // nuSIprop.hpp:1401-1418: the fallback assigns a shadowing local; a negative alpha_tu stays.
            atu *= uk;
            tot += wgt * atu;
        }
        NUSI_PHASE();
        {
            // s-t interference: eight complex dilogarithms (nuSIprop.hpp:1431-1451)
            const AlphaCorner cmm = lv.corner(0, 0, Sm, tm), cpm = lv.corner(1, 0, Sp, tm);
            const AlphaCorner cmq = lv.corner(0, 1, Sm, tp), cpq = lv.corner(1, 1, Sp, tp);
            const AlphaSEdge fSm = lv.sedge(0, Sm), fSp = lv.sedge(1, Sp);
            const AlphaTEdge fTm = lv.tedge(0, tm), fTp = lv.tedge(1, tp);
            const double Lmm = cmm.L, Lpm = cpm.L, Lmq = cmq.L, Lpq = cpq.L;
            const double lSm = fSm.lS, lSp = fSp.lS, Lmt = fTm.Lm1, Lmp = fTp.Lm1;
            const double Lsm = fSm.Ls, Lsp = fSp.Ls;
            const double cm = fTm.cm, cp = fTp.cm;
            const double L2m = fTm.L2, L2p = fTp.L2;
            const double am = fTm.am, ap = fTp.am;
            ast = P.a_st *
                  (2 * gr * (cmm.Dri - cmm.Dci - cpm.Dri + cpm.Dci - cmq.Dri + cmq.Dci + cpq.Dri - cpq.Dci)
                   - 2 * (cmm.Drr - cmm.Dcr - cpm.Drr + cpm.Dcr - cmq.Drr + cmq.Dcr + cpq.Drr - cpq.Dcr)
                   + 2 * gr * (cm - cmm.A) * Lmm
                   - 2 * gr * (cm - cpm.A) * Lpm
                   + 2 * gr * (cp - cpq.A) * Lpq
                   - 2 * gr * (cp - cmq.A) * Lmq
                   + 2 * (gr * fSm.cS - gr * fSp.cS + Lsp / 2. - Lsm / 2. + lSm - lSp) * (2 * (tm - tp) + (Lmt - Lmp))
                   + Lmm * (Lsm - L2m - 2 * (lSm - am)) - Lpm * (Lsp - L2m - 2 * (lSp - am))
                   - Lmq * (Lsm - L2p - 2 * (lSm - ap)) + Lpq * (Lsp - L2p - 2 * (lSp - ap)));
        }
        NUSI_PHASE();
    } else {
        const double brk = -((tm - tp) * (2 + tm * (-1 + tp) - tp)) - 2 * (-1 + tm) * (-1 + tp) * (Lmt - Lmp);
        at = 3. / 2. * g4 / (32 * kPi * m4 * Sm * Sp * (-1 + tm) * (-1 + tp)) * (Sm - Sp) * brk;
        if (at < 0) at = gl33_rect(1, tp, tm, Sm, Sp) * (3. / 2. * g4 / (32 * kPi * m4));
        at *= uk;
        tot += wgt * at;
        au = 1. / 2. * g4 / (32 * kPi * m4 * Sm * Sp * (-1 + tm) * (-1 + tp)) * (Sm - Sp) * brk;
        if (au < 0) au = gl33_rect(1, tp, tm, Sm, Sp) * (1. / 2. * g4 / (32 * kPi * m4));
        au *= uk;
        tot += wgt * au;
        tot += wgt * atu;   // alpha_tu = 0 for Dirac
        const double Lsm = eSm.Ls, Lsp = eSp.Ls;
        ast = P.a_st *
              ((2 * gr * eSm.cS - 2 * gr * eSp.cS + 2 * lSm - 2 * lSp + Lsp - Lsm) * (tm - tp + Lmt - Lmp));
    }
    ast *= uk;
    tot += wgt * ast;
    const double asu = maj ? ast : 0.;
    tot += wgt * asu;

    double app = 0.0;
    if (kPhiPhi && Sm > 4 && P.phiphi)   // ppt: the term shared by a batch (alpha_k_pp)
    {
        PPTerm X;
        if (ppt) X = *ppt;
        else {
            X = alpha_phiphi_core(spl, Sm, Sp, tm, tp, lSm, lSp);
            warn |= X.oob;
        }
        app = alpha_phiphi_scale(P, uk, X);
    }
    tot += wgt * app;

    const double nrm = P.a_nrm;
    // the reference's roundoff checks (:1505); every quotient needs a negative numerator (nrm > 0),
    // so the divisions are only evaluated when one is
    const double sst = ast + as + at;
    if (as < 0 || ((at < 0 || au < 0 || atu < 0 || sst < 0) &&
                   (at / nrm < -1e-11 || au / nrm < -1e-11 || atu / nrm < -1e-11 || sst / nrm < -1e-11)))
        warn |= kWarnAlpha;
}

template <bool kRef = false>
NUSI_FN double alpha_entry(const Point& P, const SplineSet& spl, double Em, double Ep, double Emp, double Epp, int& warn)
{
    const DirectLeavesT<kRef> lv{P.Ga / P.mphi, (P.Ga / P.mphi) * (P.Ga / P.mphi), P.mphi, P.Ga};
    double tot = 0;
    NUSI_MASS_LOOP
    for (int k = 0; k < 3; ++k) alpha_k(P, spl, k, Em, Ep, Emp, Epp, lv, tot, warn);
    return tot;
}

}  // namespace nusi
