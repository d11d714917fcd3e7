// TEST INFRASTRUCTURE ONLY: compiles the product's device physics headers
// (nusiprop_amd/csrc/nusi_physics.hpp) for the host so that tests/ can check
// the table formulas against the oracle without a GPU.  Never linked into
// libnusi.so; the product runs these functions only inside HIP kernels.
#include <vector>

#include "nusi_physics.hpp"

extern "C" {

// pt: mphi g mntot si norm norm_total Ga mn0 mn1 mn2 u0 u1 u2 ; flags: majorana non_resonant phiphi source
static nusi::Point mk(const double* pt, const int* flags)
{
    nusi::Point P{};
    P.mphi = pt[0]; P.g = pt[1]; P.mntot = pt[2]; P.si = pt[3]; P.norm = pt[4]; P.norm_total = pt[5]; P.Ga = pt[6];
    for (int k = 0; k < 3; ++k) { P.mn[k] = pt[7 + k]; P.u[k] = pt[10 + k]; }
    P.majorana = flags[0]; P.non_resonant = flags[1]; P.phiphi = flags[2]; P.source = flags[3];
    nusi::point_derive(P);
    return P;
}

}  // extern "C"

// ref: the NUSI_OPT_REFERENCE_ORDER instances (kRef)
template <bool kRef>
static int tables_t(const double* pt, const int* flags, int T, const double* lo, const double* hi, double* G, double* At,
                    double* A)
{
    const nusi::Point P = mk(pt, flags);
    nusi::SplineSet spl{};
    int w = 0;
    for (int n = 0; n < T; ++n) {
        G[n] = nusi::gamma_entry<kRef>(P, lo[n], hi[n], w);
        At[n] = nusi::alphat_entry<kRef>(P, spl, lo[n], hi[n], w);
        for (int m = n + 1; m < T; ++m)
            A[(size_t)n * T + m] = nusi::alpha_entry<kRef>(P, spl, lo[n], hi[n], lo[m], hi[m], w);
    }
    return w;
}

extern "C" {

int hc_tables(const double* pt, const int* flags, int T, const double* lo, const double* hi,
              double* G, double* At, double* A /* T*T dense, m>n */)
{
    return tables_t<false>(pt, flags, T, lo, hi, G, At, A);
}
int hc_tables_ref(const double* pt, const int* flags, int T, const double* lo, const double* hi, double* G, double* At,
                  double* A)
{
    return tables_t<true>(pt, flags, T, lo, hi, G, At, A);
}

}  // extern "C"

// Host emulation of k_gamma_alphat's edge-shared path (round 6): every bin's edge dilogarithms by gamma_edge_vals /
// alphat_edge_vals at the bin's own lower and upper edge (the kernel takes the upper edge's from the next lane, which
// evaluates the same function at the same bits), the channels through gamma_k / alphat_k with the pair, summed as the
// kernel's wave 0 sums them.  parts = 1: one pass per mass state (scans); 2: the two channel parts (few tables).
struct SlotSink {
    double* v;
    NUSI_FN void put(int slot, double x, double) { v[slot] = x; }
};
template <bool kRef>
static int ga_shared_t(const double* pt, const int* flags, int T, const double* lo, const double* hi, int parts,
                       double* G, double* At)
{
    using namespace nusi;
    const Point P = mk(pt, flags);
    SplineSet spl{};
    int warn = 0;
    for (int n = 0; n < T; ++n) {
        double g = 0.0, a = 0.0;
        for (int k = 0; k < 3; ++k) {
            double vg[kAlphatSlots] = {}, va[kAlphatSlots] = {};
            SlotSink sg{vg}, sa{va};
            for (int part = (parts == 1 ? -1 : 0); part < (parts == 1 ? 0 : 2); ++part) {
                const unsigned ng = part < 0 ? gamma_edge_need<-1>(P, k, lo[n], hi[n])
                                    : part == 0 ? gamma_edge_need<0>(P, k, lo[n], hi[n]) : gamma_edge_need<1>(P, k, lo[n], hi[n]);
                const unsigned na = part < 0 ? alphat_edge_need<-1>(P, k, lo[n], hi[n])
                                    : part == 0 ? alphat_edge_need<0>(P, k, lo[n], hi[n]) : alphat_edge_need<1>(P, k, lo[n], hi[n]);
                GammaEdgePair ge{};
                AlphatEdgePair ae{};
                gamma_edge_vals<kRef>(P, k, lo[n], ng, ge.lo);
                gamma_edge_vals<kRef>(P, k, hi[n], ng, ge.hi);
                alphat_edge_vals<kRef>(P, k, lo[n], na, ae.lo);
                alphat_edge_vals<kRef>(P, k, hi[n], na, ae.hi);
                if (part < 0) {
                    gamma_k<kRef, -1>(P, k, lo[n], hi[n], sg, warn, &ge);
                    alphat_k<kRef, -1>(P, spl, k, lo[n], hi[n], sa, warn, &ae);
                } else if (part == 0) {
                    gamma_k<kRef, 0>(P, k, lo[n], hi[n], sg, warn, &ge);
                    alphat_k<kRef, 0>(P, spl, k, lo[n], hi[n], sa, warn, &ae);
                } else {
                    gamma_k<kRef, 1>(P, k, lo[n], hi[n], sg, warn, &ge);
                    alphat_k<kRef, 1>(P, spl, k, lo[n], hi[n], sa, warn, &ae);
                }
            }
            const int ng = !P.non_resonant ? 1 : kGammaSlots, na = !P.non_resonant ? 1 : kAlphatSlots;
            for (int i = 0; i < ng; ++i) g += vg[i];
            for (int i = 0; i < na; ++i) a += va[i];
        }
        G[n] = g;
        At[n] = a;
    }
    return warn;
}

// Host emulation of the reference order's few-table path: k_ga_dilogs' slots (ga_pre_slot) into a bin's fields, read
// back by ga_pre_load, the channels through gamma_k / alphat_k in the two parts, summed as the kernel's wave 0 sums them
static int ga_pre_t(const double* pt, const int* flags, int T, const double* lo, const double* hi, double* G, double* At)
{
    using namespace nusi;
    const Point P = mk(pt, flags);
    SplineSet spl{};
    int warn = 0;
    for (int n = 0; n < T; ++n) {
        double g = 0.0, a = 0.0;
        for (int k = 0; k < 3; ++k) {
            double fld[kGaPreFields];
            for (int i = 0; i < kGaPreFields; ++i) fld[i] = __builtin_nan("");
            if (P.non_resonant)
                for (int slot = 0; slot < kGaPreSlots; ++slot) {
                    double v[2];
                    int f;
                    const int nv = ga_pre_slot(P, k, lo[n], hi[n], slot, v, &f);
                    fld[f] = v[0];
                    if (nv == 2) fld[f + 1] = v[1];
                }
            GammaEdgePair ge;
            AlphatEdgePair ae;
            AlphatBinVals bv;
            ga_pre_load(fld, 1, 0, ge, ae, bv);
            double vg[kAlphatSlots] = {}, va[kAlphatSlots] = {};
            SlotSink sg{vg}, sa{va};
            gamma_k<true, 0>(P, k, lo[n], hi[n], sg, warn, &ge);
            gamma_k<true, 1>(P, k, lo[n], hi[n], sg, warn, &ge);
            alphat_k<true, 0>(P, spl, k, lo[n], hi[n], sa, warn, &ae, &bv);
            alphat_k<true, 1>(P, spl, k, lo[n], hi[n], sa, warn, &ae, &bv);
            const int ng = !P.non_resonant ? 1 : kGammaSlots, na = !P.non_resonant ? 1 : kAlphatSlots;
            for (int i = 0; i < ng; ++i) g += vg[i];
            for (int i = 0; i < na; ++i) a += va[i];
        }
        G[n] = g;
        At[n] = a;
    }
    return warn;
}

extern "C" {
int hc_ga_pre(const double* pt, const int* flags, int T, const double* lo, const double* hi, double* G, double* At)
{
    return ga_pre_t(pt, flags, T, lo, hi, G, At);
}
int hc_ga_shared(const double* pt, const int* flags, int T, const double* lo, const double* hi, int parts, int ref,
                 double* G, double* At)
{
    return ref ? ga_shared_t<true>(pt, flags, T, lo, hi, parts, G, At) : ga_shared_t<false>(pt, flags, T, lo, hi, parts, G, At);
}
}  // extern "C"

// Host emulation of k_alpha_tile: the same edge lists, job helpers and TileLeaves combine, one
// tile at a time (work-items run sequentially, phases in kernel order).  alpha dense T*T, m > n.
template <bool kRef>
static int alpha_tiled_t(const double* pt, const int* flags, int T, const double* lo, const double* hi, double* A)
{
    using namespace nusi;
    const Point P = mk(pt, flags);
    SplineSet spl{};
    const int nt = (T + kAlphaTile - 1) / kAlphaTile;
    constexpr int G = 1;   // a batch of one point (the tile kernel's per-table path)
    std::vector<double> sm(alpha_tile_corner_block(2 * kAlphaTile, 2 * kAlphaTile, G) +
                           alpha_tile_edge_doubles(2 * kAlphaTile, 2 * kAlphaTile, G));
    int warn = 0;
    for (int tm = 0; tm < nt; ++tm)
        for (int tn = 0; tn <= tm; ++tn) {
            double tE[2 * kAlphaTile], sE[2 * kAlphaTile];
            int tl[kAlphaTile], th[kAlphaTile], sl[kAlphaTile], sh[kAlphaTile];
            const int n0 = tn * kAlphaTile, m0 = tm * kAlphaTile;
            const int ct = alpha_edge_list(lo, hi, n0, T, tE, tl, th);
            const int cs = alpha_edge_list(lo, hi, m0, T, sE, sl, sh);
            const int cc = cs * ct;
            double* cor = sm.data();
            double* edg = cor + alpha_tile_corner_block(cs, ct, G);
            for (int job = 0; job < 3 * (ct + cs + kAlphaTile); ++job) {
                alpha_tile_edge_job(P, job, tE, ct, sE, cs, lo, hi, m0, T, edg);
                alpha_tile_edge_member_job(P, 0, G, job, tE, ct, sE, cs, lo, hi, m0, T, edg);
            }
            double tot[kAlphaTile * kAlphaTile] = {};
            for (int k = 0; k < 3; ++k) {
                if (P.non_resonant && P.majorana) {
                    const double* edgk = edg + k * alpha_tile_edge_stride(cs, ct);
                    for (int j = 0; j < cc; ++j) {
                        alpha_tile_corner_job<kRef>(j, edgk, ct, cs, cor);
                        alpha_tile_corner_member_job<kRef>(P, 0, j, edgk, ct, cs, cor);
                    }
                    for (int j = 0; j < kAlphaTile * (cs + ct); ++j)
                        alpha_tile_mixed_job(j, edgk, ct, cs, G, tl, th, sl, sh, n0, m0, T, T, cor);
                }
                for (int e = 0; e < kAlphaTile * kAlphaTile; ++e) {
                    const int ln = e % kAlphaTile, lm = e / kAlphaTile, n = n0 + ln, m = m0 + lm;
                    if (!(n < m && m < T) || !(P.non_resonant || m == n + 1)) continue;
                    const TileLeaves lv = alpha_tile_leaves(cor, edg, k, 0, G, cs, ct, lm, sl, sh, tl, th, ln);
                    alpha_k(P, spl, k, lo[n], hi[n], lo[m], hi[m], lv, tot[e], warn);
                }
            }
            for (int e = 0; e < kAlphaTile * kAlphaTile; ++e) {
                const int ln = e % kAlphaTile, lm = e / kAlphaTile, n = n0 + ln, m = m0 + lm;
                if (n < m && m < T) A[(size_t)n * T + m] = tot[e];
            }
        }
    return warn;
}

extern "C" {

int hc_alpha_tiled(const double* pt, const int* flags, int T, const double* lo, const double* hi, double* A)
{
    return alpha_tiled_t<false>(pt, flags, T, lo, hi, A);
}
int hc_alpha_tiled_ref(const double* pt, const int* flags, int T, const double* lo, const double* hi, double* A)
{
    return alpha_tiled_t<true>(pt, flags, T, lo, hi, A);
}

double hc_lum(const double* pt, const int* flags, double z, double sfr_z, double Em, double Ep)
{
    return nusi::lum(mk(pt, flags), z, sfr_z, Em, Ep);
}
double hc_li2(double x) { return nusi::li2(x); }
void hc_cli2(double x, double y, double* re, double* im) { const nusi::cd r = nusi::cli2(x, y); *re = r.r; *im = r.i; }
double hc_li3(double x) { return nusi::li3(x); }
// GSL's algorithms as the device runs them (nusi_gsl.hpp), for the bit-identity test against oracle/ora_gsl.c
double hc_gsl_li2(double x) { return nusi::gsl_li2(x); }
void hc_gsl_cli2(double x, double y, double* re, double* im) { const nusi::cd r = nusi::gsl_cli2(x, y); *re = r.r; *im = r.i; }
double hc_gsl_clausen(double x) { return nusi::gsl::clausen(x); }
double hc_hypot(double x, double y) { return nusi::gsl::hypot(x, y); }
// the libm atan2 the device runs (nusi_libm.hpp: the select-based common path, else fdlibm's branches)
double hc_atan2(double y, double x) { return nusi::nm::atan2_i(y, x); }
// the GPU's inline log / log1p (nusi_libm.hpp: log_i without the c = 0 correction term) on n arguments
void hc_log_n(int n, const double* x, double* out) { for (int i = 0; i < n; ++i) out[i] = nusi::nm::log_i(x[i]); }
void hc_log1p_n(int n, const double* x, double* out) { for (int i = 0; i < n; ++i) out[i] = nusi::nm::log1p_i(x[i]); }
double hc_atan2_full(double y, double x) { return nusi::nm::atan2_full(y, x); }
// the series' per-k table row (d1, d2, y1, y2, l1, l2) and its division, for the two-part-reciprocal test
void hc_gsl_krow(int k, double* o)
{
    const nusi::gsl::KRow& r = nusi::gsl::kKT.row[k];
    o[0] = r.d1; o[1] = r.d2; o[2] = r.y1; o[3] = r.y2; o[4] = r.l1; o[5] = r.l2;
}
double hc_gsl_div_k(double a, double d, double y, double l) { return nusi::gsl::div_k<false>(a, d, y, l); }
}
