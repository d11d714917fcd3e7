/*
 * nuSIprop oracle -- special functions.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load anything under oracle/.  The product path (nusiprop_amd/) never does.
 *
 * The reference calls three third-party functions that are absent from
 * /root/reference:
 *   - GSL gsl_sf_dilog(x)                 (version unpinned; Homebrew build)
 *       aux.hpp:112,129,147,165  nuSIprop.hpp:1098,1202,1375-1398
 *   - GSL gsl_sf_complex_dilog_xy_e(x,y)  aux.hpp:92-93  nuSIprop.hpp:1444-1451
 *   - Expander/polylogarithm Li2(double), Li3(double)  (un-vendored submodule)
 *       nuSIprop.hpp:628-636
 * Their published semantics are restated here (values: fp64 algorithms shared
 * bit for bit with the GPU, see ora_specfun.c):
 *   gsl_sf_dilog(x)             = Re Li2(x) for all real x (x>1 included)
 *   gsl_sf_complex_dilog_xy_e   = principal-branch Li2(x+iy); for y == 0 and
 *                                 x >= 1 GSL returns Im = -pi*log(x)
 *                                 (and Re = gsl_sf_dilog(x)); for y == 0 and
 *                                 x < 1, Im = 0
 *   polylogarithm::Li2 / Li3    = real Li2 / Li3 (only x in [-1,0) reached)
 * Accuracy: within a few ulp of the exact function (GSL quotes ~2 ulp); the
 * *_ld variants (x87 long double, ~0.5 ulp) are an independent yardstick.
 * Both are pinned by mpmath known-answer vectors in tests/golden/specfun_kat.json
 * (tests/test_oracle_specfun.py).
 */
#ifndef NUSI_ORA_SPECFUN_H
#define NUSI_ORA_SPECFUN_H
#ifdef __cplusplus
extern "C" {
#endif

double ora_dilog(double x);                                  /* gsl_sf_dilog */
void ora_complex_dilog_xy(double x, double y, double *re, double *im);
/* reference-order level of the gsl_sf_dilog / gsl_sf_complex_dilog_xy_e call sites (ora_dilog,
 * ora_complex_dilog_xy): 0 = the shared-algorithm series, 1 = GSL's algorithms (ora_gsl.c), 2 = long double */
void ora_cdilog_set_general(int level);
/* GSL's published algorithms restated (ora_gsl.c): gsl_sf_dilog, gsl_sf_complex_dilog_xy_e, gsl_sf_clausen,
 * and the hypot they call; ora_gsl_stats: the series loops' iteration counts of this thread (analysis) */
double ora_gsl_dilog(double x);
void ora_gsl_complex_dilog_xy(double x, double y, double *re, double *im);
double ora_gsl_clausen(double x);
double ora_hypot(double x, double y);
void ora_gsl_stats(long *out, int reset);
/* Li2 about a real point x0 (x0 != 0, 1): coefficients and evaluation at x0 + (dr + i di) on the side
 * `side` (+-1) of the cut x0 > 1; |d| <= ORA_LI2T_RATIO min(|x0|, |1 - x0|) */
#define ORA_LI2T_TERMS 6
#define ORA_LI2T_RATIO 2.5e-3
typedef struct { double c[ORA_LI2T_TERMS + 1]; double r, b0; } ora_li2t;
void ora_li2_taylor_coeffs(double x0, ora_li2t *T);
void ora_li2_taylor_eval(const ora_li2t *T, double dr, double di, double side, double *re, double *im);
double ora_li2(double x);                                    /* polylogarithm::Li2 */
double ora_li3(double x);                                    /* polylogarithm::Li3, x in [-1,0.5] */
/* long-double yardsticks (tests only) */
double ora_dilog_ld(double x);
void ora_complex_dilog_xy_ld(double x, double y, double *re, double *im);
double ora_li3_ld(double x);

#ifdef __cplusplus
}
#endif
#endif
