/*
 * nuSIprop CPU oracle -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C99 restatement of the reference's calculate_flux (nuSIprop.hpp,
 * aux.hpp, interp.hpp) used by tests/ (as the parity checker),
 * __graft_entry__.smoke() (checker) and bench.py's cpu_baseline leg.  Nothing
 * in nusiprop_amd/ links, loads or calls it.
 *
 * Pinning: tests/test_oracle_golden.py reproduces the reference's only golden
 * data, output/data_massless.txt (test.py's run), to its printed precision;
 * the special functions are pinned by mpmath KATs (tests/golden/specfun_kat.json);
 * the t/u/t-u channel closed forms are checked against numerical quadrature
 * of the reference's own integrands (tests/test_oracle_quadrature.py).
 */
#ifndef NUSI_ORACLE_H
#define NUSI_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    double mphi, g, mntot, si, norm;
    int majorana, non_resonant, normal_ordering;
    int N_bins_E;
    double lEmin, lEmax, zmax;
    int flav, phiphi;
    int source;            /* 0 = DSNB (reference active Lum, nuSIprop.hpp:659)
                              1 = power law (reference commented Lum, nuSIprop.hpp:656) */
} ora_params;

typedef struct ora_state ora_state;

ora_state *ora_create(const ora_params *p, int *err);
void ora_destroy(ora_state *S);
int ora_set_params(ora_state *S, double mphi, double g, double mntot, double si, double norm);
int ora_load_phiphi(ora_state *S, const char *alphatilde_path, const char *alpha_path);
/* same with caller-chosen node counts (synthetic tables in the reference layout) */
int ora_load_phiphi_dims(ora_state *S, const char *at_path, const int *n2, const char *a_path, const int *n3);

/* Test hook (process-wide, not thread-safe; 0 by default): 1 = reference-order arithmetic in the alpha
 * table's s-t interference -- the general complex dilog of the reference's quotient and carg of its
 * expression (nuSIprop.hpp:1431-1456), no member Taylor path, no near-axis shortcut in any complex dilog;
 * 2 = the same with every complex dilog evaluated in long double (precision probe) */
void ora_set_reference_order(int level);

int ora_N(const ora_state *S);
int ora_Nz(const ora_state *S);
int ora_T(const ora_state *S);
void ora_grid(const ora_state *S, double *Emin, double *Emax, double *Enu, double *z);
void ora_mixing(const ora_state *S, double *U2 /* 3x3 |U_fk|^2 row-major */);
double ora_zmax(const ora_state *S);

/* per-evolve derived quantities (masses, norm_total) -- nuSIprop.hpp:184-205 */
int ora_prepare(ora_state *S);
void ora_masses(const ora_state *S, double *mn3, double *norm_total);

/* Stage A tables (nuSIprop.hpp:217-253); alpha is T*T row-major, only m>n filled */
int ora_tables(ora_state *S, double *Gamma, double *alphaTilde, double *alpha);
/* single entries (for KAT-style tests) */
double ora_Gamma(ora_state *S, double Em, double Ep);
double ora_alphaTilde(ora_state *S, double Em, double Ep);
double ora_alpha(ora_state *S, double Em, double Ep, double Emp, double Epp);

/* Stage B + finalise on given tables (nuSIprop.hpp:255-336) */
int ora_cascade(ora_state *S, const double *Gamma, const double *alphaTilde, const double *alpha,
                double *flux /*3N*/, double *flux_fla /*3N*/);
/* full evolve() */
int ora_evolve(ora_state *S, double *flux, double *flux_fla);
/* source term integral Lum(z, Em, Ep) (nuSIprop.hpp:656/659) */
double ora_Lum(const ora_state *S, double z, double Em, double Ep);
double ora_check_energy_conservation(ora_state *S, double *flux, double *flux_fla);
/* warnings emitted (negative cross sections), bitmask 1=Gamma 2=alphaTilde 4=alpha */
int ora_warnings(const ora_state *S);

/* Test hooks for the closed-form KATs (tests/test_oracle_quadrature.py).
 * ora_set_channels: Gamma / alphaTilde / alpha sum only the masked channels
 * (default ORA_CH_ALL).  Gamma's combined t+u term (nuSIprop.hpp:797) follows
 * ORA_CH_T; ORA_CH_U selects the separate u terms of alphaTilde / alpha. */
#define ORA_CH_S 1
#define ORA_CH_T 2
#define ORA_CH_U 4
#define ORA_CH_TU 8
#define ORA_CH_ST 16
#define ORA_CH_SU 32
#define ORA_CH_PP 64
#define ORA_CH_ALL 127
void ora_set_channels(ora_state *S, int mask);
/* the bracket of the analytic double-scalar absorption, nuSIprop.hpp:885 (a = max(s-, 4)):
 * Gamma_pp = g^4 / (128 pi mphi^2) * ora_Gpp_bracket(a, s+) per mass state */
double ora_Gpp_bracket(double a, double b);

#ifdef __cplusplus
}
#endif
#endif
