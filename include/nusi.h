/*
 * nusi.h -- C ABI of the MI355X-native nuSIprop cascade solver (libnusi.so).
 *
 * Drop-in boundary for the reference's calculate_flux / pyprop surface
 * (quarkquartet/nuSIprop @ 2025-02-13).  Plain C types only: pointers, sizes,
 * ints and doubles.  Every function returns 0 on success or a negative
 * NUSI_E* code; nusi_last_error() gives the message (thread-local).  Nothing
 * in the library calls exit(): the C++ facade (include/nuSIprop.hpp) maps
 * errors back to the reference's stderr text + exit(1).
 *
 * Two levels:
 *   1. object API -- one parameter point, host-side results, the exact
 *      semantics of nuSIprop::calculate_flux (each entry cites the member it
 *      replaces, nuSIprop.hpp:line);
 *   2. plan API   -- a batch of parameter points sharing one energy/redshift
 *      grid, evolved on one GPU with device-resident inputs/outputs (the
 *      MI355X throughput path; multi-GPU = one plan per device, no
 *      collectives).
 * All arithmetic is IEEE fp64.  The table build and the cascade run as HIP
 * kernels on the GPU; there is no CPU fallback -- without a usable GPU the
 * calls fail with NUSI_EHIP.
 */
#ifndef NUSI_H
#define NUSI_H

#ifdef __cplusplus
extern "C" {
#endif

/* error codes */
#define NUSI_OK 0
#define NUSI_EPARAM -1        /* bad parameters / range                          */
#define NUSI_ENOSPECTRUM -2   /* no neutrino mass spectrum (aux.hpp:48-49)       */
#define NUSI_ETABLE -3        /* phi-phi table missing (interp.hpp:251-254)      */
#define NUSI_EINTERP -4       /* phi-phi lookup out of bounds (interp.hpp:355-361) */
#define NUSI_EHIP -5          /* HIP runtime error / no GPU                      */
#define NUSI_ESTATE -6        /* call order (e.g. results before evolve)         */

/* source models.  DSNB is the reference's active Lum (nuSIprop.hpp:659-662);
 * POWER_LAW is its commented-out power law (nuSIprop.hpp:656) used by the
 * BASELINE workloads. */
#define NUSI_SOURCE_DSNB 0
#define NUSI_SOURCE_POWER_LAW 1

/* warning bits (negative cross sections, nuSIprop.hpp:909-918, 1215-1231, 1505-1516) */
#define NUSI_WARN_GAMMA 1
#define NUSI_WARN_ALPHATILDE 2
#define NUSI_WARN_ALPHA 4

/* All constructor arguments of calculate_flux (nuSIprop.hpp:61-65), in order,
 * plus the source model.  Defaults of the reference C++ constructor:
 * norm=1, majorana=1, non_resonant=1, normal_ordering=1, N_bins_E=300,
 * lEmin=12, lEmax=17, zmax=5, flav=2, phiphi=0 (see nusi_params_default). */
typedef struct nusi_params {
    double mphi;        /* mediator mass [eV]                      */
    double g;           /* coupling                                */
    double mntot;       /* sum of neutrino masses [eV]             */
    double si;          /* spectral index                          */
    double norm;        /* free-streaming normalisation at 100 TeV */
    int majorana;
    int non_resonant;
    int normal_ordering;
    int N_bins_E;
    double lEmin;
    double lEmax;
    double zmax;
    int flav;           /* 0=e 1=mu 2=tau */
    int phiphi;
    int source_model;   /* NUSI_SOURCE_* */
} nusi_params;

/* Fills the reference C++ constructor defaults (nuSIprop.hpp:61-65) around
 * the four mandatory parameters; source_model = NUSI_SOURCE_DSNB. */
void nusi_params_default(nusi_params *p, double mphi, double g, double mntot, double si);

const char *nusi_last_error(void);
int nusi_device_count(void);

/* ---------------------------------------------------------------------------
 * 1. object API  (nuSIprop::calculate_flux)
 * ------------------------------------------------------------------------- */
typedef struct nusi_handle nusi_handle;

/* calculate_flux(mphi, g, mntot, si, norm, ...)   nuSIprop.hpp:61-171.
 * Builds the energy/redshift grid and the mixing matrix.  With
 * non_resonant && phiphi the phi-phi tables are loaded like the reference,
 * from xsec/alphatilde_phiphi.bin and xsec/alpha_phiphi.bin relative to the
 * current directory (or $NUSI_XSEC_DIR), -> NUSI_ETABLE if missing.
 * The object evolves on GPU `$NUSI_DEVICE` (default 0) with the default
 * (NUSI_CASCADE_AUTO) kernels. */
int nusi_create(const nusi_params *p, nusi_handle **out);
/* copy constructor / operator=  (nuSIprop.hpp:434-525) */
int nusi_copy(const nusi_handle *src, nusi_handle **out);
void nusi_destroy(nusi_handle *h);
/* the public members mphi, g, mntot, si, norm  (nuSIprop.hpp:174) */
int nusi_set_params(nusi_handle *h, double mphi, double g, double mntot, double si, double norm);
int nusi_get_params(const nusi_handle *h, double *mphi_g_mntot_si_norm /* [5] */);
/* evolve()  (nuSIprop.hpp:176-337) */
int nusi_evolve(nusi_handle *h);
/* check_energy_conservation()  (nuSIprop.hpp:339-357): calls evolve() */
int nusi_check_energy_conservation(nusi_handle *h, double *out);
/* results of the last evolve(), row-major [k][b] (mass basis) / [f][b] (flavour) */
int nusi_get_flux(const nusi_handle *h, double *out_3xN);      /* get_flux(i,j)     :359-381 */
int nusi_get_flux_fla(const nusi_handle *h, double *out_3xN);  /* get_flux_fla(i,j) :383-405 */
int nusi_get_energies(const nusi_handle *h, double *out_N);    /* get_energy(i)     :412-429 */
int nusi_get_N_bins_E(const nusi_handle *h);                   /* get_N_bins_E()    :407-410 */
int nusi_get_N_steps_z(const nusi_handle *h);
int nusi_get_warnings(const nusi_handle *h);                   /* NUSI_WARN_* of the last evolve */
/* names of the alpha-table and cascade kernels this object's last evolve() launched (strings owned by the object,
 * valid until its next evolve() or nusi_destroy; a nusi_copy keeps its source's names); no reference
 * counterpart -- reports and tests) */
int nusi_get_kernels(const nusi_handle *h, const char **alpha, const char **cascade);
/* nusi_plan_set_option on the object's plan (NUSI_OPT_*; kept by nusi_copy).  No reference counterpart. */
int nusi_set_option(nusi_handle *h, int option, int value);

/* ---------------------------------------------------------------------------
 * 2. plan API -- batched parameter scans on one GPU
 * ------------------------------------------------------------------------- */
typedef struct nusi_plan nusi_plan;

/* One plan = one device, one grid (N_bins_E, lEmin, lEmax, zmax), room for
 * max_points points per call (tables for all of them stay in HBM). */
int nusi_plan_create(int device, int N_bins_E, double lEmin, double lEmax, double zmax, int max_points,
                     nusi_plan **out);
void nusi_plan_destroy(nusi_plan *plan);
/* Load the phi-phi tables (float32 records {x0..x_{d-1}, f}, last index
 * fastest; interp.hpp:249-291).  dims == NULL -> the reference's
 * {5000,100} and {1000,1000,100} (nuSIprop.hpp:168-169). */
int nusi_plan_load_phiphi(nusi_plan *plan, const char *alphatilde_path, const int *alphatilde_dims,
                          const char *alpha_path, const int *alpha_dims);
int nusi_plan_grid(const nusi_plan *plan, int *N, int *Nz, double *Enu /* [N] or NULL */);
/* Evolve n points (their grid fields must equal the plan's).  d_flux /
 * d_flux_fla are DEVICE pointers of n*3*N doubles ([point][k][b]); either may
 * be NULL.  stream is a hipStream_t (NULL = the plan's own stream).  The call
 * is asynchronous w.r.t. the host except for the small host->device copy of
 * the per-point constants; results are ready when the stream is. */
int nusi_plan_evolve(nusi_plan *plan, const nusi_params *pts, int n, double *d_flux, double *d_flux_fla, void *stream);
/* Same with host result buffers; synchronous. */
int nusi_plan_evolve_host(nusi_plan *plan, const nusi_params *pts, int n, double *flux, double *flux_fla);
/* Kernel times (ms) of the last nusi_plan_evolve*: [0] Gamma/alphaTilde
 * tables, [1] alpha table, [2] cascade.  Synchronises the plan's stream. */
int nusi_plan_stage_ms(nusi_plan *plan, float *ms3);
/* Kernel-time accounting over many calls (bench): after profile_begin, each
 * nusi_plan_evolve records HIP events around its three kernels on the launch
 * stream (up to max_calls calls); profile_end synchronises and returns the
 * summed ms per stage and the number of calls recorded. */
int nusi_plan_profile_begin(nusi_plan *plan, int max_calls);
int nusi_plan_profile_end(nusi_plan *plan, double *sum_ms3, int *ncalls);
/* Cascade kernel of the plan's later calls.  Every kind meets the same flux
 * tolerance against the reference algorithm (<= 1e-11 relative, the same
 * exact zeros); the choice is a performance / cross-check knob:
 * AUTO (default, also for the object API) = MFMA.
 * MFMA = the block-synchronous wavefront with the push on the fp64 matrix
 *   cores (k_cascade_bs: one pass up to 48 redshift steps, step passes
 *   beyond), for both sources and both scattering modes; points sharing a
 *   Stage-A table share one workgroup (multi-RHS: pairs, or the gamma batch
 *   of up to 16).  Grids beyond its limits (T - 1 > 14 x 128 rows) fall back
 *   to the scalar kernel.
 * WAVEFRONT, REG, LDS = the bit-exact scalar cascade k_cascade (one
 *   wavefront per point, any N; right-looking fma()s in one fixed order).
 *   The three names are kept for the API; since round 5 they select the same
 *   kernel.
 * NUSI_EPARAM for an unknown kind. */
#define NUSI_CASCADE_AUTO 0
#define NUSI_CASCADE_WAVEFRONT 1
#define NUSI_CASCADE_REG 2
#define NUSI_CASCADE_LDS 3
#define NUSI_CASCADE_MFMA 4
int nusi_plan_set_cascade(nusi_plan *plan, int kind);
/* Explicit A/B and test options of a plan (no reference counterpart).  The
 * defaults are the production choices, and nothing in the library reads the
 * environment to select kernels.  NUSI_EPARAM for an unknown option or value.
 *   NUSI_OPT_ALPHA_BATCH   max tables per alpha batch (tables sharing m_phi,
 *                          masses and flags), 1..255; 0 = automatic
 *   NUSI_OPT_ALPHA_KERNEL  0 = k_alpha_batch (default), 1 = k_alpha_tile
 *                          batches of <= 4, 2 = one entry per work-item
 *                          (all three give the same tables bit for bit)
 *   NUSI_OPT_CASCADE_RHS   max points sharing a table per MFMA-cascade
 *                          workgroup: 0 = automatic (the gamma batch for
 *                          tables with >= 3 points, pairs for two), 1 = one
 *                          point each, 2 = pairs (k_cascade_bs_pairs),
 *                          3..16 = the gamma batch k_cascade_bs_gamma (the
 *                          points of a table, gamma on the MFMA N
 *                          dimension) of up to that many.  The MFMA sums in
 *                          blocks of four columns, so a point's fluxes depend
 *                          on its grouping to rounding (<= 1e-13), not bit for
 *                          bit; 1 makes them independent of the call's other
 *                          points
 *   NUSI_OPT_STEP_PASSES   0 = automatic (step passes beyond 48 redshift
 *                          steps), 1 = always the step-pass instance (one
 *                          point per workgroup)
 *   NUSI_OPT_SHIFT_REUSE   opt-in scan mode, K in
 *                          [0, 128]; 0 = off (default).  alpha / Gamma /
 *                          alphaTilde see the energies only through
 *                          2 m_k E / m_phi^2 (nuSIprop.hpp:1253-1256), so the
 *                          tables of m_phi' = m_phi r^(-o/2) (r = Emax[0] /
 *                          Emin[0], integer o) equal those of m_phi read o
 *                          bins higher.  Tables of one (g, masses, flags)
 *                          whose m_phi lie on that lattice within K bins of
 *                          the largest are served by ONE table set of the
 *                          largest m_phi on the axis extended by K bins.  Not
 *                          bit-exact: the bin edges round differently, and the
 *                          flux's optical depth amplifies that with the
 *                          coupling, so only tables with g <= 0.05 share
 *                          (measured <= 8.8e-10 relative there; 3e-8 at g = 1
 *                          had they shared; tests/test_shift_reuse.py); the
 *                          default path is unchanged. */
#define NUSI_OPT_ALPHA_BATCH 1
#define NUSI_OPT_ALPHA_KERNEL 2
#define NUSI_OPT_CASCADE_RHS 3
#define NUSI_OPT_STEP_PASSES 4
#define NUSI_OPT_SHIFT_REUSE 5
/*   NUSI_OPT_REFERENCE_ORDER  1 (DEFAULT, plans and objects) = build Gamma /
 *                          alphaTilde / alpha in the reference's own
 *                          arithmetic: every gsl_sf_dilog /
 *                          gsl_sf_complex_dilog_xy_e call site by GSL's own
 *                          algorithms (dilog.c restated, nusi_gsl.hpp), and
 *                          the alpha table's s-t interference member leaves
 *                          as the dilogarithm of the reference's quotient
 *                          (1+S+t)/(2 - i gr + t) and carg of its expression
 *                          (nuSIprop.hpp:1428-1467, 843-878, 1135-1192).
 *                          Fluxes <= 1e-11 of the GSL-restating oracle on
 *                          every tested config.
 *                          0 = opt-in fast mode, the shared-algorithm order
 *                          (Bernoulli series, batch-shared Taylor
 *                          coefficients; ~3x faster Stage A).  Bit-identical
 *                          to the oracle's default mode, but where the closed
 *                          forms cancel it differs from the reference's
 *                          arithmetic by up to 2.5e-6 (C2a) / 1.3e-7 (C4 at
 *                          g = 1) in a flux. */
#define NUSI_OPT_REFERENCE_ORDER 6
/*   NUSI_OPT_CASCADE_SYNC  the MFMA cascade's synchronisation: 0 = automatic
 *                          = 2 = the block-synchronous kernel k_cascade_bs
 *                          (every wave meets twice per block of four
 *                          stages).  1 (the per-stage kernels k_cascade_ws /
 *                          gb / wsp of rounds 2-3) is refused: those kernels
 *                          were removed in round 5. */
#define NUSI_OPT_CASCADE_SYNC 7
/*   NUSI_OPT_REFO_CORNER_MB  the reference-order big-batch kernel's member-
 *                          corner block (per table and pair of bin edges,
 *                          Dc = Li2(quotient) as re/im for each of the 3
 *                          mass states: 6 doubles, 3.7 MB per table at
 *                          N_E = 300): at most this many MiB, the batches run
 *                          in chunks that fit (at least one batch); 0 =
 *                          automatic (8 GiB, at most half the free memory).
 *                          Any value gives the same tables bit for bit. */
#define NUSI_OPT_REFO_CORNER_MB 8
int nusi_plan_set_option(nusi_plan *plan, int option, int value);
/* per-point NUSI_WARN_* bits of the last call */
int nusi_plan_warnings(nusi_plan *plan, int *out, int n);
/* Names of the main alpha-table and cascade kernels the last call launched (static strings, e.g.
 * "k_alpha_batch", "k_cascade_bs"); for reports -- bench.py's roofline lines.  No reference
 * counterpart. */
int nusi_plan_kernels(const nusi_plan *plan, const char **alpha, const char **cascade);
/* Copy point `i`'s Stage-A tables of the last call to the host (parity
 * tests): Gamma[T], alphaTilde[T], alpha packed transposed [T(T-1)/2] with
 * alpha(n,m), n<m, at m(m-1)/2+n.  Any pointer may be NULL. */
int nusi_plan_tables(nusi_plan *plan, int i, double *Gamma, double *alphaTilde, double *alpha_packed);

/* Convenience: evolve n points on `device` with host buffers (creates a
 * transient plan; points must share the grid). */
int nusi_evolve_batch(int device, const nusi_params *pts, int n, double *flux, double *flux_fla);

#ifdef __cplusplus
}
#endif
#endif /* NUSI_H */
