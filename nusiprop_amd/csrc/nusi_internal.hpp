// nuSIprop MI355X -- internal interfaces between the C-ABI host layer and the kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

#include "nusi.h"
#include "nusi_physics.hpp"

namespace nusi {

// Grid shared by every point of a batch (constructor, nuSIprop.hpp:113-128, and
// the table axis of evolve(), nuSIprop.hpp:224-233).  Device pointers.
struct GridDev {
    int N, Nz, T;
    long long PT;          // alpha entries per point = T(T-1)/2
    const double* Emin;    // [N]
    const double* Emax;    // [N]
    const double* lo;      // [T] table-axis bin edges
    const double* hi;      // [T]
    const double* z;       // [Nz]
    const double* step_c;  // [Nz] c_i = (1+z[i-1]) dlogz / H(z[i-1]), index i (0 unused)
    const double* step_s;  // [Nz] s_i = n_nu(z[i-1]) / (1+z[i-1])^2
    const double* sfr;     // [Nz] get_SFR(z[i])
};

// Device tables of one batch.  alpha is stored transposed and packed:
// alpha(n, m), n < m, lives at m(m-1)/2 + n, so that the cascade's column
// reads (all n < m for one m) are contiguous.
struct TablesDev {
    double* G;    // [npts][T]
    double* At;   // [npts][T]
    double* A;    // [npts][PT]
    double* Med;  // [npts][3][kMedFields T]: member edge leaves of every bin edge (k_alpha_medge)
    double* Src;  // [npts][T (Nz-1)]: DSNB source terms c_i Lum (k_source_dsnb, diagonal layout), or nullptr
    int* Wmin;    // [npts][4][T] or nullptr (only the base plan of NUSI_OPT_SHIFT_REUSE): per warning bit b and table
                  // row n, the smallest column m of an entry (n, m) that raised it (Gamma / alphaTilde: m = n), so
                  // that k_table_shift passes on exactly the warnings of the rows a shifted slot reads
    double* Kt = nullptr;   // [npts][3][PT][8] or nullptr: the k-split alpha path of calls of few tables
                            // (launch_alpha): each mass state's terms of every entry, summed in order by k_alpha_ksum
    double* Gpre = nullptr;   // [npts][3][kGaPreFields][T] or nullptr: the reference order's Gamma / alphaTilde
                              // dilogarithms of calls of few tables (k_ga_dilogs, launch_gamma_alphat)
};

// Tiles of the alpha table for k_alpha_tile: kAlphaTile x kAlphaTile (n, m) bin blocks with
// tn <= tm, in three launch classes by how many distinct bin edges a side has
// (bins of the first N share edges, redshift-extended bins do not), which sets
// each class's LDS footprint.  tiles[] packs tn | tm << 16.
struct AlphaTilesDev {
    int* tiles = nullptr;   // device [ncore + nmixed + nfull]
    int ncls[3] = {0, 0, 0};
    int cs_max[3] = {0, 0, 0}, ct_max[3] = {0, 0, 0};
    int ext_lo = 0;          // bins [ext_lo, T) x [ext_lo, T) are built by the per-entry kernel
};
// Classify the tiles of a grid on the host; `shared[n]` = (hi[n] == lo[n+1]) bitwise.
hipError_t alpha_tiles_create(int T, const unsigned char* shared, AlphaTilesDev* out);
void alpha_tiles_destroy(AlphaTilesDev* t);

// NUSI_OPT_REFERENCE_ORDER on the big-batch kernel: the member corners (Dc, A of alpha_member_ref) of every table, mass
// state and corner, evaluated by k_alpha_mcorner before k_alpha_batch reads them.  A corner is a pair of distinct bin
// edges (S' edge us, t edge ut <= us; the edges numbered 0 .. U-1 along the table axis, an edge two neighbouring bins
// share counted once): c = us (us + 1) / 2 + ut, NC = U (U + 1) / 2.  The block of a batch of nb tables starting at
// slot p0 is buf + (p0 - pc0) 6 NC, laid out [k][q][c][Dcr, Dci] (a tile's corner rows contiguous; A = carg(..) is
// formed by the batch kernel); a launch chunk of batches whose tables fit cap_tables starts at table pc0.
struct MCornerDev {
    double* buf = nullptr;   // [cap_tables][3][NC][2]
    int* eu = nullptr;       // [2 T]: edge number of bin edge 2 b + side (side 0: lo[b], 1: hi[b])
    double* ue = nullptr;    // [U]: the energy of each edge
    long long NC = 0;
    int U = 0, cap_tables = 0;
};
// ref: NUSI_OPT_REFERENCE_ORDER (the kernels' kRef instances: the reference's own operation order for the complex
// dilogarithms and the s-t interference member leaves, bit-identical to the oracle's ora_set_reference_order(1))
size_t gamma_alphat_pre_doubles(int T, int npts);   // TablesDev::Gpre's size
hipError_t launch_gamma_alphat(const GridDev& g, const Point* pts, int npts, const SplineSet* spl, TablesDev t,
                               int* warn, hipStream_t s, bool ref);
// batches: device [nbatches] of first table | count << 24 (count <= gmax), tables of a batch sharing
// m_phi, the masses and the channel flags (nullptr: every table alone).  kernel = NUSI_OPT_ALPHA_KERNEL:
// 0 -- core tiles on the big-batch kernel k_alpha_batch (any count < 256; the first nb_plain batches without
// the phi-phi channel, the rest with it); 1 -- k_alpha_tile<G> batches (count <= 4); 2 -- one entry per
// work-item (k_alpha).  h_batches: the same batches in host memory, and mc the member-corner block (both read
// only by kernel 0 with ref: k_alpha_mcorner + k_alpha_batch in chunks of batches of <= mc->cap_tables tables)
hipError_t launch_alpha(const GridDev& g, const Point* pts, int npts, const SplineSet* spl, const AlphaTilesDev& tiles,
                        TablesDev t, int* warn, hipStream_t s, const int* batches, int nbatches, int gmax,
                        int kernel, int nb_plain, bool ref, const int* h_batches = nullptr,
                        const MCornerDev* mc = nullptr);
// the edge numbering of MCornerDev for a table axis (hi[n] == lo[n + 1] bitwise: one edge): eu [2 T], ue [U]
void mcorner_edges(int T, const double* lo, const double* hi, std::vector<int>& eu, std::vector<double>& ue);
// NUSI_OPT_SHIFT_REUSE: tables s0 .. s0 + nshift - 1 of t (grid g) <- base tables map[q].x of tb (grid gb, the
// axis extended on top), read map[q].y bins higher; warn[s] |= the warning bits of the base rows the slot reads
// (tb.Wmin, required)
hipError_t launch_table_shift(const GridDev& g, const GridDev& gb, const int2* map, int s0, int nshift, TablesDev tb,
                              TablesDev t, int* warn, hipStream_t s);
// The block-synchronous MFMA cascade (k_cascade_bs, round 4): workgroup k takes the grp[k].y <= P points gidx[grp[k].x
// ..] that share one table slot (gidx == grp == nullptr: P = 1, point k), P = 1, 2 or 16 (the gamma batch), any source
// and scattering mode, step passes on any grid that fits; fh: a FIFO of cascade_bs_scratch_doubles per workgroup
// (used when the steps take more than one pass).  cascade_bs_config: 0 = the grid does not fit P.
// force_passes (NUSI_OPT_STEP_PASSES = 1, P = 1): the step-pass instance even where one pass fits.
int cascade_bs_config(const GridDev& g, int P, bool force_passes);
size_t cascade_bs_scratch_doubles(const GridDev& g, int P);
hipError_t launch_cascade_bs(const GridDev& g, const Point* pts, int P, const int* gidx, const int2* grp, int nwg,
                             TablesDev t, double* fh, double* flux, double* flux_fla, hipStream_t s, bool all_nr,
                             bool force_passes);
size_t cascade_src_doubles(const GridDev& g);   // t.Src doubles per point
hipError_t launch_source_dsnb(const GridDev& g, const Point* pts, int npts, double* src, hipStream_t s);
// The bit-exact scalar cascade k_cascade (NUSI_CASCADE_WAVEFRONT / REG / LDS all select it): one wavefront per
// point, any N.
hipError_t launch_cascade_exact(const GridDev& g, const Point* pts, int npts, TablesDev t, double* flux,
                                double* flux_fla, hipStream_t s);

// 4 x 4 windows of a 3-D spline table f [n0][n1][n2] into fw [n0 n1 n2][16] (synchronous)
hipError_t spline_windows_build(const float* f, int n0, int n1, int n2, float* fw);

// names of the main alpha-table / cascade kernels the latest launch_alpha / launch_cascade_* on this
// thread chose (static strings; nusi_plan_kernels)
const char* last_alpha_kernel();
const char* last_cascade_kernel();

}  // namespace nusi
