// nuSIprop MI355X -- C ABI (include/nusi.h): host set-up, plans, object API.
//
// Host work here is the reference's per-object scalar set-up only (grid,
// mixing matrix, masses, normalisation; nuSIprop.hpp:102-171, 184-205) and
// the energy-conservation diagnostic; the table build and the cascade run
// on the GPU (nusi_kernels.hip).  There is no CPU fallback.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <tuple>
#include <array>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <sys/stat.h>
#include <string>
#include <utility>
#include <vector>

#include "nusi.h"
#include "nusi_internal.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

#define HIPCHECK(x)                                                                              \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) return fail(NUSI_EHIP, std::string("HIP error: ") + hipGetErrorString(e_) + " (" #x ")"); \
    } while (0)

inline double sq(double a) { return a * a; }
inline double cu(double a) { return a * a * a; }

// ---------------------------------------------------------------------------
// grid: constructor nuSIprop.hpp:113-128, table axis :224-233, per-step
// scalars of the cascade :256-259, 268-269, 283
// ---------------------------------------------------------------------------
struct HostGrid {
    int N = 0, Nz = 0, T = 0;
    double lEmin = 0, lEmax = 0, zmax_in = 0, zmax_eff = 0;
    std::vector<double> Emin, Emax, Enu, z, lo, hi, step_c, step_s, sfr;
};

double hubble_h(double z) { return 1.5e-33 * pow(0.692 + 0.308 * cu(1 + z), 0.5); }
double n_nu_h(double z) { return 4.3528e-13 * cu(1 + z); }
double sfr_h(double z)
{
    return pow(pow(1 + z, -3.4 * 10) + pow((1 + z) / 5161, 0.3 * 10) + pow((1 + z) / 9.06, 3.5 * 10), -1. / 10.);
}

HostGrid make_grid(int N, double lEmin, double lEmax, double zmax)
{
    HostGrid G;
    G.N = N;
    G.lEmin = lEmin;
    G.lEmax = lEmax;
    G.zmax_in = zmax;
    G.Emin.resize(N);
    G.Emax.resize(N);
    G.Enu.resize(N);
    for (int i = 0; i < N; ++i) {
        G.Emin[i] = pow(10, lEmin + (lEmax - lEmin) * (i * 1.0) / N);
        G.Enu[i] = pow(10, lEmin + (lEmax - lEmin) * (i + 0.5) / N);
        G.Emax[i] = pow(10, lEmin + (lEmax - lEmin) * (i + 1.0) / N);
    }
    G.Nz = (int)(log((1 + zmax) / (1 + 0)) / log(G.Emax[0] / G.Emin[0]) + 2);
    G.z.resize(G.Nz);
    for (int i = 0; i < G.Nz; ++i) G.z[i] = (1 + 0) * pow(G.Emax[0] / G.Emin[0], i) - 1;
    G.zmax_eff = G.z[G.Nz - 1];
    G.T = N + G.Nz - 2;
    G.lo.resize(G.T);
    G.hi.resize(G.T);
    for (int n = 0; n < G.T; ++n) {
        if (n < N) {
            G.lo[n] = G.Emin[n];
            G.hi[n] = G.Emax[n];
        } else {
            G.lo[n] = G.Emin[N - 1] * (1 + G.z[n - N + 1]);
            G.hi[n] = G.Emax[N - 1] * (1 + G.z[n - N + 1]);
        }
    }
    G.step_c.assign(G.Nz, 0.0);
    G.step_s.assign(G.Nz, 0.0);
    const double dlogz = log(1 + G.z[1]) - log(1 + G.z[0]);
    for (int i = 1; i < G.Nz; ++i) {
        const double zz = G.z[i - 1];
        G.step_c[i] = (1 + zz) * dlogz / hubble_h(zz);
        G.step_s[i] = n_nu_h(zz) / sq(1 + zz);
    }
    G.sfr.resize(G.Nz);
    for (int i = 0; i < G.Nz; ++i) G.sfr[i] = sfr_h(G.z[i]);
    return G;
}

// |U_fk|^2 from NuFIT 5.0 angles, nuSIprop.hpp:130-163.  Only std::norm(U)
// is used by the reference; the complex entries are formed with explicit real
// operations (real*complex component-wise, s13/del by Smith's division, the
// algorithm of libgcc's __divdc3 for finite operands) so that the result does
// not depend on the host compiler's complex runtime.
void pmns_sq(bool normal, double U2[9])
{
    double t12, t13, t23, dcp;
    if (normal) {
        t12 = 33.44 * (M_PI / 180);
        t13 = 8.57 * (M_PI / 180);
        t23 = 49.0 * (M_PI / 180);
        dcp = 195.0 * (M_PI / 180);
    } else {
        t12 = 33.45 * (M_PI / 180);
        t13 = 8.61 * (M_PI / 180);
        t23 = 49.3 * (M_PI / 180);
        dcp = 286.0 * (M_PI / 180);
    }
    const double c12 = cos(t12), c13 = cos(t13), c23 = cos(t23);
    const double s12 = sin(t12), s13 = sin(t13), s23 = sin(t23);
    const nusi::cd del = nusi::C(cos(dcp), sin(dcp));
    nusi::cd U[3][3];
    U[0][0] = nusi::C(c12 * c13);
    U[0][1] = nusi::C(s12 * c13);
    U[0][2] = (s13 * 1.0) / del;
    U[1][0] = -s12 * c23 - (c12 * s23 * s13) * del;
    U[1][1] = c12 * c23 - (s12 * s23 * s13) * del;
    U[1][2] = nusi::C(s23 * c13);
    U[2][0] = s12 * s23 - (c12 * c23 * s13) * del;
    U[2][1] = -c12 * s23 - (s12 * c23 * s13) * del;
    U[2][2] = nusi::C(c23 * c13);
    for (int f = 0; f < 3; ++f)
        for (int k = 0; k < 3; ++k) U2[3 * f + k] = U[f][k].r * U[f][k].r + U[f][k].i * U[f][k].i;
}

// Lightest mass, aux.hpp:12-50.  The reference's quartic + constraint filter
// selects the unique root of the un-squared mass-sum equation, found here by
// bisection to full precision; at the minimal mass sum (root 0, where GSL
// returns rounding noise and m = 0 would make the tables NaN) the lightest
// mass is set to kMlFloor.
constexpr double kMlFloor = 1e-12;
double mass_sum(double m, double dmqSL, double dmqAT)
{
    if (dmqAT > 0) return m + sqrt(sq(m) + dmqSL) + sqrt(sq(m) + dmqAT);
    const double m2 = sqrt(sq(m) - dmqAT);
    return m + m2 + sqrt(sq(m2) - dmqSL);
}
bool lightest_mass(double mSum, double dmqSL, double dmqAT, double* mL)
{
    const double f0 = mass_sum(0.0, dmqSL, dmqAT) - mSum;
    double ml;
    if (f0 >= 0) {
        if (f0 > 64 * 2.220446049250313e-16 * mSum) return false;
        ml = kMlFloor;
    } else {
        double lo = 0.0, hi = mSum;
        for (int it = 0; it < 2000; ++it) {
            const double mid = 0.5 * (lo + hi);
            if (mid <= lo || mid >= hi) break;
            if (mass_sum(mid, dmqSL, dmqAT) - mSum > 0) hi = mid;
            else lo = mid;
        }
        ml = (fabs(mass_sum(hi, dmqSL, dmqAT) - mSum) < fabs(mass_sum(lo, dmqSL, dmqAT) - mSum)) ? hi : lo;
        if (ml <= 0) ml = kMlFloor;
    }
    const bool ok1 = (mSum - ml > 1.0e-7);
    const bool ok2 = (dmqAT > 0) ? (sq(mSum) - dmqAT - dmqSL - sq(ml) - 2 * ml * mSum > 1.0e-7)
                                 : (sq(mSum) + 2 * dmqAT + dmqSL - sq(ml) - 2 * ml * mSum > 1.0e-7);
    if (!(ok1 && ok2)) return false;
    *mL = ml;
    return true;
}

const double kGLw[3] = {5. / 9., 8. / 9., 5. / 9.};
const double kGLx[3] = {-0.7745966692414834, 0.0, 0.7745966692414834};

// flux_FS_E0, nuSIprop.hpp:666-692
double flux_fs_e0(double si, double zmax_eff)
{
    double res = 0;
    const double z_min = 0, z_max = zmax_eff;
    const int NI = 100;
    for (int f = 0; f < NI; f++) {
        const double a = z_min + f * (z_max - z_min) / NI;
        const double b = z_min + (f + 1.0) * (z_max - z_min) / NI;
        double zz[3];
        for (int q = 0; q < 3; ++q) zz[q] = (b - a) / 2. * kGLx[q] + (b + a) / 2.;
        res += (b - a) / 2. * (kGLw[0] * pow(1 + zz[0], -si) * sfr_h(zz[0]) / hubble_h(zz[0])
                               + kGLw[1] * pow(1 + zz[1], -si) * sfr_h(zz[1]) / hubble_h(zz[1])
                               + kGLw[2] * pow(1 + zz[2], -si) * sfr_h(zz[2]) / hubble_h(zz[2]));
    }
    return res;
}

// energy_FS / Lum_times_E, nuSIprop.hpp:694-744 (power law; stale norm_total)
double energy_fs(double si, double norm_total, double zmax_eff, double lEmin, double lEmax)
{
    const double E0 = 1e14;
    auto lte = [&](double z, double Em, double Ep) {
        if (fabs(si - 2) < 1e-5)
            return norm_total * sfr_h(z) * pow(E0 / (1 + z), si) * (log(Ep / Em) + (2 - si) / 2.0 * (sq(log(Ep)) - sq(log(Em))));
        return norm_total * sfr_h(z) * pow(E0 / (1 + z), si) * (pow(Ep, 2 - si) - pow(Em, 2 - si)) / (2 - si);
    };
    double res = 0;
    const double z_min = 0, z_max = zmax_eff, lo = pow(10, lEmin), hi = pow(10, lEmax);
    for (int f = 0; f < 100; f++) {
        const double a = z_min + f * (z_max - z_min) / 100;
        const double b = z_min + (f + 1.0) * (z_max - z_min) / 100;
        double zz[3];
        for (int q = 0; q < 3; ++q) zz[q] = (b - a) / 2. * kGLx[q] + (b + a) / 2.;
        res += (b - a) / 2. * (kGLw[0] * lte(zz[0], lo, hi) / hubble_h(zz[0]) + kGLw[1] * lte(zz[1], lo, hi) / hubble_h(zz[1])
                               + kGLw[2] * lte(zz[2], lo, hi) / hubble_h(zz[2]));
    }
    return res;
}

// ---------------------------------------------------------------------------
// phi-phi tables (interp.hpp:173-320, binary branch) -> device SplineDev
// ---------------------------------------------------------------------------
struct SplineStore {
    int device = 0;
    std::vector<void*> bufs;
    nusi::SplineSet set;
    nusi::SplineSet* d_set = nullptr;   // `set` in device memory: the kernels take it by pointer (a by-value
                                        // kernel argument whose address reaches a call is copied to scratch
                                        // by every work-item, 320 B each)
    ~SplineStore()
    {
        if (bufs.empty()) return;
        int prev = 0;
        hipGetDevice(&prev);
        hipSetDevice(device);
        for (void* b : bufs) hipFree(b);
        hipSetDevice(prev);
    }
};

// weights of interp.hpp:576-636 (the last node's weights are never read), node-major: the 16 weights
// of node j at w[16 j + 4 a + b]
void spline_weights(const std::vector<double>& x, std::vector<double>& w)
{
    const int n = (int)x.size();
    w.assign((size_t)16 * n, 0.0);
    auto W = [&](int a, int b, int j) -> double& { return w[(size_t)16 * j + 4 * a + b]; };
    for (int j = 0; j + 1 < n; ++j) {
        const double xm = (j > 0) ? x[j - 1] : 0.0, x0 = x[j], x1 = x[j + 1], x2 = (j + 2 < n) ? x[j + 2] : 0.0;
        if (j == 0) {
            W(0, 1, j) = (x0 - x1) / (x0 - x2);
            W(0, 2, j) = (-1 + (x1 - x0) / (x0 - x2));
            W(0, 3, j) = 1;
            W(1, 1, j) = (x1 - x0) / (x1 - x2);
            W(1, 2, j) = (x0 - x2) / (x1 - x2);
            W(2, 1, j) = sq(x1 - x0) / ((x2 - x1) * (x2 - x0));
            W(2, 2, j) = sq(x1 - x0) / ((x2 - x1) * (x0 - x2));
        } else if (j == n - 2) {
            W(0, 1, j) = sq(x1 - x0) / ((xm - x0) * (xm - x1));
            W(0, 2, j) = sq(x1 - x0) / ((x0 - xm) * (xm - x1));
            W(1, 1, j) = (x1 - x0) / (xm - x0);
            W(1, 2, j) = (2 * x0 - x1 - xm) / (xm - x0);
            W(1, 3, j) = 1;
            W(2, 1, j) = (x0 - x1) / (xm - x1);
            W(2, 2, j) = (xm - x0) / (xm - x1);
        } else {
            W(0, 0, j) = sq(x1 - x0) / ((x0 - xm) * (xm - x1));
            W(0, 1, j) = 2 * sq(x1 - x0) / ((xm - x0) * (xm - x1));
            W(0, 2, j) = sq(x1 - x0) / ((x0 - xm) * (xm - x1));
            W(1, 0, j) = (x0 - x1) * (1 / (xm - x0) + 1 / (x0 - x2));
            W(1, 1, j) = (x0 - x1) * (2 / (x0 - xm) + 1 / (x2 - x0));
            W(1, 2, j) = (2 * x0 - x1 - xm) / (xm - x0);
            W(1, 3, j) = 1;
            W(2, 0, j) = (x1 - x0) * (1 / (xm - x1) + 1 / (x1 - x2));
            W(2, 1, j) = (x1 - x0) * (2 / (x1 - xm) + 1 / (x2 - x1));
            W(2, 2, j) = (xm - x0) / (xm - x1);
            W(3, 0, j) = sq(x1 - x0) / ((-x1 + x2) * (-x0 + x2));
            W(3, 1, j) = sq(x1 - x0) / ((x1 - x2) * (-x0 + x2));
        }
    }
}

// file identity for the table-set cache of nusi_plan_load_phiphi: path, device and inode, size and the
// modification time to the nanosecond (a file rewritten in place gets a new mtime)
std::string file_stamp(const char* path)
{
    struct stat sb;
    if (stat(path, &sb) != 0) return std::string(path) + "|?";
    return std::string(path) + "|" + std::to_string((unsigned long long)sb.st_dev) + ":" +
           std::to_string((unsigned long long)sb.st_ino) + "|" + std::to_string((long long)sb.st_size) + "|" +
           std::to_string((long long)sb.st_mtim.tv_sec) + "." + std::to_string((long long)sb.st_mtim.tv_nsec);
}
// the cache: one entry per key; its mutex is held while that key loads (1.6 GB read + upload + windows), so
// loads of other keys (e.g. the same files on another device) run concurrently
struct SplineSlot {
    std::mutex mu;
    std::weak_ptr<SplineStore> set;
};
std::mutex g_spl_mu;   // guards the map only
std::map<std::string, std::shared_ptr<SplineSlot>> g_spl_cache;

int load_spline(const char* path, int ndim, const int* dims, SplineStore& st, nusi::SplineDev& out)
{
    FILE* fp = fopen(path, "rb");
    if (!fp)
        return fail(NUSI_ETABLE, std::string("Error at interp: the input file ") + path + " does not exist");
    std::vector<std::vector<double>> x(ndim);
    size_t nf = 1;
    for (int i = 0; i < ndim; ++i) {
        x[i].assign(dims[i], 0.0);
        nf *= (size_t)dims[i];
    }
    std::vector<float> f(nf);
    std::vector<float> chunk((size_t)(ndim + 1) * 65536);
    size_t r = 0;
    while (r < nf) {
        const size_t want = std::min<size_t>(65536, nf - r);
        if (fread(chunk.data(), sizeof(float) * (ndim + 1), want, fp) != want) {
            fclose(fp);
            return fail(NUSI_ETABLE, std::string("Error at interp: the input file ") + path + " is truncated");
        }
        for (size_t q = 0; q < want; ++q, ++r) {
            size_t rem = r;
            int idx[nusi::kSplMaxDim];
            for (int i = ndim - 1; i >= 0; --i) {
                idx[i] = (int)(rem % (size_t)dims[i]);
                rem /= (size_t)dims[i];
            }
            const float* rec = &chunk[q * (ndim + 1)];
            for (int i = 0; i < ndim; ++i) x[i][idx[i]] = (double)rec[i];
            f[r] = rec[ndim];
        }
    }
    fclose(fp);
    nusi::SplineDev sd;
    sd.ndim = ndim;
    sd.islog[0] = 1;  // both reference tables interpolate in log(x0) (nuSIprop.hpp:168-169)
    for (int i = 0; i < ndim; ++i) {
        sd.n[i] = dims[i];
        if (sd.islog[i])
            for (double& v : x[i]) v = log(v);
        std::vector<double> w;
        spline_weights(x[i], w);
        double *dx = nullptr, *dw = nullptr;
        HIPCHECK(hipMalloc(&dx, sizeof(double) * x[i].size()));
        st.bufs.push_back(dx);
        HIPCHECK(hipMalloc(&dw, sizeof(double) * w.size()));
        st.bufs.push_back(dw);
        HIPCHECK(hipMemcpy(dx, x[i].data(), sizeof(double) * x[i].size(), hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(dw, w.data(), sizeof(double) * w.size(), hipMemcpyHostToDevice));
        sd.x[i] = dx;
        sd.w[i] = dw;
        // guide table of the node search (nusi_spline.hpp): gd[u] = the last node <= the lower end of
        // bucket u, 4 (n-1) buckets over [x[0], x[n-1]]
        const std::vector<double>& xi = x[i];
        const int n = dims[i], G = 4 * (n - 1);
        const double h = (xi[n - 1] - xi[0]) / G;
        if (n >= 2 && h > 0 && std::is_sorted(xi.begin(), xi.end())) {
            std::vector<int> gd(G);
            for (int u = 0; u < G; ++u) {
                const double lo = xi[0] + u * h;
                const int k = (int)(std::upper_bound(xi.begin(), xi.end(), lo) - xi.begin()) - 1;
                gd[u] = std::max(0, std::min(n - 2, k));
            }
            int* dg = nullptr;
            HIPCHECK(hipMalloc(&dg, sizeof(int) * G));
            st.bufs.push_back(dg);
            HIPCHECK(hipMemcpy(dg, gd.data(), sizeof(int) * G, hipMemcpyHostToDevice));
            sd.gd[i] = dg;
            sd.ng[i] = G;
            sd.ginv[i] = 1.0 / h;
        }
    }
    float* df = nullptr;
    HIPCHECK(hipMalloc(&df, sizeof(float) * nf));
    st.bufs.push_back(df);
    HIPCHECK(hipMemcpy(df, f.data(), sizeof(float) * nf, hipMemcpyHostToDevice));
    sd.f = df;
    if (ndim == 3) {
        float* dw = nullptr;   // 16 x the table: the 4 x 4 windows of nusi_spline.hpp
        HIPCHECK(hipMalloc(&dw, sizeof(float) * 16 * nf));
        st.bufs.push_back(dw);
        HIPCHECK(nusi::spline_windows_build(df, dims[0], dims[1], dims[2], dw));
        sd.fw = dw;
    }
    out = sd;
    return NUSI_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// plan
// ---------------------------------------------------------------------------
// the alpha-table batches of one call (nusi::launch_alpha): count, how many lack the phi-phi channel, the cap
struct AlphaBatches {
    int nbatch = 0, nb_plain = 0, cap = 1;
};

struct nusi_plan {
    int device = 0;
    hipStream_t stream = nullptr;
    HostGrid grid;
    int max_points = 0;
    nusi::GridDev gd{};
    double* d_grid = nullptr;
    nusi::Point* d_pts = nullptr;
    nusi::Point* h_pts = nullptr;  // pinned
    nusi::Point* d_tpts = nullptr;  // one representative per distinct table (table kernels)
    nusi::Point* h_tpts = nullptr;  // pinned
    int* d_batches = nullptr;       // alpha-table batches (nusi::launch_alpha): first table | count << 24
    int* h_batches = nullptr;       // pinned
    int alpha_batch = 0;            // NUSI_OPT_ALPHA_BATCH: max tables per batch; 0 = auto
    int alpha_kind = 0;             // NUSI_OPT_ALPHA_KERNEL: 0 k_alpha_batch, 1 k_alpha_tile<G> (<= 4), 2 per entry
    int cascade_rhs = 0;            // NUSI_OPT_CASCADE_RHS: 0 = auto, 1 = one point per MFMA-cascade workgroup,
                                    // 2 = pairs, 3..16 = gamma batches of up to that many (k_cascade_bs_gamma)
    int* d_gidx = nullptr;          // gamma batches: the points of each batch, batch after batch
    int* h_gidx = nullptr;          // pinned
    int2* d_gbgrp = nullptr;        // ... per batch: first index into gidx, count
    int2* h_gbgrp = nullptr;        // pinned
    double* d_fh = nullptr;         // k_cascade_bs's F FIFO between step passes, cascade_bs_scratch_doubles per workgroup
    int step_passes = 0;            // NUSI_OPT_STEP_PASSES: 1 = the step-pass instance of k_cascade_bs also where one pass fits
    int shift_max = 0;              // NUSI_OPT_SHIFT_REUSE: K, the largest bin offset served by a base table set
    int ref_order = 1;              // NUSI_OPT_REFERENCE_ORDER: 1 (default) = the tables in the reference's own arithmetic,
                                    // 0 = the shared-algorithm order (opt-in fast mode)
    int cascade_sync = 0;           // NUSI_OPT_CASCADE_SYNC: 0 = auto, 2 = block-synchronous (the same kernel; 1 is refused)
    int corner_mb = 0;              // NUSI_OPT_REFO_CORNER_MB: the member-corner block's budget (0 = automatic)
    size_t fh_doubles = 0;          // capacity of d_fh in doubles (the block-synchronous kernels' FIFOs)
    nusi_plan* shift = nullptr;     // ... its plan: the same grid with K more redshift steps (axis T + K)
    int2* d_smap = nullptr;         // per shifted table: base index in `shift`, bin offset
    int2* h_smap = nullptr;         // pinned
    AlphaBatches shift_batches;     // the base plan's alpha batches of the last call
    double* d_src = nullptr;        // DSNB source terms of the MFMA cascade [src_cap][cascade_src_doubles]
    int src_cap = 0;
    std::vector<int> slot_of;       // table slot of each point of the last call
    int last_ntab = 0;
    int* d_warn = nullptr;
    // The per-call inputs in ONE device block and its pinned mirror, uploaded by ONE copy per call (a single
    // propagation paid a DMA blit of ~4 us per array, five of them, plus a fill for the warnings): sections
    // [warn | batches | gbgrp | gidx | pts | tpts], each sized for max_points (in_sections); the warnings are zeroed
    // on the host side of the copy
    char* d_in = nullptr;
    char* h_in = nullptr;      // pinned
    int* h_warn0 = nullptr;    // pinned: the warn section of h_in (zeros)
    size_t in_tpts = 0;        // byte offset of the tpts section (the copy runs up to its ntab-th Point)
    // evolve_host's output staging (pinned; the warnings, then flux / flux_fla; only for calls of at most
    // kStageBytes) and the warnings it fetched, for nusi_plan_warnings without a second round trip
    char* h_out = nullptr;
    size_t h_out_bytes = 0;
    std::vector<int> warn_host;
    bool warn_host_valid = false;
    nusi::TablesDev tabs{};
    nusi::AlphaTilesDev atiles{};
    nusi::MCornerDev mc{};         // NUSI_OPT_REFERENCE_ORDER: member corners of the big-batch kernel (mcorner_ensure)
    double* d_scratch = nullptr;   // flux outputs when the caller passes NULL
    double* d_kt = nullptr;        // the k-split alpha path's term buffer (TablesDev::Kt), kt_doubles doubles
    size_t kt_doubles = 0;
    double* d_gpre = nullptr;      // the reference order's Gamma / alphaTilde dilogarithms (TablesDev::Gpre)
    size_t gpre_doubles = 0;
    std::shared_ptr<SplineStore> spl;
    nusi::SplineSet* d_nospl = nullptr;   // an empty spline set in device memory (no phi-phi tables loaded)
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t ev_copy = nullptr;
    hipEvent_t ev_done = nullptr;      // end of the latest call's kernels (the next call waits for it)
    hipStream_t side = nullptr;        // Gamma / alphaTilde beside alpha in calls of few tables (kOverlapTables)
    hipEvent_t ev_fork = nullptr;
    bool ran = false;
    int last_n = 0;
    std::vector<hipEvent_t> prof_ev;   // 4 per recorded call
    hipEvent_t last_ev[4] = {nullptr, nullptr, nullptr, nullptr};   // the latest call's stage events (handles)
    const char* alpha_kernel = "";     // main kernels of the latest call (nusi_plan_kernels)
    std::string alpha_label;           // ... storage of a composed alpha label (shift reuse)
    const char* cascade_kernel = "";
    int prof_max = 0, prof_n = 0;
    int cascade_kind = NUSI_CASCADE_AUTO;
    double U2[2][9];
    std::map<double, double> fs_cache;                      // si -> flux_FS_E0
    std::map<std::pair<double, int>, std::vector<double>> mass_cache;
};

namespace {

// the Point fields the Stage-A kernels read (nusi_physics.hpp gamma/alphat/alpha_entry)
using TableKey = std::array<double, 12>;
TableKey table_key(const nusi::Point& P)
{
    return TableKey{P.mphi, P.g, P.Ga, P.mn[0], P.mn[1], P.mn[2], P.u[0], P.u[1], P.u[2],
                    (double)P.majorana, (double)P.non_resonant, (double)P.phiphi};
}

int build_point(nusi_plan* pl, const nusi_params& p, nusi::Point& P)
{
    const HostGrid& G = pl->grid;
    if (p.N_bins_E != G.N || p.lEmin != G.lEmin || p.lEmax != G.lEmax || p.zmax != G.zmax_in)
        return fail(NUSI_EPARAM, "point grid (N_bins_E, lEmin, lEmax, zmax) differs from the plan's");
    if (p.flav < 0 || p.flav > 2) return fail(NUSI_EPARAM, "flav must be 0, 1 or 2");
    if (p.source_model != NUSI_SOURCE_DSNB && p.source_model != NUSI_SOURCE_POWER_LAW)
        return fail(NUSI_EPARAM, "unknown source_model");
    const int no = p.normal_ordering ? 1 : 0;
    // masses, nuSIprop.hpp:184-203
    const double dmq21 = 7.42e-5;
    const double dmqAT = no ? 2.514e-3 : -2.497e-3;
    auto key = std::make_pair(p.mntot, no);
    auto it = pl->mass_cache.find(key);
    if (it == pl->mass_cache.end()) {
        double mL;
        if (!lightest_mass(p.mntot, dmq21, dmqAT, &mL)) {
            char buf[256];
            snprintf(buf, sizeof buf,
                     "No neutrino mass spectrum was found corresponding to \\sum m = %g, dmqAT = %g, dmqSL = %g. Exiting...",
                     p.mntot, dmqAT, dmq21);
            return fail(NUSI_ENOSPECTRUM, buf);
        }
        std::vector<double> mn(3);
        if (no) {
            mn[0] = mL;
            mn[1] = sqrt(dmq21 + sq(mL));
            mn[2] = sqrt(dmqAT + sq(mL));
        } else {
            mn[2] = mL;
            mn[1] = sqrt(sq(mL) - dmqAT);
            mn[0] = sqrt(sq(mn[1]) - dmq21);
        }
        it = pl->mass_cache.emplace(key, mn).first;
    }
    auto fit = pl->fs_cache.find(p.si);
    if (fit == pl->fs_cache.end()) fit = pl->fs_cache.emplace(p.si, flux_fs_e0(p.si, G.zmax_eff)).first;
    memset(&P, 0, sizeof(P));
    P.mphi = p.mphi;
    P.g = p.g;
    P.mntot = p.mntot;
    P.si = p.si;
    P.norm = p.norm;
    P.norm_total = p.norm / fit->second;
    P.Ga = p.majorana ? sq(p.g) * p.mphi / (16.0 * M_PI) : sq(p.g) * p.mphi / (8.0 * M_PI);
    for (int k = 0; k < 3; ++k) P.mn[k] = it->second[k];
    for (int k = 0; k < 9; ++k) P.U2[k] = pl->U2[no][k];
    for (int k = 0; k < 3; ++k) P.u[k] = pl->U2[no][3 * p.flav + k];
    P.majorana = p.majorana ? 1 : 0;
    P.non_resonant = p.non_resonant ? 1 : 0;
    P.phiphi = p.phiphi ? 1 : 0;
    P.source = p.source_model;
    nusi::point_derive(P);
    if (P.non_resonant && P.phiphi && !pl->spl)
        return fail(NUSI_ETABLE, "phiphi requested but the phi-phi tables are not loaded (nusi_plan_load_phiphi)");
    return NUSI_OK;
}


// Order the tables h_tpts[0, ntab) so that those sharing m_phi, the masses and the flags -- whose alpha tables
// share every leaf of (S', t) alone -- are neighbours (slots renumbered; perm[old] = new), and cut them into the
// batches h_batches.
AlphaBatches alpha_batches(nusi_plan* pl, int ntab, std::vector<int>& perm)
{
    AlphaBatches ab;
    std::vector<int> order(ntab);
    perm.assign(ntab, 0);
    for (int j = 0; j < ntab; ++j) order[j] = j;
    auto bkey = [&](int j) {
        const nusi::Point& P = pl->h_tpts[j];
        // phi-phi first: the tables with the channel come last (their batches run on their own launch)
        return std::make_tuple(P.phiphi && P.non_resonant, P.mphi, P.mn[0], P.mn[1], P.mn[2], P.majorana, P.non_resonant,
                               P.phiphi);
    };
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return bkey(a) < bkey(b); });
    {
        std::vector<nusi::Point> tmp(pl->h_tpts, pl->h_tpts + ntab);
        for (int j = 0; j < ntab; ++j) {
            pl->h_tpts[j] = tmp[order[j]];
            perm[order[j]] = j;
        }
    }
    for (int j = 0; j < ntab; ++j) pl->h_tpts[j].tslot = j;
    // batch cap: the tile kernel's LDS holds <= 4 (3 measured best); the big-batch kernel shares the leaves of
    // any number, but one workgroup runs a batch's points one after the other, so the cap keeps ~2 rounds of
    // workgroups per CU slot (256 CUs x 3) in the grid: ntab x class-0 tiles / cap >= 1536
    int cap = pl->alpha_kind == 1 ? std::min(pl->alpha_batch, 4) : pl->alpha_batch;
    if (cap <= 0) {
        if (pl->alpha_kind == 1) cap = 3;
        else {
            const long long work = (long long)ntab * std::max(1, pl->atiles.ncls[0]);
            cap = (int)std::max(1LL, std::min(64LL, (work + 1535) / 1536));
        }
    }
    ab.cap = cap;
    for (int j = 0; j < ntab;) {
        int run = 1;   // the group of tables sharing bkey, split into near-equal batches of <= cap
        while (j + run < ntab && bkey(j + run) == bkey(j)) ++run;
        const int nb = (run + cap - 1) / cap;
        for (int b = 0; b < nb; ++b) {
            const int lo = j + (int)((long long)run * b / nb), hi = j + (int)((long long)run * (b + 1) / nb);
            pl->h_batches[ab.nbatch++] = lo | ((hi - lo) << 24);
        }
        j += run;
    }
    while (ab.nb_plain < ab.nbatch) {   // batches without the phi-phi channel (sorted first by bkey)
        const nusi::Point& F = pl->h_tpts[pl->h_batches[ab.nb_plain] & 0xffffff];
        if (F.phiphi && F.non_resonant) break;
        ++ab.nb_plain;
    }
    return ab;
}

// NUSI_OPT_REFERENCE_ORDER on the big-batch kernel: the member-corner block of plan p (MCornerDev) for the batches of
// this call -- 6 NC doubles per table (C4's N_E = 300 axis: NC = 77 421, 3.7 MB), allocated for at most
// NUSI_OPT_REFO_CORNER_MB (automatic: kMCornerBudget bytes and half the free memory) of tables, at least the largest
// batch; launch_alpha runs the batches in chunks that fit
constexpr size_t kMCornerBudget = size_t(8) << 30;
#ifndef NUSI_GA_PRE   // A/B: 0 = the reference order's Gamma / alphaTilde of few tables without k_ga_dilogs
#define NUSI_GA_PRE 1
#endif
constexpr bool kGaPre = NUSI_GA_PRE != 0;
constexpr int kOverlapTables = 16;   // calls of at most this many tables overlap Gamma / alphaTilde with alpha
constexpr size_t kStageBytes = size_t(4) << 20;   // nusi_plan_evolve_host's pinned output staging, at most
constexpr int kSplitTables = 2;   // calls of at most this many tables (no phi-phi) run the k-split alpha path
int mcorner_ensure(nusi_plan* p, int ntab, const AlphaBatches& ab, int budget_mb)
{
    nusi::MCornerDev& mc = p->mc;
    if (!mc.eu) {
        std::vector<int> eu;
        std::vector<double> ue;
        nusi::mcorner_edges(p->grid.T, p->grid.lo.data(), p->grid.hi.data(), eu, ue);
        HIPCHECK(hipMalloc(&mc.eu, sizeof(int) * eu.size()));
        HIPCHECK(hipMemcpy(mc.eu, eu.data(), sizeof(int) * eu.size(), hipMemcpyHostToDevice));
        HIPCHECK(hipMalloc(&mc.ue, sizeof(double) * ue.size()));
        HIPCHECK(hipMemcpy(mc.ue, ue.data(), sizeof(double) * ue.size(), hipMemcpyHostToDevice));
        mc.U = (int)ue.size();
        mc.NC = (long long)mc.U * (mc.U + 1) / 2;
    }
    const size_t per = sizeof(double) * 6 * (size_t)mc.NC;
    if (mc.buf && budget_mb == 0 && mc.cap_tables >= ntab && per * mc.cap_tables <= kMCornerBudget)
        return NUSI_OK;   // every table of the call fits the block already (no hipMemGetInfo per call)
    int nbmax = 1;
    for (int b = 0; b < ab.nbatch; ++b) nbmax = std::max(nbmax, (int)((unsigned)p->h_batches[b] >> 24));
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = kMCornerBudget;
    const size_t budget = budget_mb > 0 ? ((size_t)budget_mb << 20)
                                        : std::min(kMCornerBudget, (fr + (mc.buf ? per * mc.cap_tables : 0)) / 2);
    const int want = std::max(nbmax, (int)std::min<size_t>((size_t)ntab, budget / per));
    if (mc.buf && mc.cap_tables >= want && (budget_mb == 0 || mc.cap_tables == want)) return NUSI_OK;
    hipFree(mc.buf);
    mc.buf = nullptr;
    mc.cap_tables = 0;
    HIPCHECK(hipMalloc(&mc.buf, per * want));
    mc.cap_tables = want;
    return NUSI_OK;
}

// NUSI_OPT_SHIFT_REUSE.  alpha / Gamma / alphaTilde see the energies only through
// 2 m_k E / m_phi^2 (nuSIprop.hpp:1253-1256) and g through g^4 and Gamma_phi / m_phi = g^2 / 16 pi, so the tables of
// m_phi' = m_phi r^(-o/2) (r = Emax[0] / Emin[0] = the table axis' bin ratio) are those of m_phi read o bins higher.
// Only tables with g <= kShiftReuseGMax = 0.05 take part (the optical depth amplifies the shifted tables' rounding
// with g); the others are built directly.  Tables of one (g, masses, |U|^2, flags) are taken in
// decreasing m_phi: each group starts at its largest m_phi (the base) and takes the following ones whose offset
// o = 2 ln(m_base / m_phi) / ln r is within |o - round(o)| ln(r) / 2 < 1e-13 of an integer (m_phi reproduced to
// ~1e-13 relative) in [1, K].  Groups of two or more go to slots [nd, ntab) in group order (remap[old slot] = new slot; smap[slot - nd]
// = (base index, o); bases[] = the base Points); the rest stay in [0, nd).  Returns nd.
int shift_groups(nusi_plan* pl, int ntab, std::vector<int>& remap, std::vector<int2>& smap, std::vector<nusi::Point>& bases)
{
    const double lr = log(pl->grid.Emax[0] / pl->grid.Emin[0]);
    const int K = pl->shift_max;
    const nusi::Point* tp = pl->h_tpts;
    auto gkey = [&](int j) {
        const nusi::Point& P = tp[j];
        return std::make_tuple(P.g, P.mn[0], P.mn[1], P.mn[2], P.u[0], P.u[1], P.u[2], P.majorana, P.non_resonant,
                               P.phiphi);
    };
    // only couplings up to kShiftReuseGMax share: the shifted tables differ from a point's own by rounding, and the
    // flux's optical depth amplifies that with the coupling (scripts/dev_shift_reuse_errors.py on the GPU, vs each
    // point's own evolution: c4s lattice <= 1.7e-11 for g <= 0.044, 6.4e-10 at 0.135, 3e-8 at g = 1; N_E = 850,
    // m_phi = 3e7: 8.8e-10 at g = 0.05, 1.4e-8 at 0.1; the north star bounds fluxes at 1e-9)
    constexpr double kShiftReuseGMax = 0.05;
    std::vector<int> idx;
    for (int j = 0; j < ntab; ++j)
        if (tp[j].g <= kShiftReuseGMax) idx.push_back(j);
    const int nsh = (int)idx.size();
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) {
        const auto ka = gkey(a), kb = gkey(b);
        return ka != kb ? ka < kb : tp[a].mphi > tp[b].mphi;
    });
    std::vector<int> grp(ntab, -1), off(ntab, 0);
    std::vector<std::vector<int>> members;
    for (int a = 0; a < nsh;) {
        int b = a + 1;
        while (b < nsh && gkey(idx[b]) == gkey(idx[a])) ++b;
        std::vector<int> cur{idx[a]};
        int last = 0;
        for (int c = a + 1; c <= b; ++c) {
            bool join = false;
            int o = 0;
            if (c < b) {
                const double kf = 2.0 * log(tp[cur[0]].mphi / tp[idx[c]].mphi) / lr;
                o = (int)lround(kf);
                // the lattice m_phi must reproduce the point's own to a few ulp: m_base r^(-o/2) differs from it by
                // |kf - o| ln(r) / 2 relative, and the cascade sees only the tables (1e-6 in o let a
                // point 2e-8 off the lattice take the tables of a slightly different m_phi)
                join = o > last && o <= K && fabs(kf - o) * lr * 0.5 < 1e-13;
            }
            if (join) {
                cur.push_back(idx[c]);
                off[idx[c]] = last = o;
                continue;
            }
            if (cur.size() >= 2) {
                for (int m : cur) grp[m] = (int)members.size();
                members.push_back(cur);
            }
            if (c < b) {
                cur.assign(1, idx[c]);
                off[idx[c]] = last = 0;
            }
        }
        a = b;
    }
    remap.assign(ntab, 0);
    int nd = 0;
    for (int j = 0; j < ntab; ++j)
        if (grp[j] < 0) remap[j] = nd++;
    int s = nd;
    smap.clear();
    bases.clear();
    for (size_t g = 0; g < members.size(); ++g) {
        bases.push_back(tp[members[g][0]]);
        for (int m : members[g]) {
            remap[m] = s++;
            smap.push_back(make_int2((int)g, off[m]));
        }
    }
    return nd;
}

// the base plan of NUSI_OPT_SHIFT_REUSE: the plan's grid with K more redshift steps, so that its table axis is
// the plan's, bit for bit, extended by K bins on top (nuSIprop.hpp:224-233: bins >= N are Emin/Emax[N-1] (1 + z));
// sized for the call's nbase base tables (grown on demand, at most max_points / 2: a base serves >= 2 tables), with
// the per-row warning records (TablesDev::Wmin) that k_table_shift reads
int ensure_shift_plan(nusi_plan* pl, int nbase)
{
    const int K = pl->shift_max;
    if (pl->shift && pl->shift->grid.T == pl->grid.T + K && pl->shift->max_points >= nbase) return NUSI_OK;
    int cap = nbase;
    if (pl->shift) {
        cap = std::max(nbase, std::min(2 * pl->shift->max_points, std::max(1, pl->max_points / 2)));
        if (pl->ran) {   // the previous call's kernels read the old base tables
            HIPCHECK(hipSetDevice(pl->device));
            HIPCHECK(hipEventSynchronize(pl->ev_done));
        }
        nusi_plan_destroy(pl->shift);
        pl->shift = nullptr;
    }
    const HostGrid& G = pl->grid;
    const double r = G.Emax[0] / G.Emin[0];
    const double zb = pow(r, G.Nz + K - 1.5) - 1;   // N_steps_z = (int)(ln(1 + zb) / ln r + 2) = Nz + K
    nusi_plan* sp = nullptr;
    int rc = nusi_plan_create(pl->device, G.N, G.lEmin, G.lEmax, zb, std::max(1, cap), &sp);
    if (rc) return rc;
    const HostGrid& B = sp->grid;
    bool same = B.T == G.T + K;
    for (int n = 0; same && n < G.T; ++n) same = B.lo[n] == G.lo[n] && B.hi[n] == G.hi[n];
    if (!same) {
        nusi_plan_destroy(sp);
        return fail(NUSI_EPARAM, "shift reuse: the extended axis does not match the plan's below T");
    }
    sp->alpha_batch = pl->alpha_batch;
    sp->alpha_kind = pl->alpha_kind;
    sp->spl = pl->spl;
    HIPCHECK(hipSetDevice(pl->device));
    if (hipMalloc(&sp->tabs.Wmin, sizeof(int) * 4 * (size_t)B.T * sp->max_points) != hipSuccess) {
        nusi_plan_destroy(sp);
        return fail(NUSI_EHIP, "shift reuse: no device memory for the base plan's warning records");
    }
    if (!pl->d_smap) {
        HIPCHECK(hipMalloc(&pl->d_smap, sizeof(int2) * pl->max_points));
        HIPCHECK(hipHostMalloc((void**)&pl->h_smap, sizeof(int2) * pl->max_points, hipHostMallocDefault));
    }
    pl->shift = sp;
    return NUSI_OK;
}
}  // namespace

extern "C" {

const char* nusi_last_error(void) { return g_err.c_str(); }

int nusi_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void nusi_params_default(nusi_params* p, double mphi, double g, double mntot, double si)
{
    p->mphi = mphi;
    p->g = g;
    p->mntot = mntot;
    p->si = si;
    p->norm = 1;
    p->majorana = 1;
    p->non_resonant = 1;
    p->normal_ordering = 1;
    p->N_bins_E = 300;
    p->lEmin = 12.0;
    p->lEmax = 17.0;
    p->zmax = 5.0;
    p->flav = 2;
    p->phiphi = 0;
    p->source_model = NUSI_SOURCE_DSNB;
}

void nusi_plan_destroy(nusi_plan* pl)
{
    if (!pl) return;
    int prev = 0;
    hipGetDevice(&prev);
    hipSetDevice(pl->device);
    if (pl->stream) hipStreamSynchronize(pl->stream);
    for (auto& e : pl->ev)
        if (e) hipEventDestroy(e);
    if (pl->ev_copy) hipEventDestroy(pl->ev_copy);
    if (pl->ev_done) hipEventDestroy(pl->ev_done);
    if (pl->ev_fork) hipEventDestroy(pl->ev_fork);
    if (pl->side) hipStreamDestroy(pl->side);
    for (auto& e : pl->prof_ev) hipEventDestroy(e);
    hipFree(pl->d_grid);
    hipFree(pl->d_in);   // (d_pts, d_tpts, d_batches, d_warn, d_gidx, d_gbgrp and their pinned mirrors live in it)
    if (pl->h_in) hipHostFree(pl->h_in);
    if (pl->h_out) hipHostFree(pl->h_out);
    hipFree(pl->tabs.G);
    hipFree(pl->tabs.At);
    hipFree(pl->tabs.A);
    hipFree(pl->tabs.Med);
    hipFree(pl->tabs.Wmin);
    hipFree(pl->d_nospl);
    hipFree(pl->d_src);
    hipFree(pl->d_smap);
    if (pl->h_smap) hipHostFree(pl->h_smap);
    hipFree(pl->d_fh);
    nusi::alpha_tiles_destroy(&pl->atiles);
    hipFree(pl->mc.buf);
    hipFree(pl->mc.eu);
    hipFree(pl->mc.ue);
    hipFree(pl->d_scratch);
    hipFree(pl->d_kt);
    hipFree(pl->d_gpre);
    if (pl->stream) hipStreamDestroy(pl->stream);
    pl->spl.reset();
    nusi_plan* sh = pl->shift;
    hipSetDevice(prev);
    delete pl;
    nusi_plan_destroy(sh);
}

int nusi_plan_create(int device, int N_bins_E, double lEmin, double lEmax, double zmax, int max_points, nusi_plan** out)
{
    *out = nullptr;
    if (N_bins_E < 2 || !(lEmax > lEmin) || !(zmax > 0) || max_points < 1)
        return fail(NUSI_EPARAM, "bad grid: need N_bins_E >= 2, lEmax > lEmin, zmax > 0, max_points >= 1");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(NUSI_EHIP, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(NUSI_EPARAM, "device index out of range");
    HIPCHECK(hipSetDevice(device));
    std::unique_ptr<nusi_plan, void (*)(nusi_plan*)> pl(new nusi_plan, nusi_plan_destroy);
    pl->device = device;
    pl->grid = make_grid(N_bins_E, lEmin, lEmax, zmax);
    pl->max_points = max_points;
    pmns_sq(true, pl->U2[1]);
    pmns_sq(false, pl->U2[0]);
    const HostGrid& G = pl->grid;
    if (G.Nz < 2) return fail(NUSI_EPARAM, "redshift grid has fewer than two steps");
    HIPCHECK(hipStreamCreateWithFlags(&pl->stream, hipStreamNonBlocking));
    for (auto& e : pl->ev) HIPCHECK(hipEventCreate(&e));
    HIPCHECK(hipEventCreateWithFlags(&pl->ev_copy, hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&pl->ev_done, hipEventDisableTiming));
    HIPCHECK(hipStreamCreateWithFlags(&pl->side, hipStreamNonBlocking));
    HIPCHECK(hipEventCreateWithFlags(&pl->ev_fork, hipEventDisableTiming));
    // grid arrays in one allocation
    const size_t ng = 2 * (size_t)G.N + 2 * (size_t)G.T + 4 * (size_t)G.Nz;
    HIPCHECK(hipMalloc(&pl->d_grid, sizeof(double) * ng));
    std::vector<double> hg;
    hg.reserve(ng);
    hg.insert(hg.end(), G.Emin.begin(), G.Emin.end());
    hg.insert(hg.end(), G.Emax.begin(), G.Emax.end());
    hg.insert(hg.end(), G.lo.begin(), G.lo.end());
    hg.insert(hg.end(), G.hi.begin(), G.hi.end());
    hg.insert(hg.end(), G.z.begin(), G.z.end());
    hg.insert(hg.end(), G.step_c.begin(), G.step_c.end());
    hg.insert(hg.end(), G.step_s.begin(), G.step_s.end());
    hg.insert(hg.end(), G.sfr.begin(), G.sfr.end());
    HIPCHECK(hipMemcpy(pl->d_grid, hg.data(), sizeof(double) * ng, hipMemcpyHostToDevice));
    nusi::GridDev& gd = pl->gd;
    gd.N = G.N;
    gd.Nz = G.Nz;
    gd.T = G.T;
    gd.PT = (long long)G.T * (G.T - 1) / 2;
    double* q = pl->d_grid;
    gd.Emin = q;
    q += G.N;
    gd.Emax = q;
    q += G.N;
    gd.lo = q;
    q += G.T;
    gd.hi = q;
    q += G.T;
    gd.z = q;
    q += G.Nz;
    gd.step_c = q;
    q += G.Nz;
    gd.step_s = q;
    q += G.Nz;
    gd.sfr = q;
    {   // the per-call input block (nusi_plan::d_in)
        const size_t mp = (size_t)max_points;
        auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
        const size_t o_warn = 0, o_bat = al(o_warn + sizeof(int) * mp), o_grp = al(o_bat + sizeof(int) * mp);
        const size_t o_gidx = al(o_grp + sizeof(int2) * mp), o_pts = al(o_gidx + sizeof(int) * mp);
        const size_t o_tpts = al(o_pts + sizeof(nusi::Point) * mp), tot = o_tpts + sizeof(nusi::Point) * mp;
        HIPCHECK(hipMalloc(&pl->d_in, tot));
        HIPCHECK(hipHostMalloc((void**)&pl->h_in, tot, hipHostMallocDefault));
        memset(pl->h_in, 0, tot);
        pl->d_warn = (int*)(pl->d_in + o_warn);
        pl->h_warn0 = (int*)(pl->h_in + o_warn);
        pl->d_batches = (int*)(pl->d_in + o_bat);
        pl->h_batches = (int*)(pl->h_in + o_bat);
        pl->d_gbgrp = (int2*)(pl->d_in + o_grp);
        pl->h_gbgrp = (int2*)(pl->h_in + o_grp);
        pl->d_gidx = (int*)(pl->d_in + o_gidx);
        pl->h_gidx = (int*)(pl->h_in + o_gidx);
        pl->d_pts = (nusi::Point*)(pl->d_in + o_pts);
        pl->h_pts = (nusi::Point*)(pl->h_in + o_pts);
        pl->d_tpts = (nusi::Point*)(pl->d_in + o_tpts);
        pl->h_tpts = (nusi::Point*)(pl->h_in + o_tpts);
        pl->in_tpts = o_tpts;
    }
    HIPCHECK(hipMalloc(&pl->tabs.G, sizeof(double) * (size_t)G.T * max_points));
    HIPCHECK(hipMalloc(&pl->tabs.At, sizeof(double) * (size_t)G.T * max_points));
    HIPCHECK(hipMalloc(&pl->tabs.A, sizeof(double) * (size_t)gd.PT * max_points));
    HIPCHECK(hipMalloc(&pl->tabs.Med, sizeof(double) * 3 * nusi::kMedFields * (size_t)G.T * max_points));
    {   // the empty spline set of plans without phi-phi tables (device memory, like SplineStore::d_set)
        const nusi::SplineSet none{};
        HIPCHECK(hipMalloc(&pl->d_nospl, sizeof(nusi::SplineSet)));
        HIPCHECK(hipMemcpy(pl->d_nospl, &none, sizeof(nusi::SplineSet), hipMemcpyHostToDevice));
    }
    std::vector<unsigned char> shared(G.T, 0);   // bin edges shared bitwise with the next bin
    for (int n = 0; n + 1 < G.T; ++n) shared[n] = (G.hi[n] == G.lo[n + 1]);
    HIPCHECK(nusi::alpha_tiles_create(G.T, shared.data(), &pl->atiles));
    *out = pl.release();
    return NUSI_OK;
}

// Loaded table sets are shared by every plan / object on the same device that loads the same files
// (path, dims, size and mtime): the reference reads the tables in every constructor
// (nuSIprop.hpp:166-170); here a set costs 400 MB + its 6.4 GB of windows in HBM, so a second
// calculate_flux object reuses the first one's while it is alive.
int nusi_plan_load_phiphi(nusi_plan* pl, const char* at_path, const int* at_dims, const char* a_path, const int* a_dims)
{
    static const int def2[2] = {5000, 100}, def3[3] = {1000, 1000, 100};
    if (!pl) return fail(NUSI_EPARAM, "plan is NULL");
    if (!at_path || !a_path) return fail(NUSI_EPARAM, "phi-phi table path is NULL");
    HIPCHECK(hipSetDevice(pl->device));
    const int* d2 = at_dims ? at_dims : def2;
    const int* d3 = a_dims ? a_dims : def3;
    const std::string key = std::to_string(pl->device) + "|" + file_stamp(at_path) + "|" + std::to_string(d2[0]) + "x" +
                            std::to_string(d2[1]) + "|" + file_stamp(a_path) + "|" + std::to_string(d3[0]) + "x" +
                            std::to_string(d3[1]) + "x" + std::to_string(d3[2]);
    std::shared_ptr<SplineSlot> slot;
    {
        std::lock_guard<std::mutex> lock(g_spl_mu);
        auto& e = g_spl_cache[key];
        if (!e) e = std::make_shared<SplineSlot>();
        slot = e;
    }
    std::lock_guard<std::mutex> lock(slot->mu);
    if (auto hit = slot->set.lock()) {
        pl->spl = hit;
        return NUSI_OK;
    }
    auto st = std::make_shared<SplineStore>();
    st->device = pl->device;
    int r = load_spline(at_path, 2, d2, *st, st->set.at);
    if (r) return r;
    r = load_spline(a_path, 3, d3, *st, st->set.a);
    if (r) return r;
    HIPCHECK(hipMalloc(&st->d_set, sizeof(nusi::SplineSet)));
    st->bufs.push_back(st->d_set);
    HIPCHECK(hipMemcpy(st->d_set, &st->set, sizeof(nusi::SplineSet), hipMemcpyHostToDevice));
    slot->set = st;
    pl->spl = st;
    return NUSI_OK;
}

int nusi_plan_grid(const nusi_plan* pl, int* N, int* Nz, double* Enu)
{
    if (N) *N = pl->grid.N;
    if (Nz) *Nz = pl->grid.Nz;
    if (Enu) memcpy(Enu, pl->grid.Enu.data(), sizeof(double) * pl->grid.N);
    return NUSI_OK;
}

int nusi_plan_evolve(nusi_plan* pl, const nusi_params* pts, int n, double* d_flux, double* d_fla, void* stream)
{
    if (n < 1 || n > pl->max_points) return fail(NUSI_EPARAM, "number of points outside [1, max_points]");
    HIPCHECK(hipSetDevice(pl->device));
    pl->warn_host_valid = false;
    hipStream_t s = stream ? (hipStream_t)stream : pl->stream;
    if (pl->ran) {
        HIPCHECK(hipEventSynchronize(pl->ev_copy));          // the pinned h_pts / h_tpts / h_batches are reused
        HIPCHECK(hipStreamWaitEvent(s, pl->ev_done, 0));     // so are d_pts, the tables and the warnings: one plan
    }                                                        // serialises its calls, whatever streams they use
    for (int i = 0; i < n; ++i) {
        const int r = build_point(pl, pts[i], pl->h_pts[i]);
        if (r) return r;
    }
    // one Stage-A table per distinct (mphi, g, Gamma_phi, masses, |U|^2, flags): the tables do not
    // depend on si, norm or the source (nuSIprop.hpp:217-253), so e.g. a gamma scan shares them
    std::map<TableKey, int> slots;
    pl->slot_of.resize(n);
    int ntab = 0;
    for (int i = 0; i < n; ++i) {
        nusi::Point& P = pl->h_pts[i];
        const TableKey key = table_key(P);
        auto it = slots.find(key);
        if (it == slots.end()) {
            it = slots.emplace(key, ntab).first;
            pl->h_tpts[ntab++] = P;
        }
        P.tslot = it->second;
        pl->slot_of[i] = it->second;
    }
    // NUSI_OPT_SHIFT_REUSE (opt-in): the tables a shifted base set serves go to the slots
    // [nd, ntab) (filled by k_table_shift), the others are built directly in [0, nd)
    int nd = ntab, nbase = 0;
    if (pl->shift_max > 0) {
        std::vector<int> remap;
        std::vector<nusi::Point> bases;
        std::vector<int2> smap;
        nd = shift_groups(pl, ntab, remap, smap, bases);
        nbase = (int)bases.size();
        if (nbase) {
            const int r = ensure_shift_plan(pl, nbase);
            if (r) return r;
            if (nbase > pl->shift->max_points) return fail(NUSI_EPARAM, "shift reuse: more base tables than the base plan holds");
            std::vector<nusi::Point> tmp(pl->h_tpts, pl->h_tpts + ntab);
            for (int j = 0; j < ntab; ++j) pl->h_tpts[remap[j]] = tmp[j];
            for (int j = 0; j < ntab; ++j) pl->h_tpts[j].tslot = j;
            for (int i = 0; i < n; ++i) pl->h_pts[i].tslot = pl->slot_of[i] = remap[pl->slot_of[i]];
            // the base plan's tables, ordered and batched like any others (their slots move: remap the map)
            nusi_plan* sp = pl->shift;
            sp->spl = pl->spl;   // (the phi-phi set may have been loaded after the base plan was made)
            sp->alpha_batch = pl->alpha_batch;   // (and the alpha options may have changed since)
            sp->alpha_kind = pl->alpha_kind;
            if (sp->ran) HIPCHECK(hipEventSynchronize(sp->ev_copy));
            for (int b = 0; b < nbase; ++b) {
                sp->h_tpts[b] = bases[b];
                sp->h_tpts[b].tslot = b;
            }
            std::vector<int> bperm;
            const AlphaBatches bb = alpha_batches(sp, nbase, bperm);
            for (int q = 0; q < ntab - nd; ++q) pl->h_smap[q] = make_int2(bperm[smap[q].x], smap[q].y);
            pl->shift_batches = bb;
        }
        if (!nbase) nd = ntab;
    }
    // the directly built tables, ordered so that those sharing m_phi, the masses and the flags -- whose alpha
    // tables share every leaf of (S', t) alone -- are neighbours, and cut into batches
    std::vector<int> perm;
    const AlphaBatches ab = alpha_batches(pl, nd, perm);
    for (int i = 0; i < n; ++i)
        if (pl->slot_of[i] < nd) pl->h_pts[i].tslot = pl->slot_of[i] = perm[pl->slot_of[i]];
    const int cap = ab.cap, nbatch = ab.nbatch, nb_plain = ab.nb_plain;
    const size_t N3 = (size_t)3 * pl->grid.N;
    if (!d_flux || !d_fla) {
        if (!pl->d_scratch) HIPCHECK(hipMalloc(&pl->d_scratch, sizeof(double) * 2 * N3 * pl->max_points));
        if (!d_flux) d_flux = pl->d_scratch;
        if (!d_fla) d_fla = pl->d_scratch + N3 * pl->max_points;
    }
    // the cascade.  AUTO / MFMA: the block-synchronous MFMA cascade k_cascade_bs for every point kind -- the points of
    // a table slot in workgroups of up to 16 (>= 3 points: the gamma batch), pairs, or one per workgroup
    // (NUSI_OPT_CASCADE_RHS caps the group size; NUSI_OPT_STEP_PASSES = 1: one point per workgroup on the
    // step-pass instance), any source and scattering mode, step passes on long grids.  WAVEFRONT / REG / LDS, and a
    // grid k_cascade_bs does not fit: the bit-exact scalar cascade k_cascade.
    const int kind = pl->cascade_kind == NUSI_CASCADE_AUTO ? NUSI_CASCADE_MFMA : pl->cascade_kind;
    bool any_dsnb = false, all_nr = true;
    for (int i = 0; i < n; ++i) {
        any_dsnb = any_dsnb || pl->h_pts[i].source == NUSI_SOURCE_DSNB;
        all_nr = all_nr && pl->h_pts[i].non_resonant;
    }
    const bool force_passes = pl->step_passes == 1;
    const bool bs = kind == NUSI_CASCADE_MFMA && nusi::cascade_bs_config(pl->gd, 1, force_passes) != 0;
    int ngb = 0, ngidx = 0;
    int bs_nwg[3] = {0, 0, 0};   // workgroups of P = 16, 2, 1 (their groups in h_gbgrp in that order)
    if (bs) {
        const int rmax = force_passes ? 1 : pl->cascade_rhs == 0 ? 16 : pl->cascade_rhs;
        const bool g16 = rmax >= 3 && nusi::cascade_bs_config(pl->gd, 16, false) != 0;
        const bool g2 = rmax >= 2 && nusi::cascade_bs_config(pl->gd, 2, false) != 0;
        std::vector<std::vector<int>> by(ntab);
        for (int i = 0; i < n; ++i) by[pl->h_pts[i].tslot].push_back(i);
        std::vector<std::vector<int>> grs[3];   // groups for P = 16, 2, 1
        for (int j = 0; j < ntab; ++j) {
            const int c = (int)by[j].size();
            const int cap = (g16 && c >= 3) ? std::min(rmax, 16) : (g2 && c >= 2) ? 2 : 1;
            const int nb = (c + cap - 1) / cap;   // near-equal groups
            for (int k = 0; k < nb; ++k) {
                const int lo = (int)((long long)c * k / nb), hi = (int)((long long)c * (k + 1) / nb);
                const int sz = hi - lo, w = sz >= 3 ? 0 : sz == 2 ? 1 : 2;
                grs[w].emplace_back(by[j].begin() + lo, by[j].begin() + hi);
            }
        }
        size_t fhd = 0;
        const int Pk[3] = {16, 2, 1};
        for (int w = 0; w < 3; ++w) {
            for (const auto& gp : grs[w]) {
                pl->h_gbgrp[ngb++] = make_int2(ngidx, (int)gp.size());
                for (int i : gp) pl->h_gidx[ngidx++] = i;
            }
            bs_nwg[w] = (int)grs[w].size();
            fhd += nusi::cascade_bs_scratch_doubles(pl->gd, Pk[w]) * grs[w].size();
        }
        if (fhd > pl->fh_doubles) {
            hipFree(pl->d_fh);
            pl->d_fh = nullptr;
            pl->fh_doubles = 0;
            HIPCHECK(hipMalloc(&pl->d_fh, sizeof(double) * fhd));
            pl->fh_doubles = fhd;
        }
    }
    if (bs && any_dsnb && pl->src_cap < pl->max_points) {
        hipFree(pl->d_src);
        pl->d_src = nullptr;
        pl->src_cap = 0;
        HIPCHECK(hipMalloc(&pl->d_src, sizeof(double) * nusi::cascade_src_doubles(pl->gd) * pl->max_points));
        pl->src_cap = pl->max_points;
        pl->tabs.Src = pl->d_src;
    }
    // NUSI_OPT_REFERENCE_ORDER on the big-batch kernel: the member-corner blocks sized (allocations, the edge maps'
    // synchronous upload) before the first event of the call and before any fork to the side stream
    const bool refo = pl->ref_order != 0;
    const bool mcorn = refo && pl->alpha_kind == 0;
    if (mcorn && nd && nbatch) {
        AlphaBatches ab;
        ab.nbatch = nbatch;
        if (int r = mcorner_ensure(pl, nd, ab, pl->corner_mb)) return r;
    }
    if (mcorn && nbase && pl->shift_batches.nbatch)
        if (int r = mcorner_ensure(pl->shift, nbase, pl->shift_batches, pl->corner_mb)) return r;
    // a call of few tables without the phi-phi channel: the k-split alpha path (TablesDev::Kt, 8 doubles per entry,
    // mass state and table; 11.5 MB per table at N_E = 300); scans keep the k loop inside the workgroup
    pl->tabs.Kt = nullptr;
    if (nbase == 0 && nd > 0 && nd <= kSplitTables && nb_plain == nbatch && pl->alpha_kind == 0) {
        const size_t need = (size_t)8 * 3 * (size_t)pl->gd.PT * nd;
        if (pl->kt_doubles < need) {
            hipFree(pl->d_kt);
            pl->d_kt = nullptr;
            pl->kt_doubles = 0;
            HIPCHECK(hipMalloc(&pl->d_kt, sizeof(double) * need));
            pl->kt_doubles = need;
        }
        pl->tabs.Kt = pl->d_kt;
    }
    // a call of few tables in the reference order: Gamma / alphaTilde's GSL dilogarithms one per work-item first
    // (k_ga_dilogs; 2.2 MB per table at N_E = 300)
    pl->tabs.Gpre = nullptr;
#ifndef NUSI_GA_PRE_ALL
#define NUSI_GA_PRE_ALL 0
#endif
    if (kGaPre && refo && nbase == 0 && nd > 0 && (nd <= kOverlapTables || NUSI_GA_PRE_ALL)) {
        const size_t need = nusi::gamma_alphat_pre_doubles(pl->gd.T, nd);
        if (pl->gpre_doubles < need) {
            hipFree(pl->d_gpre);
            pl->d_gpre = nullptr;
            pl->gpre_doubles = 0;
            HIPCHECK(hipMalloc(&pl->d_gpre, sizeof(double) * need));
            pl->gpre_doubles = need;
        }
        pl->tabs.Gpre = pl->d_gpre;
    }
    // one upload: the zeroed warnings, batches, gamma groups, points and tables (nusi_plan::d_in)
    HIPCHECK(hipMemcpyAsync(pl->d_in, pl->h_in, pl->in_tpts + sizeof(nusi::Point) * ntab, hipMemcpyHostToDevice, s));
    nusi_plan* sp = nbase ? pl->shift : nullptr;
    if (sp) {
        HIPCHECK(hipMemcpyAsync(pl->d_smap, pl->h_smap, sizeof(int2) * (ntab - nd), hipMemcpyHostToDevice, s));
        HIPCHECK(hipMemcpyAsync(sp->d_tpts, sp->h_tpts, sizeof(nusi::Point) * nbase, hipMemcpyHostToDevice, s));
        HIPCHECK(hipMemcpyAsync(sp->d_batches, sp->h_batches, sizeof(int) * pl->shift_batches.nbatch,
                                hipMemcpyHostToDevice, s));
        HIPCHECK(hipEventRecord(sp->ev_copy, s));
        HIPCHECK(hipMemsetAsync(sp->d_warn, 0, sizeof(int) * nbase, s));
        HIPCHECK(hipMemsetAsync(sp->tabs.Wmin, 0x7f, sizeof(int) * 4 * (size_t)sp->grid.T * nbase, s));   // no row warned
        sp->ran = true;
    }
    HIPCHECK(hipEventRecord(pl->ev_copy, s));
    const nusi::SplineSet* spl = pl->spl ? pl->spl->d_set : pl->d_nospl;
    hipEvent_t* ev = pl->ev;
    if (pl->prof_n < pl->prof_max) ev = &pl->prof_ev[4 * (size_t)pl->prof_n++];
    HIPCHECK(hipEventRecord(ev[0], s));
    // A call of few tables leaves most of the GPU idle in each Stage-A kernel: Gamma / alphaTilde (independent of
    // alpha) run on the side stream beside the alpha kernels, and the cascade waits for both.  (Stage times: ev[1]
    // is then Gamma / alphaTilde's end on the side stream, and the alpha stage counts from there.)  Scans keep the
    // stages in order: beside a full alpha launch the overlap measured no gain (C4 155.0 -> 155.4 k, round 4).
    const bool ovl = !sp && nd > 0 && nd <= kOverlapTables;
    // after a fork, any early error return still joins the side stream into s (the next call's memsets and table
    // writes on s must not race a still-running Gamma / alphaTilde kernel)
    struct SideJoin {
        hipStream_t s = nullptr, side = nullptr;
        hipEvent_t done = nullptr;
        bool armed = false;
        ~SideJoin()
        {
            if (!armed) return;
            if (hipEventRecord(done, side) != hipSuccess) (void)hipStreamSynchronize(side);
            else (void)hipStreamWaitEvent(s, done, 0);
        }
    } join{s, pl->side, pl->ev_fork, false};
    if (ovl) {
        HIPCHECK(hipEventRecord(pl->ev_fork, s));
        HIPCHECK(hipStreamWaitEvent(pl->side, pl->ev_fork, 0));
        join.armed = true;
        HIPCHECK(nusi::launch_gamma_alphat(pl->gd, pl->d_tpts, nd, spl, pl->tabs, pl->d_warn, pl->side, refo));
        HIPCHECK(hipEventRecord(ev[1], pl->side));
    } else {
        if (nd) HIPCHECK(nusi::launch_gamma_alphat(pl->gd, pl->d_tpts, nd, spl, pl->tabs, pl->d_warn, s, refo));
        if (sp) HIPCHECK(nusi::launch_gamma_alphat(sp->gd, sp->d_tpts, nbase, spl, sp->tabs, sp->d_warn, s, refo));
        HIPCHECK(hipEventRecord(ev[1], s));
    }
    if (nd) {
        HIPCHECK(nusi::launch_alpha(pl->gd, pl->d_tpts, nd, spl, pl->atiles, pl->tabs, pl->d_warn, s, pl->d_batches,
                                    nbatch, cap, pl->alpha_kind, nb_plain, refo, pl->h_batches, &pl->mc));
    }
    if (sp) {
        const AlphaBatches& bb = pl->shift_batches;
        HIPCHECK(nusi::launch_alpha(sp->gd, sp->d_tpts, nbase, spl, sp->atiles, sp->tabs, sp->d_warn, s, sp->d_batches,
                                    bb.nbatch, bb.cap, pl->alpha_kind, bb.nb_plain, refo, sp->h_batches, &sp->mc));
        HIPCHECK(nusi::launch_table_shift(pl->gd, sp->gd, pl->d_smap, nd, ntab - nd, sp->tabs, pl->tabs, pl->d_warn, s));
    }
    if (ovl) {
        join.armed = false;
        HIPCHECK(hipStreamWaitEvent(s, ev[1], 0));
    }
    HIPCHECK(hipEventRecord(ev[2], s));
    if (bs && any_dsnb) HIPCHECK(nusi::launch_source_dsnb(pl->gd, pl->d_pts, n, pl->d_src, s));
    const char* gb_name = nullptr;
    if (bs) {
        const int Pk[3] = {16, 2, 1};
        static const char* const names[8] = {"", "k_cascade_bs_gamma", "k_cascade_bs_pairs", "k_cascade_bs_gamma + pairs",
                                             "k_cascade_bs", "k_cascade_bs_gamma + k_cascade_bs",
                                             "k_cascade_bs_pairs + k_cascade_bs", "k_cascade_bs_gamma + pairs + k_cascade_bs"};
        int off = 0, mask = 0;
        double* fh = pl->d_fh;
        for (int w = 0; w < 3; ++w) {
            if (bs_nwg[w]) {
                HIPCHECK(nusi::launch_cascade_bs(pl->gd, pl->d_pts, Pk[w], pl->d_gidx, pl->d_gbgrp + off, bs_nwg[w], pl->tabs,
                                                 fh, d_flux, d_fla, s, all_nr, force_passes));
                mask |= 1 << w;
            }
            fh += nusi::cascade_bs_scratch_doubles(pl->gd, Pk[w]) * bs_nwg[w];
            off += bs_nwg[w];
        }
        gb_name = names[mask];
    } else {
        HIPCHECK(nusi::launch_cascade_exact(pl->gd, pl->d_pts, n, pl->tabs, d_flux, d_fla, s));
    }
    HIPCHECK(hipEventRecord(ev[3], s));
    HIPCHECK(hipEventRecord(pl->ev_done, s));
    pl->alpha_kernel = nusi::last_alpha_kernel();
    if (sp) {   // the label of the kernel that built the base tables (the base launch runs last)
        pl->alpha_label = std::string(nusi::last_alpha_kernel()) + (nd ? " + k_table_shift" : " (shift base) + k_table_shift");
        pl->alpha_kernel = pl->alpha_label.c_str();
    }
    pl->cascade_kernel = gb_name ? gb_name : nusi::last_cascade_kernel();
    for (int k = 0; k < 4; ++k) pl->last_ev[k] = ev[k];   // stage_ms / warnings / tables refer to the latest call
    pl->ran = true;
    pl->last_n = n;
    pl->last_ntab = ntab;
    return NUSI_OK;
}

int nusi_plan_profile_begin(nusi_plan* pl, int max_calls)
{
    HIPCHECK(hipSetDevice(pl->device));
    if (max_calls < 0) return fail(NUSI_EPARAM, "max_calls < 0");
    if ((int)pl->prof_ev.size() < 4 * max_calls) {
        const size_t old = pl->prof_ev.size();
        pl->prof_ev.resize(4 * (size_t)max_calls, nullptr);
        for (size_t k = old; k < pl->prof_ev.size(); ++k) HIPCHECK(hipEventCreate(&pl->prof_ev[k]));
    }
    pl->prof_max = max_calls;
    pl->prof_n = 0;
    return NUSI_OK;
}

int nusi_plan_profile_end(nusi_plan* pl, double* sum_ms3, int* ncalls)
{
    HIPCHECK(hipSetDevice(pl->device));
    for (int k = 0; k < 3; ++k) sum_ms3[k] = 0.0;
    for (int c = 0; c < pl->prof_n; ++c) {
        hipEvent_t* e = &pl->prof_ev[4 * (size_t)c];
        HIPCHECK(hipEventSynchronize(e[3]));
        for (int k = 0; k < 3; ++k) {
            float ms = 0.f;
            HIPCHECK(hipEventElapsedTime(&ms, e[k], e[k + 1]));
            sum_ms3[k] += ms;
        }
    }
    *ncalls = pl->prof_n;
    pl->prof_max = 0;
    pl->prof_n = 0;
    return NUSI_OK;
}

int nusi_plan_stage_ms(nusi_plan* pl, float* ms3)
{
    if (!pl->ran) return fail(NUSI_ESTATE, "no evolve has run on this plan");
    HIPCHECK(hipSetDevice(pl->device));
    HIPCHECK(hipEventSynchronize(pl->last_ev[3]));
    for (int k = 0; k < 3; ++k) HIPCHECK(hipEventElapsedTime(&ms3[k], pl->last_ev[k], pl->last_ev[k + 1]));
    return NUSI_OK;
}

int nusi_plan_set_cascade(nusi_plan* pl, int kind)
{
    if (!pl) return fail(NUSI_EPARAM, "plan is NULL");
    if (kind < NUSI_CASCADE_AUTO || kind > NUSI_CASCADE_MFMA) return fail(NUSI_EPARAM, "unknown cascade kind");
    pl->cascade_kind = kind;
    return NUSI_OK;
}

int nusi_plan_set_option(nusi_plan* pl, int option, int value)
{
    if (!pl) return fail(NUSI_EPARAM, "plan is NULL");
    switch (option) {
    case NUSI_OPT_ALPHA_BATCH:
        if (value < 0 || value > 255) return fail(NUSI_EPARAM, "NUSI_OPT_ALPHA_BATCH outside [0, 255]");
        pl->alpha_batch = value;
        return NUSI_OK;
    case NUSI_OPT_ALPHA_KERNEL:
        if (value < 0 || value > 2) return fail(NUSI_EPARAM, "NUSI_OPT_ALPHA_KERNEL outside [0, 2]");
        pl->alpha_kind = value;
        return NUSI_OK;
    case NUSI_OPT_CASCADE_RHS:
        if (value < 0 || value > 16) return fail(NUSI_EPARAM, "NUSI_OPT_CASCADE_RHS outside [0, 16]");
        pl->cascade_rhs = value;
        return NUSI_OK;
    case NUSI_OPT_STEP_PASSES:
        if (value < 0 || value > 1) return fail(NUSI_EPARAM, "NUSI_OPT_STEP_PASSES outside [0, 1]");
        pl->step_passes = value;
        return NUSI_OK;
    case NUSI_OPT_CASCADE_SYNC:
        if (value < 0 || value > 2) return fail(NUSI_EPARAM, "NUSI_OPT_CASCADE_SYNC outside [0, 2]");
        if (value == 1)   // the per-stage kernels (k_cascade_ws / gb / wsp) were removed in round 5
            return fail(NUSI_EPARAM, "NUSI_OPT_CASCADE_SYNC = 1: the per-stage cascade kernels are gone; k_cascade_bs is the MFMA cascade");
        pl->cascade_sync = value;
        return NUSI_OK;
    case NUSI_OPT_REFO_CORNER_MB:
        if (value < 0 || value > (1 << 20)) return fail(NUSI_EPARAM, "NUSI_OPT_REFO_CORNER_MB outside [0, 2^20]");
        pl->corner_mb = value;
        return NUSI_OK;
    case NUSI_OPT_REFERENCE_ORDER:
        if (value < 0 || value > 1) return fail(NUSI_EPARAM, "NUSI_OPT_REFERENCE_ORDER outside [0, 1]");
        pl->ref_order = value;
        return NUSI_OK;
    case NUSI_OPT_SHIFT_REUSE:
        if (value < 0 || value > 128) return fail(NUSI_EPARAM, "NUSI_OPT_SHIFT_REUSE outside [0, 128]");
        if (value != pl->shift_max && pl->shift) {   // the base plan's axis follows K
            if (pl->ran) {
                HIPCHECK(hipSetDevice(pl->device));
                HIPCHECK(hipEventSynchronize(pl->ev_done));
            }
            nusi_plan_destroy(pl->shift);
            pl->shift = nullptr;
        }
        pl->shift_max = value;
        return NUSI_OK;
    default:
        return fail(NUSI_EPARAM, "unknown plan option");
    }
}

int nusi_plan_warnings(nusi_plan* pl, int* out, int n)
{
    if (!pl->ran) return fail(NUSI_ESTATE, "no evolve has run on this plan");
    if (n > pl->last_n) n = pl->last_n;
    if (pl->warn_host_valid) {   // (fetched by nusi_plan_evolve_host with the fluxes)
        for (int i = 0; i < n; ++i) out[i] = pl->warn_host[pl->slot_of[i]];
        return NUSI_OK;
    }
    HIPCHECK(hipSetDevice(pl->device));
    HIPCHECK(hipEventSynchronize(pl->last_ev[3]));
    std::vector<int> w(pl->last_ntab);
    HIPCHECK(hipMemcpy(w.data(), pl->d_warn, sizeof(int) * w.size(), hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) out[i] = w[pl->slot_of[i]];
    return NUSI_OK;
}

int nusi_plan_kernels(const nusi_plan* pl, const char** alpha, const char** cascade)
{
    if (!pl->ran) return fail(NUSI_ESTATE, "no evolve has run on this plan");
    if (alpha) *alpha = pl->alpha_kernel;
    if (cascade) *cascade = pl->cascade_kernel;
    return NUSI_OK;
}

int nusi_plan_tables(nusi_plan* pl, int i, double* G, double* At, double* A)
{
    if (!pl->ran) return fail(NUSI_ESTATE, "no evolve has run on this plan");
    if (i < 0 || i >= pl->last_n) return fail(NUSI_EPARAM, "point index out of range");
    HIPCHECK(hipSetDevice(pl->device));
    HIPCHECK(hipEventSynchronize(pl->last_ev[3]));
    const size_t T = (size_t)pl->gd.T, PT = (size_t)pl->gd.PT, j = (size_t)pl->slot_of[i];
    if (G) HIPCHECK(hipMemcpy(G, pl->tabs.G + T * j, sizeof(double) * T, hipMemcpyDeviceToHost));
    if (At) HIPCHECK(hipMemcpy(At, pl->tabs.At + T * j, sizeof(double) * T, hipMemcpyDeviceToHost));
    if (A) HIPCHECK(hipMemcpy(A, pl->tabs.A + PT * j, sizeof(double) * PT, hipMemcpyDeviceToHost));
    return NUSI_OK;
}

int nusi_plan_evolve_host(nusi_plan* pl, const nusi_params* pts, int n, double* flux, double* fla)
{
    int r = nusi_plan_evolve(pl, pts, n, nullptr, nullptr, nullptr);
    if (r) return r;
    const size_t N3 = (size_t)3 * pl->grid.N, fb = sizeof(double) * N3 * n;
    const size_t wb = (sizeof(int) * pl->last_ntab + 255) & ~(size_t)255;
    hipStream_t s = pl->stream;
    const double* dflux = pl->d_scratch;
    const double* dfla = pl->d_scratch + N3 * pl->max_points;
    pl->warn_host.resize(pl->last_ntab);
    if (wb + 2 * fb <= kStageBytes) {
        // small calls (the object API's single propagation): the warnings and both flux arrays into one pinned
        // staging buffer, one synchronisation, then host copies (pageable hipMemcpy round trips cost ~20 us each)
        if (pl->h_out_bytes < wb + 2 * fb) {
            if (pl->h_out) HIPCHECK(hipHostFree(pl->h_out));
            pl->h_out = nullptr;
            pl->h_out_bytes = 0;
            HIPCHECK(hipHostMalloc((void**)&pl->h_out, wb + 2 * fb, hipHostMallocDefault));
            pl->h_out_bytes = wb + 2 * fb;
        }
        HIPCHECK(hipMemcpyAsync(pl->h_out, pl->d_warn, sizeof(int) * pl->last_ntab, hipMemcpyDeviceToHost, s));
        if (n == pl->max_points)   // flux and flux_fla adjacent in d_scratch
            HIPCHECK(hipMemcpyAsync(pl->h_out + wb, dflux, 2 * fb, hipMemcpyDeviceToHost, s));
        else {
            HIPCHECK(hipMemcpyAsync(pl->h_out + wb, dflux, fb, hipMemcpyDeviceToHost, s));
            HIPCHECK(hipMemcpyAsync(pl->h_out + wb + fb, dfla, fb, hipMemcpyDeviceToHost, s));
        }
        HIPCHECK(hipStreamSynchronize(s));
        memcpy(pl->warn_host.data(), pl->h_out, sizeof(int) * pl->last_ntab);
        if (flux) memcpy(flux, pl->h_out + wb, fb);
        if (fla) memcpy(fla, pl->h_out + wb + fb, fb);
    } else {
        HIPCHECK(hipStreamSynchronize(s));
        HIPCHECK(hipMemcpy(pl->warn_host.data(), pl->d_warn, sizeof(int) * pl->last_ntab, hipMemcpyDeviceToHost));
        if (flux) HIPCHECK(hipMemcpy(flux, dflux, fb, hipMemcpyDeviceToHost));
        if (fla) HIPCHECK(hipMemcpy(fla, dfla, fb, hipMemcpyDeviceToHost));
    }
    pl->warn_host_valid = true;
    int bad = 0;
    for (int v : pl->warn_host) bad |= (v & nusi::kWarnSplineOOB);
    if (bad) return fail(NUSI_EINTERP, "Error at interp: a phi-phi table lookup fell outside the node range");
    return NUSI_OK;
}

int nusi_evolve_batch(int device, const nusi_params* pts, int n, double* flux, double* fla)
{
    if (n < 1) return fail(NUSI_EPARAM, "n must be >= 1");
    nusi_plan* pl = nullptr;
    int r = nusi_plan_create(device, pts[0].N_bins_E, pts[0].lEmin, pts[0].lEmax, pts[0].zmax, n, &pl);
    if (r) return r;
    r = nusi_plan_evolve_host(pl, pts, n, flux, fla);
    nusi_plan_destroy(pl);
    return r;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// object API
// ---------------------------------------------------------------------------
// One-point plans of destroyed objects are kept for the next object on the same device and grid (the reference
// builds a calculate_flux per parameter point in its own usage, test.py: a fresh plan costs ~a dozen device
// allocations, a stream and the grid upload).  A plan is handed out with the options at their defaults and no
// phi-phi tables; its buffers are overwritten by the next evolve.  At most kPlanPoolMax are kept; the pool is never
// torn down (process exit reclaims the device).
namespace {
constexpr size_t kPlanPoolMax = 8;
struct PlanPool {
    std::mutex mu;
    std::vector<nusi_plan*> free;
};
PlanPool& plan_pool()
{
    static PlanPool* p = new PlanPool;
    return *p;
}
nusi_plan* pool_take(int dev, int N, double lEmin, double lEmax, double zmax)
{
    PlanPool& pp = plan_pool();
    std::lock_guard<std::mutex> lock(pp.mu);
    for (size_t i = 0; i < pp.free.size(); ++i) {
        nusi_plan* pl = pp.free[i];
        const HostGrid& G = pl->grid;
        if (pl->device == dev && G.N == N && G.lEmin == lEmin && G.lEmax == lEmax && G.zmax_in == zmax) {
            pp.free.erase(pp.free.begin() + (long)i);
            return pl;
        }
    }
    return nullptr;
}
void pool_give(nusi_plan* pl)
{
    if (!pl) return;
    if (pl->max_points == 1 && !pl->shift) {
        // the defaults of nusi_plan_create
        pl->alpha_batch = pl->alpha_kind = pl->cascade_rhs = pl->step_passes = pl->shift_max = 0;
        pl->cascade_sync = pl->corner_mb = 0;
        pl->ref_order = 1;
        pl->cascade_kind = NUSI_CASCADE_AUTO;
        pl->prof_max = pl->prof_n = 0;
        pl->spl.reset();
        PlanPool& pp = plan_pool();
        std::lock_guard<std::mutex> lock(pp.mu);
        if (pp.free.size() < kPlanPoolMax) {
            pp.free.push_back(pl);
            return;
        }
    }
    nusi_plan_destroy(pl);
}
}  // namespace

struct nusi_handle {
    nusi_params p{};
    nusi_plan* plan = nullptr;
    std::vector<double> flux, fla;
    double norm_total = 0.0;   // of the last evolve() (stale in check_energy_conservation)
    bool evolved = false;      // an evolve() has run (norm_total is set)
    int warn = 0;
    std::map<int, int> opts;   // the last value nusi_set_option set per option, replayed by nusi_copy
    std::string alpha_kernel, cascade_kernel;   // what this object's last evolve() launched (copied by nusi_copy;
                                                // the pooled plan of a copy may have run another object's call)
    ~nusi_handle() { pool_give(plan); }
};

extern "C" {

static int open_handle(const nusi_params* p, const std::shared_ptr<SplineStore>* share, nusi_handle** out)
{
    *out = nullptr;
    if (p->flav < 0 || p->flav > 2) return fail(NUSI_EPARAM, "flav must be 0, 1 or 2");
    int dev = 0;
    if (const char* e = getenv("NUSI_DEVICE")) dev = atoi(e);
    std::unique_ptr<nusi_handle> h(new nusi_handle);
    h->p = *p;
    int r = NUSI_OK;
    h->plan = pool_take(dev, p->N_bins_E, p->lEmin, p->lEmax, p->zmax);
    if (!h->plan) r = nusi_plan_create(dev, p->N_bins_E, p->lEmin, p->lEmax, p->zmax, 1, &h->plan);
    if (r) return r;
    if (p->non_resonant && p->phiphi) {   // nuSIprop.hpp:166-170
        if (share && *share) h->plan->spl = *share;
        else {
            std::string dir = "xsec";
            if (const char* e = getenv("NUSI_XSEC_DIR")) dir = e;
            r = nusi_plan_load_phiphi(h->plan, (dir + "/alphatilde_phiphi.bin").c_str(), nullptr,
                                      (dir + "/alpha_phiphi.bin").c_str(), nullptr);
            if (r) return r;
        }
    }
    h->flux.assign((size_t)3 * p->N_bins_E, 0.0);
    h->fla.assign((size_t)3 * p->N_bins_E, 0.0);
    *out = h.release();
    return NUSI_OK;
}

int nusi_create(const nusi_params* p, nusi_handle** out) { return open_handle(p, nullptr, out); }

int nusi_copy(const nusi_handle* src, nusi_handle** out)
{
    int r = open_handle(&src->p, &src->plan->spl, out);
    if (r) return r;
    (*out)->flux = src->flux;
    (*out)->fla = src->fla;
    (*out)->norm_total = src->norm_total;
    (*out)->evolved = src->evolved;
    (*out)->warn = src->warn;
    (*out)->alpha_kernel = src->alpha_kernel;
    (*out)->cascade_kernel = src->cascade_kernel;
    for (const auto& o : src->opts) {
        r = nusi_set_option(*out, o.first, o.second);
        if (r) {
            nusi_destroy(*out);
            *out = nullptr;
            return r;
        }
    }
    return NUSI_OK;
}

void nusi_destroy(nusi_handle* h) { delete h; }

int nusi_set_params(nusi_handle* h, double mphi, double g, double mntot, double si, double norm)
{
    h->p.mphi = mphi;
    h->p.g = g;
    h->p.mntot = mntot;
    h->p.si = si;
    h->p.norm = norm;
    return NUSI_OK;
}

int nusi_get_params(const nusi_handle* h, double* v)
{
    v[0] = h->p.mphi;
    v[1] = h->p.g;
    v[2] = h->p.mntot;
    v[3] = h->p.si;
    v[4] = h->p.norm;
    return NUSI_OK;
}

int nusi_evolve(nusi_handle* h)
{
    int r = nusi_plan_evolve_host(h->plan, &h->p, 1, h->flux.data(), h->fla.data());
    if (r) return r;
    h->norm_total = h->plan->h_pts[0].norm_total;
    h->evolved = true;
    h->alpha_kernel = h->plan->alpha_kernel;
    h->cascade_kernel = h->plan->cascade_kernel;
    int w = 0;
    r = nusi_plan_warnings(h->plan, &w, 1);
    h->warn = w & (NUSI_WARN_GAMMA | NUSI_WARN_ALPHATILDE | NUSI_WARN_ALPHA);
    return r;
}

int nusi_check_energy_conservation(nusi_handle* h, double* out)
{
    const HostGrid& G = h->plan->grid;
    // the reference evaluates E_FS with the previous evolve()'s norm_total (nuSIprop.hpp:341-343)
    const bool unset = !h->evolved;
    const double E_FS = energy_fs(h->p.si, h->norm_total, G.zmax_eff, G.lEmin, G.lEmax);
    int r = nusi_evolve(h);
    if (r) return r;
    if (unset) {   // deliberate difference: the reference reads an uninitialised member here (inf / garbage)
        *out = NAN;
        return fail(NUSI_ESTATE, "check_energy_conservation before any evolve(): norm_total is not set "
                                 "(the reference reads it uninitialised); evolved now, result NaN");
    }
    double E_int = 0;
    const int N = G.N;
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < 3; ++k) E_int += (log(G.Emax[i]) - log(G.Emin[i])) * sq(G.Enu[i]) * h->flux[(size_t)k * N + i];
    *out = (E_int - E_FS) / E_FS;
    return NUSI_OK;
}

int nusi_get_flux(const nusi_handle* h, double* out)
{
    memcpy(out, h->flux.data(), sizeof(double) * h->flux.size());
    return NUSI_OK;
}
int nusi_get_flux_fla(const nusi_handle* h, double* out)
{
    memcpy(out, h->fla.data(), sizeof(double) * h->fla.size());
    return NUSI_OK;
}
int nusi_get_energies(const nusi_handle* h, double* out)
{
    memcpy(out, h->plan->grid.Enu.data(), sizeof(double) * h->plan->grid.N);
    return NUSI_OK;
}
int nusi_get_N_bins_E(const nusi_handle* h) { return h->plan->grid.N; }
int nusi_get_N_steps_z(const nusi_handle* h) { return h->plan->grid.Nz; }
int nusi_get_warnings(const nusi_handle* h) { return h->warn; }
int nusi_set_option(nusi_handle* h, int option, int value)
{
    const int r = nusi_plan_set_option(h->plan, option, value);
    if (r == NUSI_OK) h->opts[option] = value;
    return r;
}

int nusi_get_kernels(const nusi_handle* h, const char** alpha, const char** cascade)
{
    if (!h->evolved) return fail(NUSI_ESTATE, "no evolve has run on this object");
    if (alpha) *alpha = h->alpha_kernel.c_str();
    if (cascade) *cascade = h->cascade_kernel.c_str();
    return NUSI_OK;
}

}  // extern "C"
