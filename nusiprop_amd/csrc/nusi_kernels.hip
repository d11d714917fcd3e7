// nuSIprop MI355X -- HIP kernels for calculate_flux::evolve() (nuSIprop.hpp:176-337).
//
//   k_gamma_alphat  Stage A, absorption + same-bin regeneration tables   (:217-235)
//   k_alpha         Stage A, inter-bin regeneration table, one entry per
//                   work-item, packed transposed                          (:237-252)
//   k_cascade       Stage B, the implicit redshift cascade + finalisation (:255-336),
//                   one wavefront per parameter point
#include <hip/hip_runtime.h>

#include "nusi_internal.hpp"

namespace nusi {

// ---------------------------------------------------------------------------
// Stage A
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_gamma_alphat(GridDev g, const Point* __restrict__ pts, SplineSet spl,
                                                     double* __restrict__ G, double* __restrict__ At,
                                                     int* __restrict__ warn)
{
    const int p = blockIdx.y;
    const int n = blockIdx.x * 64 + threadIdx.x;
    if (n >= g.T) return;
    const Point& P = pts[p];
    int w = 0;
    const double lo = g.lo[n], hi = g.hi[n];
    G[(size_t)p * g.T + n] = gamma_entry(P, lo, hi, w);
    At[(size_t)p * g.T + n] = alphat_entry(P, spl, lo, hi, w);
    if (w) atomicOr(&warn[p], w);
}

__global__ __launch_bounds__(256) void k_alpha(GridDev g, const Point* __restrict__ pts, SplineSet spl,
                                               double* __restrict__ A, int* __restrict__ warn)
{
    const int p = blockIdx.y;
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    if (e >= g.PT) return;
    // packed transposed index e = m(m-1)/2 + n, n < m
    int m = (int)((1.0 + sqrt(1.0 + 8.0 * (double)e)) * 0.5);
    while ((long long)m * (m - 1) / 2 > e) --m;
    while ((long long)(m + 1) * m / 2 <= e) ++m;
    const int n = (int)(e - (long long)m * (m - 1) / 2);
    const Point& P = pts[p];
    int w = 0;
    double v = 0.0;
    // without non-s channels the cascade reads only alpha(n, n+1) (nuSIprop.hpp:273-275)
    if (P.non_resonant || m == n + 1) v = alpha_entry(P, spl, g.lo[n], g.hi[n], g.lo[m], g.hi[m], w);
    A[(size_t)p * g.PT + e] = v;
    if (w) atomicOr(&warn[p], w);
}

hipError_t launch_gamma_alphat(const GridDev& g, const Point* pts, int npts, const SplineSet& spl, TablesDev t,
                               int* warn, hipStream_t s)
{
    dim3 grid((g.T + 63) / 64, npts);
    hipLaunchKernelGGL(k_gamma_alphat, grid, dim3(64), 0, s, g, pts, spl, t.G, t.At, warn);
    return hipGetLastError();
}

hipError_t launch_alpha(const GridDev& g, const Point* pts, int npts, const SplineSet& spl, TablesDev t, int* warn,
                        hipStream_t s)
{
    dim3 grid((unsigned)((g.PT + 255) / 256), npts);
    hipLaunchKernelGGL(k_alpha, grid, dim3(256), 0, s, g, pts, spl, t.A, warn);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Stage B -- the cascade.
//
// For each redshift step i (sequential, z_max -> 0) the bins are swept from
// the top down; bin b needs the already-updated bins m > b of the same step
// (nuSIprop.hpp:289-291), i.e. an upper-triangular solve.  It is done
// right-looking: as soon as bin b is final, its weight
//     T_b = s_i * sum_l u_l F_l[b] / dE_b
// is pushed into every lower bin's accumulator acc[b'] += alpha(b', b) T_b
// (one coalesced column read of the packed transposed table per bin), so the
// sequential chain per bin is only the 3x3 solve.  Everything that does not
// depend on the flux (Zdr, the LU of M, the source term) is precomputed for
// 64 bins at a time, one bin per lane, into LDS.
//
// One wavefront (64 lanes) per point; F[3][N] and acc[N] live in LDS.
// ---------------------------------------------------------------------------
constexpr int kPreFields = 14;
enum { PR_RZ0, PR_RZ1, PR_RZ2, PR_SRC, PR_L10, PR_L20, PR_L21, PR_U01, PR_U02, PR_U12, PR_RU00, PR_RU11, PR_RU22, PR_SDE };

size_t cascade_lds_bytes(int N) { return sizeof(double) * (4 * (size_t)N + kPreFields * 64) + sizeof(int) * 64; }

// gsl_linalg_LU_decomp on 3x3 (partial pivoting, Doolittle), nuSIprop.hpp:309
NUSI_FN void lu3_factor(double A[3][3], int perm[3])
{
    perm[0] = 0; perm[1] = 1; perm[2] = 2;
    for (int j = 0; j < 2; ++j) {
        double amax = fabs(A[j][j]);
        int ip = j;
        for (int i = j + 1; i < 3; ++i)
            if (fabs(A[i][j]) > amax) { amax = fabs(A[i][j]); ip = i; }
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
}

__global__ __launch_bounds__(64) void k_cascade(GridDev g, const Point* __restrict__ pts, TablesDev t,
                                                double* __restrict__ flux, double* __restrict__ flux_fla)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int N = g.N, Nz = g.Nz, T = g.T;
    const int p = blockIdx.x, lane = threadIdx.x;
    const Point& P = pts[p];
    double* F0 = lds;
    double* F1 = lds + N;
    double* F2 = lds + 2 * N;
    double* acc = lds + 3 * N;
    double* pre = lds + 4 * N;
    int* perm = (int*)(pre + kPreFields * 64);
    const double u0 = P.u[0], u1 = P.u[1], u2 = P.u[2];
    const double uk[3] = {u0, u1, u2};
    const double* __restrict__ Gt = t.G + (size_t)p * T;
    const double* __restrict__ At = t.At + (size_t)p * T;
    const double* __restrict__ Al = t.A + (size_t)p * g.PT;
    const bool nonres = P.non_resonant;

    for (int b = lane; b < N; b += 64) F0[b] = F1[b] = F2[b] = 0.0;

    for (int i = Nz - 1; i > 0; --i) {
        const double c = g.step_c[i], s = g.step_s[i], zi = g.z[i], sfri = g.sfr[i];
        for (int b = lane; b < N; b += 64) acc[b] = 0.0;
        double next_acc = 0.0;     // acc of the next (lower) bin, carried in registers
        double racc = 0.0;         // resonant-only running sum (nuSIprop.hpp:261-278)
        double px0 = 0.0, px1 = 0.0, px2 = 0.0;   // F[:, b+1] of this step
        for (int base = ((N - 1) / 64) * 64; base >= 0; base -= 64) {
            __syncthreads();
            {   // ---- parallel: flux-independent quantities for bins base..base+63
                const int b = base + lane;
                if (b < N) {
                    const double dEb = g.Emax[b] - g.Emin[b];
                    const double Gw = s * Gt[b + i - 1], Aw = s * At[b + i - 1];
                    double Zd[3], M[3][3];
                    for (int k = 0; k < 3; ++k) Zd[k] = 1.0 + c * (Gw * uk[k] - Aw * (uk[k] * uk[k])) / dEb;
                    for (int k = 0; k < 3; ++k)
                        for (int l = 0; l < 3; ++l) M[k][l] = (k == l) ? 1.0 : (Aw * uk[k] * uk[l] / dEb) / Zd[k];
                    int pm[3];
                    lu3_factor(M, pm);
                    const double src0 = c * lum(P, zi, sfri, g.Emin[b], g.Emax[b]);
                    pre[PR_RZ0 * 64 + lane] = 1.0 / Zd[0];
                    pre[PR_RZ1 * 64 + lane] = 1.0 / Zd[1];
                    pre[PR_RZ2 * 64 + lane] = 1.0 / Zd[2];
                    pre[PR_SRC * 64 + lane] = src0;
                    pre[PR_L10 * 64 + lane] = M[1][0];
                    pre[PR_L20 * 64 + lane] = M[2][0];
                    pre[PR_L21 * 64 + lane] = M[2][1];
                    pre[PR_U01 * 64 + lane] = M[0][1];
                    pre[PR_U02 * 64 + lane] = M[0][2];
                    pre[PR_U12 * 64 + lane] = M[1][2];
                    pre[PR_RU00 * 64 + lane] = 1.0 / M[0][0];
                    pre[PR_RU11 * 64 + lane] = 1.0 / M[1][1];
                    pre[PR_RU22 * 64 + lane] = 1.0 / M[2][2];
                    pre[PR_SDE * 64 + lane] = nonres ? s / dEb : dEb;
                    perm[lane] = pm[0] | (pm[1] << 2) | (pm[2] << 4);
                }
            }
            __syncthreads();
            const int top = (base + 63 < N - 1) ? base + 63 : N - 1;
            for (int b = top; b >= base; --b) {
                const int l = b - base;
                const double accb_lds = (b > 0) ? acc[b - 1] : 0.0;   // for next_acc (before this bin's pushes)
                double src0 = pre[PR_SRC * 64 + l];
                double add;   // c * (coupling of this bin to the bins above)
                if (nonres) {
                    add = c * next_acc;
                } else {
                    if (b != N - 1) {
                        const double Sres = u0 * px0 + u1 * px1 + u2 * px2;
                        const size_t rd = (size_t)(b + i) * (b + i - 1) / 2 + (b + i - 1);   // alpha(b+i-1, b+i)
                        racc += Sres * (s * Al[rd]) / (g.Emax[b + 1] - g.Emin[b + 1]) / pre[PR_SDE * 64 + l];
                    }
                    add = c * racc * pre[PR_SDE * 64 + l];
                }
                const double v0 = (F0[b] + (src0 + u0 * add)) * pre[PR_RZ0 * 64 + l];
                const double v1 = (F1[b] + (src0 + u1 * add)) * pre[PR_RZ1 * 64 + l];
                const double v2 = (F2[b] + (src0 + u2 * add)) * pre[PR_RZ2 * 64 + l];
                const int pmv = perm[l];
                const int p0 = pmv & 3, p1 = (pmv >> 2) & 3, p2 = (pmv >> 4) & 3;
                double x0 = (p0 == 0) ? v0 : (p0 == 1) ? v1 : v2;
                double x1 = (p1 == 0) ? v0 : (p1 == 1) ? v1 : v2;
                double x2 = (p2 == 0) ? v0 : (p2 == 1) ? v1 : v2;
                x1 = x1 - pre[PR_L10 * 64 + l] * x0;
                x2 = x2 - pre[PR_L20 * 64 + l] * x0;
                x2 = x2 - pre[PR_L21 * 64 + l] * x1;
                x2 = x2 * pre[PR_RU22 * 64 + l];
                x1 = (x1 - pre[PR_U12 * 64 + l] * x2) * pre[PR_RU11 * 64 + l];
                x0 = (x0 - pre[PR_U01 * 64 + l] * x1 - pre[PR_U02 * 64 + l] * x2) * pre[PR_RU00 * 64 + l];
                if (lane == 0) { F0[b] = x0; F1[b] = x1; F2[b] = x2; }
                px0 = x0; px1 = x1; px2 = x2;
                if (nonres && b > 0) {
                    const double Tb = (u0 * x0 + u1 * x1 + u2 * x2) * pre[PR_SDE * 64 + l];
                    const int r = b + i - 1;                       // table column of bin b
                    const double* col = Al + (size_t)r * (r - 1) / 2 + (i - 1);
                    next_acc = accb_lds + col[b - 1] * Tb;
                    for (int bp = lane; bp < b - 1; bp += 64) acc[bp] += col[bp] * Tb;
                }
            }
        }
    }
    __syncthreads();
    // finalise (nuSIprop.hpp:328-336)
    for (int b = lane; b < N; b += 64) {
        const double dE = g.Emax[b] - g.Emin[b];
        const double f0 = F0[b] / dE, f1 = F1[b] / dE, f2 = F2[b] / dE;
        double* fo = flux + (size_t)p * 3 * N;
        double* fl = flux_fla + (size_t)p * 3 * N;
        fo[b] = f0;
        fo[N + b] = f1;
        fo[2 * N + b] = f2;
        for (int f = 0; f < 3; ++f) fl[f * N + b] = P.U2[3 * f + 0] * f0 + P.U2[3 * f + 1] * f1 + P.U2[3 * f + 2] * f2;
    }
}

hipError_t launch_cascade(const GridDev& g, const Point* pts, int npts, TablesDev t, double* flux, double* flux_fla,
                          hipStream_t s)
{
    const size_t lds = cascade_lds_bytes(g.N);
    hipLaunchKernelGGL(k_cascade, dim3(npts), dim3(64), lds, s, g, pts, t, flux, flux_fla);
    return hipGetLastError();
}

}  // namespace nusi
