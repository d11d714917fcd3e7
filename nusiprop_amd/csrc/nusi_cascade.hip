// nuSIprop MI355X -- Stage B: the implicit redshift cascade + finalisation
// (calculate_flux::evolve, nuSIprop.hpp:255-336).
//
//   k_cascade_bs<NJ, P, SPL, RT, CW, kNR>  the wavefront with its push on the fp64 matrix cores, block-synchronous
//                         roles; one point, two or up to 16 points sharing a table per workgroup, step passes on
//                         long grids (NUSI_CASCADE_AUTO / MFMA, every shape)
//   k_source_dsnb         the DSNB source terms it reads
//   k_cascade             the bit-exact scalar cascade, one wavefront per point, any N (NUSI_CASCADE_WAVEFRONT /
//                         REG / LDS).  (The per-stage kernels of rounds 1-3 -- k_cascade_wf, _reg, _ws, _wsp, _gb --
//                         are gone; DESIGN.md Appendix A keeps their measurements.)
#include <hip/hip_runtime.h>

#include <utility>

#include "nusi_internal.hpp"

namespace nusi {
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

// Per-point tables shared by the records of every (step, bin) (LDS; cascade_aux_init):
//   rdE[b] = 1 / dE_b                                                           [N]
//   pw[e]  = pow(E_e / E0 * (1 + z_i), -si) on table edge e = b + i (lower edge of bin b at
//            step i; the upper edge is e + 1), power-law source only            [T + 2]
// Along e the argument depends on b + i only (E_b (1 + z_i) = E_{b+i}, the index-shift
// identity), so 2 (Nz-1) N pow() calls per point become T + 1.  pw[e] is evaluated at one
// (b, i) of its edge; the other pairs' arguments differ from it by rounding only (<= 2 ulp).
constexpr int kAuxDoubles = 2;   // cascade_aux_doubles(N, T) = N + T + kAuxDoubles
NUSI_FN int cascade_aux_doubles(int N, int T) { return N + T + kAuxDoubles; }
__device__ inline void cascade_aux_init(const GridDev& g, const Point& P, double* rdE, double* pw, int tid, int nthr)
{
    const int N = g.N, Nz = g.Nz, T = g.T;
    for (int b = tid; b < N; b += nthr) rdE[b] = 1.0 / (g.Emax[b] - g.Emin[b]);
    if (P.source == 1)
        for (int e = tid + 1; e <= T + 1; e += nthr) {
            const int i = min(Nz - 1, max(1, e - N + 1)), b = e - i;
            const double E = (b < N) ? g.Emin[b] : g.Emax[N - 1];
            pw[e] = nm::pow(E / 1e14 * (1 + g.z[i]), -P.si);
        }
}

// the DSNB source, out of line: it is not the scans' source and inlined it would cost every
// record's caller registers
__device__ __attribute__((noinline)) double lum_out(const Point& P, double z, double sfr_z, double Em, double Ep)
{
    return lum(P, z, sfr_z, Em, Ep);
}

// flux-independent fields of bin b at step i (every PR_* field, the LU permutation in R[kPreFields]):
// Zdr, M = I + offdiag and its LU (nuSIprop.hpp:289-310) and the source term c_i Lum (:283).
// 1/dE_b and 1/Zdr are multiplied in (the reference divides; M's off-diagonals are ~1e-22 of
// the diagonal), the power-law source reads pw[]; the DSNB source is evaluated in full.

// 1/x to about an ulp: the hardware reciprocal estimate (v_rcp_f64) refined by two Newton steps.  The
// records' divisions use it (a correctly rounded fp64 division is a ~10-instruction dependent chain);
// the reference divides, so the fluxes move by rounding only (tests: FLUX_RTOL against the oracle).
NUSI_FN double rcp_nr(double x)
{
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

// The record of (step i, bin b) in two phases (k_cascade_bs runs them on different waves; cascade_record runs them
// back to back -- the same operations either way):
//   phase 1: 1/Zdr_k and the off-diagonals of M = I + offdiag (nuSIprop.hpp:289-300)
//   phase 2: the LU of M (GSL's partial pivoting, :309) from those
struct RecM { double rz0, rz1, rz2, m01, m02, m10, m12, m20, m21; };
NUSI_FN RecM record_phase1(const GridDev& g, const Point& P, const double* __restrict__ Gt,
                           const double* __restrict__ At, const double* rdE, int i, int b)
{
    const double c = g.step_c[i], s = g.step_s[i];
    const double u0 = P.u[0], u1 = P.u[1], u2 = P.u[2];
    const double rd = rdE[b];
    const double Gw = s * Gt[b + i - 1], Aw = s * At[b + i - 1];
    RecM m;
    m.rz0 = rcp_nr(1.0 + c * (Gw * u0 - Aw * (u0 * u0)) * rd);
    m.rz1 = rcp_nr(1.0 + c * (Gw * u1 - Aw * (u1 * u1)) * rd);
    m.rz2 = rcp_nr(1.0 + c * (Gw * u2 - Aw * (u2 * u2)) * rd);
    // M = I + offdiag, M[k][l] = Aw u_k u_l / dE_b / Zdr_k
    m.m01 = Aw * u0 * u1 * rd * m.rz0;
    m.m02 = Aw * u0 * u2 * rd * m.rz0;
    m.m10 = Aw * u1 * u0 * rd * m.rz1;
    m.m12 = Aw * u1 * u2 * rd * m.rz1;
    m.m20 = Aw * u2 * u0 * rd * m.rz2;
    m.m21 = Aw * u2 * u1 * rd * m.rz2;
    return m;
}
__device__ __attribute__((noinline)) void lu3_factor_out(double (&A)[3][3], int (&perm)[3]) { lu3_factor(A, perm); }
// the LU fields PR_L10 .. PR_RU22 and the permutation (R[kPreFields * stride])
template <bool kCallFree>
NUSI_FN void record_phase2(const RecM& m, double* R, int stride)
{
    // LU without row exchanges when partial pivoting would not exchange (M ~ I: always, in
    // practice); the same operations as lu3_factor on that path (a / 1.0 == a), else lu3_factor
    const double a11 = 1.0 - m.m10 * m.m01, a12 = m.m12 - m.m10 * m.m02;
    const double a21 = m.m21 - m.m20 * m.m01, a22 = 1.0 - m.m20 * m.m02;
    if (fabs(m.m10) <= 1.0 && fabs(m.m20) <= 1.0 && fabs(a21) <= fabs(a11) && a11 != 0.0) {
        const double ra11 = rcp_nr(a11);
        const double l21 = a21 * ra11;
        const double u22 = a22 - l21 * a12;
        R[PR_L10 * stride] = m.m10;
        R[PR_L20 * stride] = m.m20;
        R[PR_L21 * stride] = l21;
        R[PR_U01 * stride] = m.m01;
        R[PR_U02 * stride] = m.m02;
        R[PR_U12 * stride] = a12;
        R[PR_RU00 * stride] = 1.0;
        R[PR_RU11 * stride] = ra11;
        R[PR_RU22 * stride] = rcp_nr(u22);
        R[kPreFields * stride] = (double)(0 | (1 << 2) | (2 << 4));
    } else {
        double M[3][3] = {{1.0, m.m01, m.m02}, {m.m10, 1.0, m.m12}, {m.m20, m.m21, 1.0}};
        int pm[3];
        if (kCallFree) lu3_factor(M, pm);
        else lu3_factor_out(M, pm);
        R[PR_L10 * stride] = M[1][0];
        R[PR_L20 * stride] = M[2][0];
        R[PR_L21 * stride] = M[2][1];
        R[PR_U01 * stride] = M[0][1];
        R[PR_U02 * stride] = M[0][2];
        R[PR_U12 * stride] = M[1][2];
        R[PR_RU00 * stride] = 1.0 / M[0][0];
        R[PR_RU11 * stride] = 1.0 / M[1][1];
        R[PR_RU22 * stride] = 1.0 / M[2][2];
        R[kPreFields * stride] = (double)(pm[0] | (pm[1] << 2) | (pm[2] << 4));
    }
}

// kCallFree: the caller's points all use the power-law source and the pivoting LU is inlined, so
// the record code makes no calls (a call inside the wavefront kernel's stage loop makes the
// compiler drain every outstanding alpha prefetch, vmcnt(0), after it)
template <bool kCallFree>
NUSI_FN void cascade_record(const GridDev& g, const Point& P, const double* __restrict__ Gt,
                            const double* __restrict__ At, const double* rdE, const double* pw, int i, int b,
                            double* R, int stride)
{
    const double c = g.step_c[i], s = g.step_s[i];
    const double rd = rdE[b];
    const RecM m = record_phase1(g, P, Gt, At, rdE, i, b);
    R[PR_RZ0 * stride] = m.rz0;
    R[PR_RZ1 * stride] = m.rz1;
    R[PR_RZ2 * stride] = m.rz2;
    record_phase2<kCallFree>(m, R, stride);
    double src;
    if (kCallFree || P.source == 1)   // nuSIprop.hpp:656
        src = P.norm_total / 3.0 * g.sfr[i] * (g.Emax[b] * pw[b + i + 1] - g.Emin[b] * pw[b + i]) * rcp_nr(1 - P.si);
    else
        src = lum_out(P, g.z[i], g.sfr[i], g.Emin[b], g.Emax[b]);
    R[PR_SRC * stride] = c * src;
    R[PR_SDE * stride] = P.non_resonant ? s * rd : (g.Emax[b] - g.Emin[b]);
}

// the 3x3 solve of one bin (nuSIprop.hpp:289-313) from its fields and the coupling `add` to the
// bins above; x = F[:, b] of this step
NUSI_FN void cascade_solve(double f0, double f1, double f2, double add, double src0, double u0, double u1, double u2,
                           double rz0, double rz1, double rz2, int pmb, double l10, double l20, double l21, double u01,
                           double u02, double u12, double ru00, double ru11, double ru22, double& x0, double& x1,
                           double& x2)
{
    const double v0 = (f0 + (src0 + u0 * add)) * rz0;
    const double v1 = (f1 + (src0 + u1 * add)) * rz1;
    const double v2 = (f2 + (src0 + u2 * add)) * rz2;
    const int p0 = pmb & 3, p1 = (pmb >> 2) & 3, p2 = (pmb >> 4) & 3;
    x0 = (p0 == 0) ? v0 : (p0 == 1) ? v1 : v2;
    x1 = (p1 == 0) ? v0 : (p1 == 1) ? v1 : v2;
    x2 = (p2 == 0) ? v0 : (p2 == 1) ? v1 : v2;
    x1 = x1 - l10 * x0;
    x2 = x2 - l20 * x0;
    x2 = x2 - l21 * x1;
    x2 = x2 * ru22;
    x1 = (x1 - u12 * x2) * ru11;
    x0 = (x0 - u01 * x1 - u02 * x2) * ru00;
}

// cascade_solve where every lane's LU kept the rows in place (the permutation 0 | 1 << 2 | 2 << 4, and then ru00 =
// 1 / 1.0 = 1.0: the product by it is exact and dropped) -- the same bits as cascade_solve
constexpr int kIdPerm = 0 | (1 << 2) | (2 << 4);
NUSI_FN void cascade_solve_id(double f0, double f1, double f2, double add, double src0, double u0, double u1, double u2,
                              double rz0, double rz1, double rz2, double l10, double l20, double l21, double u01,
                              double u02, double u12, double ru11, double ru22, double& x0, double& x1, double& x2)
{
    x0 = (f0 + (src0 + u0 * add)) * rz0;
    x1 = (f1 + (src0 + u1 * add)) * rz1;
    x2 = (f2 + (src0 + u2 * add)) * rz2;
    x1 = x1 - l10 * x0;
    x2 = x2 - l20 * x0;
    x2 = x2 - l21 * x1;
    x2 = x2 * ru22;
    x1 = (x1 - u12 * x2) * ru11;
    x0 = x0 - u01 * x1 - u02 * x2;
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
    const double* __restrict__ Gt = t.G + (size_t)P.tslot * T;
    const double* __restrict__ At = t.At + (size_t)P.tslot * T;
    const double* __restrict__ Al = t.A + (size_t)P.tslot * g.PT;
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

typedef double nusi_f64x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
#ifndef NUSI_BS_SRC_AHEAD   // A/B: 0 = the DSNB sources loaded and stored within one phase B
#define NUSI_BS_SRC_AHEAD 1
#endif
constexpr bool kSrcAhead = NUSI_BS_SRC_AHEAD != 0;
// Helpers of the MFMA cascade k_cascade_bs (below): the power-law source, the DSNB source table, the chain's
// hand-off between redshift steps and the resonant-only running sum.
// ---------------------------------------------------------------------------

// the power-law source term c_i Lum of bin b at step i (nuSIprop.hpp:283, :656), the expression
// cascade_record stores in PR_SRC
NUSI_FN double powerlaw_src(const GridDev& g, const Point& P, const double* pw, int i, int b)
{
    return g.step_c[i] * (P.norm_total / 3.0 * g.sfr[i] * (g.Emax[b] * pw[b + i + 1] - g.Emin[b] * pw[b + i]) * rcp_nr(1 - P.si));
}
// the same with the point's factors hoisted: a3 = norm_total / 3.0, rs = rcp_nr(1 - si) (the same operations,
// once per point instead of once per record)
struct SrcFactors { double a3, rs; };
NUSI_FN SrcFactors src_factors(const Point& P) { return SrcFactors{P.norm_total / 3.0, rcp_nr(1 - P.si)}; }
NUSI_FN double powerlaw_src_h(const GridDev& g, const SrcFactors& f, const double* pw, int i, int b)
{
    return g.step_c[i] * (f.a3 * g.sfr[i] * (g.Emax[b] * pw[b + i + 1] - g.Emin[b] * pw[b + i]) * f.rs);
}

// The DSNB source term c_i Lum(z_i, Emin_b, Emax_b) (nuSIprop.hpp:283, :659-662) of every (step slot J, bin b)
// of a point, computed before the MFMA cascade (it costs two Li2 / Li3 pairs per record, far more than a
// wavefront stage) in the diagonal layout src[(b - J + Nz - 2) (Nz - 1) + J]: the lanes of one stage (b - J
// constant) read consecutive doubles.  The expression is cascade_record's, so the records are the same bits.
NUSI_FN size_t src_index(int Nz, int J, int b) { return (size_t)(b - J + Nz - 2) * (Nz - 1) + J; }
__global__ __launch_bounds__(256) void k_source_dsnb(GridDev g, const Point* __restrict__ pts, double* __restrict__ src)
{
    const int p = blockIdx.y, N = g.N, Nz = g.Nz, nst = Nz - 1;
    const Point& P = pts[p];
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (P.source != NUSI_SOURCE_DSNB || e >= nst * N) return;
    const int J = e / N, b = e - J * N, i = Nz - 1 - J;
    src[(size_t)p * g.T * nst + src_index(Nz, J, b)] = g.step_c[i] * lum(P, g.z[i], g.sfr[i], g.Emin[b], g.Emax[b]);
}
size_t cascade_src_doubles(const GridDev& g) { return (size_t)g.T * (g.Nz - 1); }
hipError_t launch_source_dsnb(const GridDev& g, const Point* pts, int npts, double* src, hipStream_t s)
{
    const int ne = (g.Nz - 1) * g.N;
    hipLaunchKernelGGL(k_source_dsnb, dim3((ne + 255) / 256, npts), dim3(256), 0, s, g, pts, src);
    return hipGetLastError();
}

// The chain's hand-off between steps: step slot j solves bin b at stage sg, right after slot j-1 solved the same
// bin at stage sg-1 (nuSIprop.hpp:257-315: step i starts from step i+1's F[:, b]).  wave_shr1 moves each lane's
// value to the next lane (DPP wave_shr:1, a register move across the wave); lane 0 receives `fill`.  It must run
// with every lane of the wave active (a disabled source lane would leave its neighbour's old value).
__device__ __forceinline__ double wave_shr1(double v, double fill)
{
    const long long x = __double_as_longlong(v), f = __double_as_longlong(fill);
    const int lo = __builtin_amdgcn_update_dpp((int)f, (int)x, 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(f >> 32), (int)(x >> 32), 0x138, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// The resonant-only chain (nuSIprop.hpp:261-278, 285-287): the running sum of the bins above, from the
// lane's own solve of bin b+1 (x = F[:, b+1] of this step).  sde = dE_b.
NUSI_FN double resonant_add(double& racc, double u0, double u1, double u2, double px0, double px1, double px2,
                            double sj, double sd, double dEb1, double sde, double cj, bool top)
{
    if (!top) racc += (u0 * px0 + u1 * px1 + u2 * px2) * (sj * sd) / dEb1 / sde;
    return cj * racc * sde;
}


// Diagnostic build only (-DNUSI_WS_TRACE, scripts/build_variant.sh): s_memtime stamps of workgroup 0's waves
// at the start of each stage's work and at its barrier (read the shares, not the length: the stamps cost
// cycles).  nusi_debug_ws_trace() copies them out.  Compiled out of the product.
#ifdef NUSI_WS_TRACE
constexpr int kTrWaves = 16, kTrStages = 512, kTrBlocks = 8192;
__device__ unsigned long long g_ws_trace[kTrWaves * kTrStages * 4];   // [wave][stage][start, barrier, chain: loaded, solved]
__device__ unsigned int g_ws_hwid[kTrBlocks * kTrWaves];   // HW_ID (SE, CU, SIMD, wave slot) of every wave
#define NUSI_WS_HWID()                                                                                             \
    do {                                                                                                           \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < kTrBlocks)                                                     \
            g_ws_hwid[blockIdx.x * kTrWaves + (threadIdx.x >> 6)] = __builtin_amdgcn_s_getreg(4 | (31 << 11));     \
    } while (0)
// k_cascade_bs: [wave][block][phase A start, its barrier, phase B start, its barrier], no waits
#define NUSI_BS_STAMP(blk, which)                                                                                  \
    do {                                                                                                           \
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (blk) < kTrStages)                                       \
            g_ws_trace[((threadIdx.x >> 6) * kTrStages + (blk)) * 4 + (which)] = __builtin_amdgcn_s_memtime();      \
    } while (0)
// k_cascade_bs chain wave 0, phase B, in wave slot 15: [block][stage 4q+1 loaded, solved, 4q+2 loaded, solved]
// (the "loaded" stamps wait for the stage's LDS loads first)
#define NUSI_BS_CSTAMP(blk, which)                                                                                 \
    do {                                                                                                           \
        if (((which) & 1) == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                \
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (blk) < kTrStages)                                       \
            g_ws_trace[(15 * kTrStages + (blk)) * 4 + (which)] = __builtin_amdgcn_s_memtime();                      \
    } while (0)
#else
#define NUSI_BS_STAMP(blk, which) do { } while (0)
#define NUSI_BS_CSTAMP(blk, which) do { } while (0)
#define NUSI_WS_HWID() do { } while (0)
#endif

// ---------------------------------------------------------------------------
// k_cascade_bs: the MFMA cascade with block-synchronous roles (round 4).  The wavefront (stage sg: step slot j
// solves bin N-1-sg+j; every active step reads the same table column r = T-1-sg, the index-shift identity), its
// push as rank-4 blocks on v_mfma_f64_16x16x4f64 (ACC[rows, steps] += alpha[rows, 4 columns] . T[4 columns, steps],
// the transfer-matrix x flux-batch GEMM whose batch is the steps in flight and, for points sharing a table, the
// points), the records and the solves.  The per-stage kernels of rounds 2-3 synchronised every wave of
// the workgroup once per STAGE, so a stage cost a barrier, an LDS round trip of the chain's records and its
// dependent solve (~2 000 cycles against a ~700-cycle floor).  The data dependencies only
// need a meeting point twice per BLOCK of four stages:
//   * block q's push (columns of stages 4q-4 .. 4q-1) needs the chain's T_j of those stages;
//   * the chain's stages 4q+1 .. 4q+4 need the rows block q publishes; stage 4q needs block q-1's.
// So every block runs in two phases between two barriers:
//   phase A: the waves holding the four rows block q publishes push block q into those tiles and publish
//            them (AX); the chain solves stage 4q (block q-1's rows);
//   phase B: the chain solves stages 4q+1 .. 4q+3 back to back (block q's rows, its own four diagonal
//            columns as before); the other push tiles add block q (their rows are published later).
// The record wave forms block q + 1's records over both phases (a third in A, where the chain solves one stage,
// the rest in B) and stages the DSNB sources; the chain forms the power-law sources itself.
// The chain is CW waves of PPW = P / CW whole points: lane (point p, j) runs step slot j (SPL = 1); slot j takes
// F[:, b] from slot j-1's solve of the previous stage by a DPP wave shift, or (first step of a pass > 0) the previous
// pass' last step through a global FIFO prefetched a block ahead.  Each stage's loads are issued a stage ahead of
// its solve, and the last pass' finalise (three divisions and six stores per bin) runs on the record wave.
// The A operands of block q + 2 are loaded while block q is pushed (two register buffers, the block loop
// unrolled by two), so the publishing tiles never wait for HBM.
// Columns: the NC = NJ P right-hand sides (point p, step j) at c = j P + p; a push tile is 16 columns (one
// step of 16 points, or 16 steps of one point), so one template <NJ, P, SPL, RT, CW> covers
//   <48, 1, 1, 4, 1>  one point per workgroup (C4)
//   <48, 2, 1, 2, 2>  two points sharing a table, a chain wave per point
//   <6, 16, 1, 2, 2>  the gamma batch, up to 16 points of a table, 8 per chain wave, step passes of 6
//   <16, 1, 1, 8, 1>  step passes of 16 on long grids (C3)
// (kNR: every point of the launch non-resonant, the resonant-only terms compiled out).  The MFMA sums each
// element's four columns in its own order whichever column it is, so a point's fluxes depend on its grouping only
// through the step passes (to rounding).  Waves: push waves of 16 RT rows, the chain waves, the record wave.
// ---------------------------------------------------------------------------
#ifndef NUSI_BS_SIMDMAP   // the chain and record waves beside the least-busy push waves (wave w runs on SIMD f(w % 4),
#define NUSI_BS_SIMDMAP 1    // HW_ID in the trace build): C5 cascade 3.19 -> 2.82 ms, C3 23.4 -> 21.4, C4 equal
#endif                       // (profiles/r4/ab/r4u, r4v); 0 = the push waves' rows in wave order
#ifndef NUSI_BS_LONG32   // A/B: step passes of 32 on long grids (<32, 1, 1, 6, 1>: 14 push waves of 96 rows)
#define NUSI_BS_LONG32 0
#endif
#ifndef NUSI_BS_PRIO   // the chain and record waves at raised issue priority (s_setprio 3; the push waves 0): C5
#define NUSI_BS_PRIO 1    // cascade 3.51 -> 3.25 ms, C3 29.1 -> 24.8, C4 0.555 -> 0.528 (profiles/r4/ab/r4n, r4o); 0 = off.
#endif                    // Sleeping the push waves at phase B's start (to let the chain's loads first) measured no gain
#ifndef NUSI_BS_PIPE   // A/B: k_cascade_bs's chain issues stage d + 1's loads before stage d's solve (two stages'
#define NUSI_BS_PIPE 0  // operands live: spills at the 128-VGPR budget)
#endif
template <int NJ, int P, int SPL, int RT, int CW>
struct BsCfg {
    static constexpr int LPP = NJ / SPL;   // chain lanes per point
    static constexpr int PPW = P / CW;     // points per chain wave
    static constexpr int NC = NJ * P;      // right-hand columns
    static constexpr int NB = NC / 16;     // push column tiles
    static_assert(SPL == 1 && P % CW == 0 && NC % 16 == 0 && LPP * PPW <= 64, "a step slot per chain lane, whole points per chain wave, whole column tiles");
};

// record fields of the block-synchronous kernel: PR_* without PR_SRC (the sources have a block of their own), so
// fields >= PR_L10 sit one lower -- record_phase2 writes them through a base pointer one field stride lower
enum { BR_RZ0, BR_RZ1, BR_RZ2, BR_L10, BR_L20, BR_L21, BR_U01, BR_U02, BR_U12, BR_RU00, BR_RU11, BR_RU22, BR_SDE, BR_PERM,
       kBsFields };
static_assert(PR_L10 - 1 == BR_L10 && PR_RU22 - 1 == BR_RU22 && kPreFields - 1 == BR_PERM, "record_phase2's fields, shifted");

template <int NJ, int P, int SPL, int RT, int CW, bool kNR>   // kNR: every point of the launch non-resonant
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 4)))
void k_cascade_bs(GridDev g, const Point* __restrict__ pts, const int* __restrict__ gidx, const int2* __restrict__ grp,
                  TablesDev t, double* __restrict__ fh, double* __restrict__ flux, double* __restrict__ flux_fla)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    using Cfg = BsCfg<NJ, P, SPL, RT, CW>;
    // the power-law sources: formed on the record wave (into srcb, a block ahead) where that is one round of 64 (one
    // point, 16 steps: C3, cascade 24.8 -> 23.7 ms), else in the chain (the record wave's loop of 6 rounds for the
    // gamma batch cost C5 3.25 -> 4.16 ms; at 48 steps its records already fill both phases, C4)
    constexpr bool kSrcRec = 4 * NJ * P <= 64;
    constexpr int LPP = Cfg::LPP, PPW = Cfg::PPW, NC = Cfg::NC, NB = Cfg::NB, NF = kBsFields, S4 = 4 * NJ, NQ = 12 * P;
    const int N = g.N, Nz = g.Nz, T = g.T, nst = Nz - 1;
    // the wave index through readfirstlane: wave-uniform in an SGPR, so every role test and per-wave row base is scalar
    const int tid = threadIdx.x, nthr = blockDim.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), nw = nthr >> 6;
#if NUSI_BS_SIMDMAP
    // the record wave before the chain waves, and the push row blocks dealt so that the push waves sharing a SIMD with
    // a chain wave (wave w on SIMD w % 4) hold the top rows, which the wavefront consumes first (fewest MFMAs)
    const int recw = nw - 1 - CW, chw = nw - CW;
    const bool is_chain = wave >= chw, is_rec = wave == recw;
#else
    const int chw = nw - 1 - CW, recw = nw - 1;   // push waves 0 .. chw-1, the CW chain waves, the record wave
    const bool is_chain = wave >= chw && wave < recw, is_rec = wave == recw;
#endif
    NUSI_WS_HWID();
    const int2 gr = grp ? grp[blockIdx.x] : make_int2((int)blockIdx.x, 1);
    const int R = gr.y;                                   // points of this workgroup (<= P), one table
    auto pidx = [&](int p) { return gidx ? gidx[gr.x + p] : gr.x + p; };   // (gidx == nullptr: point blockIdx.x)
    const Point& P0 = pts[pidx(0)];
    double* rec = lds;                       // [2][NF][4][NJ]  records of block q in slot q & 1
    double* srcb = rec + 2 * NF * S4;        // [2][4][NJ][P]   block q's DSNB sources c_i Lum (stage, step, point)
    double* Tp = srcb + 8 * NC;              // [8][NC]         T_j of each column by stage
    double* AX = Tp + 8 * NC;                // [2][4][NC]      rows published by block q (parity q & 1)
    double* fqb = AX + 8 * NC;               // [2][4][3][P]    the previous pass' last step, F[:, N-1-sg], block q
    double* fin = fqb + 2 * NQ;              // [2][4][3][P]    the last pass' output F[:, b] of block q's stages (to finalise)
    double* pinf = fin + 2 * NQ;             // [13][P]         per point: a3, rs, power law (1) / DSNB (0), index, U2[9]
    double* rdE = pinf + 13 * P;             // [N]
    double* pw = rdE + N;                    // [P][T + 2]      each power-law point's pw on table edge e
    double* sGt = pw + (size_t)P * (T + 2);
    double* sAt = sGt + T;
    double* sdg = sAt + T;                   // [4][T]: alpha(n, n+k), k = 1..4 (0 past the table)
    double* sEmin = sdg + 4 * T;
    double* sEmax = sEmin + N;
    double* sgz = sEmax + N;                 // z, step_c, step_s, sfr [Nz each]
    GridDev gl = g;
    gl.Emin = sEmin;
    gl.Emax = sEmax;
    gl.z = sgz;
    gl.step_c = sgz + Nz;
    gl.step_s = sgz + 2 * Nz;
    gl.sfr = sgz + 3 * Nz;
    const double* __restrict__ Al = t.A + (size_t)P0.tslot * g.PT;
    {
        const double* __restrict__ Gt = t.G + (size_t)P0.tslot * T;
        const double* __restrict__ At = t.At + (size_t)P0.tslot * T;
        for (int n = tid; n < T; n += nthr) {
            sGt[n] = Gt[n];
            sAt[n] = At[n];
#pragma unroll
            for (int k = 1; k <= 4; ++k) sdg[(k - 1) * T + n] = (n + k < T) ? Al[(size_t)(n + k) * (n + k - 1) / 2 + n] : 0.0;
        }
        for (int b = tid; b < N; b += nthr) {
            sEmin[b] = g.Emin[b];
            sEmax[b] = g.Emax[b];
            rdE[b] = 1.0 / (g.Emax[b] - g.Emin[b]);   // cascade_aux_init's expression
        }
        for (int i = tid; i < Nz; i += nthr) {
            sgz[i] = g.z[i];
            sgz[Nz + i] = g.step_c[i];
            sgz[2 * Nz + i] = g.step_s[i];
            sgz[3 * Nz + i] = g.sfr[i];
        }
        for (int p = tid; p < P; p += nthr) {   // the points' source factors (src_factors), kind and index
            const int pid = p < R ? pidx(p) : 0;
            const SrcFactors f = src_factors(pts[pid]);
            pinf[p] = f.a3;
            pinf[P + p] = f.rs;
            pinf[2 * P + p] = p < R && pts[pid].source == NUSI_SOURCE_POWER_LAW ? 1.0 : 0.0;
            pinf[3 * P + p] = (double)pid;
#pragma unroll
            for (int f = 0; f < 9; ++f) pinf[(4 + f) * P + p] = pts[pid].U2[f];   // the finalise's, off the chain's global path
        }
        for (int q = tid; q < P * (T + 1); q += nthr) {   // cascade_aux_init's pw[e] of every power-law point
            const int p = q / (T + 1), e = 1 + q - p * (T + 1);
            if (p >= R) continue;
            const Point& Q = pts[pidx(p)];
            if (Q.source != NUSI_SOURCE_POWER_LAW) continue;
            const int i = min(Nz - 1, max(1, e - N + 1)), b = e - i;
            const double E = (b < N) ? g.Emin[b] : g.Emax[N - 1];
            pw[(size_t)p * (T + 2) + e] = nm::pow(E / 1e14 * (1 + g.z[i]), -Q.si);
        }
    }
    const bool nonres = kNR || P0.non_resonant;   // the points of a workgroup share a table, hence the flags
    const int npass = (nst + NJ - 1) / NJ;
    double* const fhw = fh + (size_t)blockIdx.x * 3 * N * P;   // this workgroup's F FIFO [3][N][P] (passes > 1)
    int jb = 0, njp = 0, Ts = 0, c0 = 0, nblk = 0;
    auto pass_geom = [&](int pass) {
        jb = pass * NJ;
        njp = nst - jb < NJ ? nst - jb : NJ;   // steps of this pass
        Ts = N - 1 + njp;                      // its stages
        c0 = T - 1 - jb;                       // the table column of its stage 0
        nblk = (Ts + 3) / 4;
    };
    if (is_chain) {
        // ---- chain wave cw: lane (cp, cjp) solves step slot j = cjp of point cp (PPW points per wave, so a point's
        // steps never cross waves).  A stage is split into its loads (records, source operands, published row,
        // diagonal alphas: none depends on the previous stage's solve) and its solve, and the loads of stage d + 1
        // are issued before the solve of stage d, so one LDS latency per stage is hidden behind the dependent
        // solve.  The power-law sources are formed here (powerlaw_src_h), the DSNB ones read from srcb; the
        // finalise of the last pass goes to the record wave through `fin`
#if NUSI_BS_PRIO
        __builtin_amdgcn_s_setprio(3);   // the chain's instructions (and LDS requests) before the push waves'
#endif
        const int cw = wave - chw;
        const int cp = cw * PPW + lane / LPP, cjp = lane - LPP * (lane / LPP);
        const bool clane = lane < PPW * LPP && cp < R;
        const double u0 = P0.u[0], u1 = P0.u[1], u2 = P0.u[2];
        const int cpc = cp < P ? cp : P - 1;
        const double* const cpw = pw + (size_t)cpc * (T + 2);
        struct StageIn {
            double rz0, rz1, rz2, l10, l20, l21, u01, u02, u12, ru00, ru11, ru22, sde, src, cj, ab, sd[4], fq0, fq1, fq2;
            double ss, dEb1;   // the resonant-only running sum's step_s and dE of the bin above
            int pmb;
        };
#pragma unroll 1
        for (int pass = 0; pass < npass; ++pass) {
            pass_geom(pass);
            const bool last_pass = pass == npass - 1;
            __syncthreads();   // the previous pass is done with Tp, AX and the records (pass 0: the prologue's LDS)
            for (int q = lane; q < 16 * NC; q += 64) Tp[q] = 0.0;   // Tp and AX
            const bool cpl = pinf[2 * P + cpc] != 0.0;
            const SrcFactors csf{pinf[cpc], pinf[P + cpc]};
            __syncthreads();
            double px0 = 0.0, px1 = 0.0, px2 = 0.0, racc = 0.0, Th[4] = {0.0, 0.0, 0.0, 0.0};
            const int j = cjp, i = Nz - 1 - jb - j;
            const int ic = i < 1 ? 1 : i;   // (lanes past the pass' steps read in range and are masked)
            // stage sg = 4 q + d of the pass: its loads
            auto load = [&](int q, int d) {
                const int sg = 4 * q + d, r = c0 - sg;
                const int b = N - 1 - sg + j, bc = b < 0 ? 0 : (b > N - 1 ? N - 1 : b);
                const int rc = r < 0 ? 0 : r;
                const double* Rc = rec + (size_t)(q & 1) * NF * S4 + d * NJ + j;
                StageIn in;
                in.rz0 = Rc[BR_RZ0 * S4]; in.rz1 = Rc[BR_RZ1 * S4]; in.rz2 = Rc[BR_RZ2 * S4];
                in.pmb = (int)Rc[BR_PERM * S4];
                in.l10 = Rc[BR_L10 * S4]; in.l20 = Rc[BR_L20 * S4]; in.l21 = Rc[BR_L21 * S4];
                in.u01 = Rc[BR_U01 * S4]; in.u02 = Rc[BR_U02 * S4]; in.u12 = Rc[BR_U12 * S4];
                in.ru00 = Rc[BR_RU00 * S4]; in.ru11 = Rc[BR_RU11 * S4]; in.ru22 = Rc[BR_RU22 * S4];
                in.sde = Rc[BR_SDE * S4];
                const double sdn = srcb[(q & 1) * 4 * NC + d * NC + j * P + cpc];
                if (kSrcRec) {   // the record wave formed every source
                    in.src = sdn;
                } else {         // both, selected branch-free (a branch here made the compiler wait for every LDS load)
                    const double spw = powerlaw_src_h(gl, csf, cpw, ic, bc);
                    in.src = cpl ? spw : sdn;
                }
                in.cj = gl.step_c[ic];
                const int qq = (sg - 1) >> 2;   // block whose publication serves stage sg
                in.ab = AX[((qq & 1) * 4 + (sg - 1 - 4 * qq)) * NC + j * P + cpc];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) in.sd[kk] = sdg[kk * T + rc];
                const double* fq = fqb + (q & 1) * NQ + d * 3 * P + cpc;
                in.fq0 = fq[0]; in.fq1 = fq[P]; in.fq2 = fq[2 * P];
                if (!nonres) {
                    in.ss = gl.step_s[ic];
                    in.dEb1 = (bc + 1 < N) ? sEmax[bc + 1] - sEmin[bc + 1] : 1.0;
                } else {
                    in.ss = in.dEb1 = 0.0;
                }
                return in;
            };
            // ... and its solve
            auto solve = [&](int q, int d, const StageIn& in) {
                const int sg = 4 * q + d;
                const int b = N - 1 - sg + j;
                const int nu = (d == 0) ? 4 : d;   // columns r+1 .. r+nu not yet pushed
                double f0 = wave_shr1(px0, 0.0), f1 = wave_shr1(px1, 0.0), f2 = wave_shr1(px2, 0.0);   // every lane active
                if (cjp == 0) {   // the first step: the previous pass' last step (fqb, staged by the record wave), or 0
                    f0 = in.fq0;
                    f1 = in.fq1;
                    f2 = in.fq2;
                }
                double Tn = 0.0;
                if (clane && j < njp && b >= 0 && b < N) {
                    double add;
                    if (nonres) {
                        double sa = in.ab;
#pragma unroll
                        for (int kk = 4; kk >= 1; --kk)
                            if (kk <= nu) sa = fma(in.sd[kk - 1], Th[kk - 1], sa);
                        add = in.cj * sa;
                    } else {
                        add = resonant_add(racc, u0, u1, u2, px0, px1, px2, in.ss, in.sd[0], in.dEb1, in.sde, in.cj,
                                           b == N - 1);
                    }
                    double x0, x1, x2;
                    if (__all(in.pmb == kIdPerm))   // (every active lane: no row exchange -- always, in practice)
                        cascade_solve_id(f0, f1, f2, add, in.src, u0, u1, u2, in.rz0, in.rz1, in.rz2, in.l10, in.l20,
                                         in.l21, in.u01, in.u02, in.u12, in.ru11, in.ru22, x0, x1, x2);
                    else
                        cascade_solve(f0, f1, f2, add, in.src, u0, u1, u2, in.rz0, in.rz1, in.rz2, in.pmb, in.l10,
                                      in.l20, in.l21, in.u01, in.u02, in.u12, in.ru00, in.ru11, in.ru22, x0, x1, x2);
                    if (j == njp - 1) {   // the pass's last step: the output (the record wave finalises it), or the next pass' input
                        if (last_pass) {
                            double* fo = fin + (((q & 1) * 4 + d) * 3) * P + cp;
                            fo[0] = x0;
                            fo[P] = x1;
                            fo[2 * P] = x2;
                        } else {
                            fhw[((size_t)0 * N + b) * P + cp] = x0;
                            fhw[((size_t)1 * N + b) * P + cp] = x1;
                            fhw[((size_t)2 * N + b) * P + cp] = x2;
                        }
                    }
                    px0 = x0; px1 = x1; px2 = x2;
                    if (nonres && b > 0) Tn = (u0 * x0 + u1 * x1 + u2 * x2) * in.sde;
                }
                Th[3] = Th[2]; Th[2] = Th[1]; Th[1] = Th[0]; Th[0] = Tn;
                if (clane && j < njp) Tp[(sg & 7) * NC + j * P + cp] = Tn;
            };
#pragma unroll 1
            for (int q = 0; q < nblk; ++q) {
                NUSI_BS_STAMP(pass * nblk + q, 0);
                if (4 * q < Ts) solve(q, 0, load(q, 0));           // phase A
                NUSI_BS_STAMP(pass * nblk + q, 1);
                __syncthreads();
                NUSI_BS_STAMP(pass * nblk + q, 2);
#if NUSI_BS_PIPE
                {                                                    // phase B: stage d + 1 loaded before d solves
                    StageIn in1 = load(q, 1), in2 = load(q, 2);
                    if (4 * q + 1 < Ts) solve(q, 1, in1);
                    in1 = load(q, 3);
                    if (4 * q + 2 < Ts) solve(q, 2, in2);
                    if (4 * q + 3 < Ts) solve(q, 3, in1);
                }
#else
#pragma unroll
                for (int d = 1; d < 4; ++d)                          // phase B
                    if (4 * q + d < Ts) {
                        const StageIn in = load(q, d);
                        if (d < 3 && cw == 0) NUSI_BS_CSTAMP(pass * nblk + q, 2 * (d - 1));
                        solve(q, d, in);
                        if (d < 3 && cw == 0) NUSI_BS_CSTAMP(pass * nblk + q, 2 * (d - 1) + 1);
                    }
#endif
                NUSI_BS_STAMP(pass * nblk + q, 3);
                __syncthreads();
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the FIFO stores land before the next pass reads them
        }
    } else if (is_rec) {
#if NUSI_BS_PRIO
        __builtin_amdgcn_s_setprio(3);
#endif
        // ---- records and DSNB sources: block 0 (and the FIFO of blocks 0, 1) before the blocks; in block q the
        // records of block q + 1 (block q + 1's slot was last read in block q - 1): one round of 64 lanes goes wholly
        // into phase B, where the chain solves three stages (C5 / C3: phase A then waits on the chain alone); of
        // three rounds (48 steps) the first goes into phase A; the DSNB sources into phase B.  The FIFO values of
        // block q + 2 are loaded in phase A of block q and stored in phase A of block q + 1
        constexpr int kRecRounds = (S4 + 63) / 64, kRecA = kRecRounds <= 1 ? 0 : (kRecRounds + 2) / 3;
        constexpr int kRecSplit = 64 * kRecA < S4 ? 64 * kRecA : S4;
        auto records = [&](int qb, int e0, int e1) {
            for (int e = e0 + lane; e < e1; e += 64) {
                const int sb = e / NJ, jj = e - NJ * (e / NJ), s2 = 4 * qb + sb;
                const int b = N - 1 - s2 + jj, i = Nz - 1 - jb - jj;
                if (jj < njp && s2 < Ts && b >= 0 && b < N) {
                    double* Rw = rec + (size_t)(qb & 1) * NF * S4 + e;
                    const RecM m = record_phase1(gl, P0, sGt, sAt, rdE, i, b);
                    Rw[BR_RZ0 * S4] = m.rz0;
                    Rw[BR_RZ1 * S4] = m.rz1;
                    Rw[BR_RZ2 * S4] = m.rz2;
                    Rw[BR_SDE * S4] = nonres ? gl.step_s[i] * rdE[b] : (gl.Emax[b] - gl.Emin[b]);
                    record_phase2<true>(m, Rw - S4, S4);   // (PR_L10 .. PR_RU22, the permutation: BR_* = PR_* - 1)
                }
            }
        };
        bool any_dsnb = false;   // (set after the first barrier: the prologue writes pinf)
        auto sources = [&](int qb) {   // the DSNB points' (k_source_dsnb's table); with kSrcRec the power-law ones too
            if (!kSrcRec && !any_dsnb) return;
            for (int e = lane; e < S4 * P; e += 64) {
                const int p = e % P, sj = e / P, sb = sj / NJ, jj = sj - NJ * sb, s2 = 4 * qb + sb;
                const int b = N - 1 - s2 + jj, i = Nz - 1 - jb - jj;
                if (p < R && jj < njp && s2 < Ts && b >= 0 && b < N) {
                    if (pinf[2 * P + p] == 0.0)
                        srcb[(qb & 1) * 4 * NC + e] = t.Src[(size_t)pinf[3 * P + p] * T * nst + src_index(Nz, jb + jj, b)];
                    else if (kSrcRec)
                        srcb[(qb & 1) * 4 * NC + e] =
                            powerlaw_src_h(gl, SrcFactors{pinf[p], pinf[P + p]}, pw + (size_t)p * (T + 2), i, b);
                }
            }
        };
        // The DSNB sources of block qb from k_source_dsnb's table a block ahead (src_load into registers in phase B of
        // block qb - 2, src_store into srcb in phase B of block qb - 1): the table's latency off the record wave's path
        // (sources() loaded and stored them within one phase B: C2a's cascade 0.295 against C2b's 0.176 ms).  The same
        // values in the same places.
        constexpr bool kAhead = kSrcAhead && P == 1 && RT == 4;   // (one point, one pass shape: the others' registers)
        constexpr int SQL = (S4 * P + 63) / 64;
        auto src_valid = [&](int qb, int e, int& p, int& b, int& i) {
            p = e % P;
            const int sj = e / P, sb = sj / NJ, jj = sj - NJ * sb, s2 = 4 * qb + sb;
            b = N - 1 - s2 + jj;
            i = Nz - 1 - jb - jj;
            return e < S4 * P && p < R && jj < njp && s2 < Ts && b >= 0 && b < N;
        };
        auto src_load = [&](int qb, double (&v)[SQL]) {
            if (!any_dsnb) return;
#pragma unroll
            for (int u = 0; u < SQL; ++u) {
                int p, b, i;
                const int e = lane + 64 * u;
                v[u] = (src_valid(qb, e, p, b, i) && pinf[2 * P + p] == 0.0)
                           ? t.Src[(size_t)pinf[3 * P + p] * T * nst + src_index(Nz, jb + (e / P) % NJ, b)] : 0.0;
            }
        };
        auto src_store = [&](int qb, const double (&v)[SQL]) {
            if (!kSrcRec && !any_dsnb) return;
#pragma unroll
            for (int u = 0; u < SQL; ++u) {
                int p, b, i;
                const int e = lane + 64 * u;
                if (src_valid(qb, e, p, b, i)) {
                    if (pinf[2 * P + p] == 0.0)
                        srcb[(qb & 1) * 4 * NC + e] = v[u];
                    else if (kSrcRec)
                        srcb[(qb & 1) * 4 * NC + e] =
                            powerlaw_src_h(gl, SrcFactors{pinf[p], pinf[P + p]}, pw + (size_t)p * (T + 2), i, b);
                }
            }
        };
        auto finalise = [&](int qb) {   // the last pass' stages of block qb (nuSIprop.hpp:328-336)
            for (int e = lane; e < 4 * P; e += 64) {
                const int d = e / P, p = e - P * (e / P), sg = 4 * qb + d, b = N - 1 - sg + njp - 1;
                if (p < R && sg < Ts && b >= 0 && b < N) {
                    const double* fo = fin + (((qb & 1) * 4 + d) * 3) * P + p;
                    const int cpid = (int)pinf[3 * P + p];
                    const double* U2 = pinf + 4 * P + p;
                    const double dE = gl.Emax[b] - gl.Emin[b];
                    const double g0 = fo[0] / dE, g1 = fo[P] / dE, g2 = fo[2 * P] / dE;
                    double* fx = flux + (size_t)cpid * 3 * N;
                    double* fl = flux_fla + (size_t)cpid * 3 * N;
                    fx[b] = g0;
                    fx[N + b] = g1;
                    fx[2 * N + b] = g2;
                    for (int f = 0; f < 3; ++f)
                        fl[f * N + b] = U2[(3 * f + 0) * P] * g0 + U2[(3 * f + 1) * P] * g1 + U2[(3 * f + 2) * P] * g2;
                }
            }
        };
        constexpr int FQL = (NQ + 63) / 64;   // FIFO values per lane and block
        auto fifo_load = [&](int pass, int qb, double (&v)[FQL]) {
#pragma unroll
            for (int u = 0; u < FQL; ++u) {
                const int e = lane + 64 * u, d = e / (3 * P), c = (e / P) % 3, p = e % P, sg = 4 * qb + d, bq = N - 1 - sg;
                v[u] = (pass > 0 && e < NQ && sg < Ts && bq >= 0)
                           ? __builtin_nontemporal_load(fhw + ((size_t)c * N + bq) * P + p) : 0.0;
            }
        };
        auto fifo_store = [&](int qb, const double (&v)[FQL]) {
#pragma unroll
            for (int u = 0; u < FQL; ++u)
                if (lane + 64 * u < NQ) fqb[(qb & 1) * NQ + lane + 64 * u] = v[u];
        };
#pragma unroll 1
        for (int pass = 0; pass < npass; ++pass) {
            pass_geom(pass);
            __syncthreads();
            any_dsnb = false;
            for (int p = 0; p < R; ++p) any_dsnb = any_dsnb || pinf[2 * P + p] == 0.0;
            records(0, 0, S4);
            sources(0);
            double sv[SQL];
            if (kAhead) src_load(1, sv);
            double fv[FQL];
            fifo_load(pass, 0, fv);
            fifo_store(0, fv);
            fifo_load(pass, 1, fv);
            __syncthreads();
#pragma unroll 1
            for (int q = 0; q < nblk; ++q) {
                NUSI_BS_STAMP(pass * nblk + q, 0);
                fifo_store(q + 1, fv);                  // block q + 1's FIFO values (loaded a block ago)
                fifo_load(pass, q + 2, fv);
                if (4 * (q + 1) < Ts) records(q + 1, 0, kRecSplit);   // phase A
                NUSI_BS_STAMP(pass * nblk + q, 1);
                __syncthreads();
                NUSI_BS_STAMP(pass * nblk + q, 2);
                if (4 * (q + 1) < Ts) {                                // phase B
                    records(q + 1, kRecSplit, S4);
                    if (kAhead) {
                        src_store(q + 1, sv);           // block q + 1's sources (loaded a block ago)
                        if (4 * (q + 2) < Ts) src_load(q + 2, sv);
                    } else
                        sources(q + 1);
                }
                if (pass == npass - 1 && q > 0) finalise(q - 1);
                NUSI_BS_STAMP(pass * nblk + q, 3);
                __syncthreads();
            }
            if (pass == npass - 1) finalise(nblk - 1);   // (after the loop's last barrier: the chain's last block is in fin)
        }
    } else {
        // ---- push: block q adds columns c0+1-4q .. c0+4-4q (the T of stages 4q-1 .. 4q-4) into the rows below
        // r = c0-4q: in phase A the tiles holding rows r-1 .. r-4 (published to AX), in phase B the others
#if NUSI_BS_SIMDMAP
        int rb = 0;   // this push wave's row block: the waves sharing no SIMD with a chain or the record wave take the
        {             // bottom rows (busiest), then those beside the record wave, then those beside a chain wave
            const int npush = nw - 1 - CW;
            auto cls = [&](int w) {
                for (int c = chw; c < nw; ++c)
                    if ((c & 3) == (w & 3)) return 2;
                return (recw & 3) == (w & 3) ? 1 : 0;
            };
            const int mine = cls(wave);
            for (int w = 0; w < npush; ++w) {
                const int o = cls(w);
                if (o < mine || (o == mine && w < wave)) ++rb;
            }
        }
        const int rw0 = rb * 16 * RT;
#else
        const int rw0 = wave * 16 * RT;
#endif
#pragma unroll 1
        for (int pass = 0; pass < npass; ++pass) {
            pass_geom(pass);
            __syncthreads();
            __syncthreads();
            nusi_f64x4 acc[RT][NB];
#pragma unroll
            for (int a = 0; a < RT; ++a)
#pragma unroll
                for (int s = 0; s < NB; ++s) acc[a][s] = nusi_f64x4{0.0, 0.0, 0.0, 0.0};
            auto load_blk = [&](int q, double (&dst)[RT]) {
                int c = c0 + 1 - 4 * q + (lane >> 4);
                c = c < 1 ? 1 : (c > T - 1 ? T - 1 : c);
                const size_t cb = (size_t)c * (c - 1) / 2;
#pragma unroll
                for (int a = 0; a < RT; ++a) {
                    const int row = rw0 + 16 * a + (lane & 15);
                    dst[a] = Al[cb + (row < c - 1 ? row : c - 1)];
                }
            };
            auto push = [&](int q, const double (&ab)[RT], bool phase_a) {
                const int r = c0 - 4 * q, hi = r - 1;
                const double* Tq = Tp + ((4 * q - 1 - (lane >> 4)) & 7) * NC + (lane & 15);
#pragma unroll
                for (int a = 0; a < RT; ++a) {
                    const bool crit = rw0 + 16 * a <= hi && rw0 + 16 * a + 15 >= hi - 3;   // uniform
                    if (crit == phase_a && rw0 + 16 * a < r)   // tiles wholly at or above r hold consumed rows only
#pragma unroll
                        for (int s = 0; s < NB; ++s)
#ifdef NUSI_BS_NOPUSH   // timing diagnostic only (wrong fluxes): the block pushes without the matrix core
                            acc[a][s][0] += ab[a] * Tq[16 * s];
#else
                            acc[a][s] = __builtin_amdgcn_mfma_f64_16x16x4f64(ab[a], Tq[16 * s], acc[a][s], 0, 0, 0);
#endif
                }
                if (phase_a)
#pragma unroll
                    for (int a = 0; a < RT; ++a)
                        if (rw0 + 16 * a <= hi && rw0 + 16 * a + 15 >= hi - 3)
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const int row = rw0 + 16 * a + (lane >> 4) + 4 * e;
                                const int slot = hi - row;
                                if (slot >= 0 && slot < 4)
#pragma unroll
                                    for (int s = 0; s < NB; ++s)
                                        AX[((q & 1) * 4 + slot) * NC + 16 * s + (lane & 15)] = acc[a][s][e];
                            }
            };
            auto block = [&](int q, double (&ab)[RT]) {   // ab holds block q's A operands; then block q + 2's
                const bool doq = nonres && q >= 1 && 4 * q < Ts;
                NUSI_BS_STAMP(pass * nblk + q, 0);
                if (doq) push(q, ab, true);
                NUSI_BS_STAMP(pass * nblk + q, 1);
                __syncthreads();
                NUSI_BS_STAMP(pass * nblk + q, 2);
                if (doq) push(q, ab, false);
                load_blk(q + 2, ab);
                NUSI_BS_STAMP(pass * nblk + q, 3);
                __syncthreads();
            };
            double ab0[RT], ab1[RT];
            load_blk(0, ab0);
            load_blk(1, ab1);
#pragma unroll 1
            for (int q = 0; q < nblk; q += 2) {
                block(q, ab0);
                if (q + 1 < nblk) block(q + 1, ab1);
            }
        }
    }
}
// the redshift-step slots of a one-pass wavefront: up to 48 (Nz - 1 rounded up to 16, 32 or 48), 0 beyond
static int wf_nj(const GridDev& g) { const int n = g.Nz - 1; return n <= 16 ? 16 : n <= 32 ? 32 : n <= 48 ? 48 : 0; }

static thread_local const char* t_cascade_kernel = "";   // the kernel the latest launch on this thread chose
const char* last_cascade_kernel() { return t_cascade_kernel; }

// the block-synchronous kernel (k_cascade_bs): push waves of 16 RT rows, the chain wave, the record wave
static int bs_push_waves(const GridDev& g, int RT) { return (g.T - 1 + 16 * RT - 1) / (16 * RT); }
template <int NJ, int P, int SPL, int RT, int CW>
static size_t bs_lds(const GridDev& g)
{
    constexpr int NC = NJ * P;
    return sizeof(double) * (2 * (size_t)kBsFields * 4 * NJ + 3 * 8 * (size_t)NC + 48 * (size_t)P + 13 * (size_t)P +
                             3 * (size_t)g.N + (size_t)P * (g.T + 2) + 6 * (size_t)g.T + 4 * (size_t)g.Nz);
}
template <int NJ, int P, int SPL, int RT, int CW>
static bool bs_fits_t(const GridDev& g)
{
    return g.T >= 2 && g.Nz >= 2 && bs_push_waves(g, RT) + CW + 1 <= 16 && bs_lds<NJ, P, SPL, RT, CW>(g) <= 160 * 1024;
}
template <int NJ, int P, int SPL, int RT, int CW>
static void launch_bs_t(const GridDev& g, const Point* pts, const int* gidx, const int2* grp, int nwg, TablesDev t,
                        double* fh, double* flux, double* flux_fla, hipStream_t s, bool all_nr)
{
    const int nthr = 64 * (bs_push_waves(g, RT) + CW + 1);
    const size_t lds = bs_lds<NJ, P, SPL, RT, CW>(g);
    if (all_nr)   // the instance without the resonant-only running sum (every BASELINE workload)
        hipLaunchKernelGGL((k_cascade_bs<NJ, P, SPL, RT, CW, true>), dim3(nwg), dim3(nthr), lds, s, g, pts, gidx, grp, t, fh,
                           flux, flux_fla);
    else
        hipLaunchKernelGGL((k_cascade_bs<NJ, P, SPL, RT, CW, false>), dim3(nwg), dim3(nthr), lds, s, g, pts, gidx, grp, t,
                           fh, flux, flux_fla);
}
// P = 1: <wf_nj, 1, 1, 4, 1> for one pass of up to 48 steps, else step passes of 48 (rows <= 14 x 64) or of 16 (rows
// <= 14 x 128; force_passes: that instance on any grid it fits); P = 2: <wf_nj or 48, 2, 1, 2, 2>; P = 16 (the gamma
// batch): <6, 16, 1, 2, 2>
int cascade_bs_config(const GridDev& g, int P, bool force_passes)
{
    const int nj = wf_nj(g);
    if (P == 1 && force_passes) return bs_fits_t<16, 1, 1, 8, 1>(g) ? 16 + 1000 : 0;   // NUSI_OPT_STEP_PASSES = 1
    if (P == 1) {
        if (nj && bs_fits_t<48, 1, 1, 4, 1>(g)) return nj;
        if (bs_fits_t<48, 1, 1, 4, 1>(g)) return 48;
        if (NUSI_BS_LONG32 && bs_fits_t<32, 1, 1, 6, 1>(g)) return 32 + 2000;   // 96-row push waves, passes of 32
        if (bs_fits_t<16, 1, 1, 8, 1>(g)) return 16 + 1000;   // 128-row push waves
        return 0;
    }
    if (P == 2) return bs_fits_t<48, 2, 1, 2, 2>(g) ? (nj ? nj : 48) : 0;
    if (P == 16) return bs_fits_t<6, 16, 1, 2, 2>(g) ? 6 : 0;
    return 0;
}
size_t cascade_bs_scratch_doubles(const GridDev& g, int P) { return (size_t)3 * g.N * P; }
hipError_t launch_cascade_bs(const GridDev& g, const Point* pts, int P, const int* gidx, const int2* grp, int nwg,
                             TablesDev t, double* fh, double* flux, double* flux_fla, hipStream_t s, bool all_nr,
                             bool force_passes)
{
    if (nwg <= 0) return hipSuccess;
    const int c = cascade_bs_config(g, P, force_passes && P == 1);
    if (!c) return hipErrorInvalidValue;
    if (P == 1) {
        t_cascade_kernel = "k_cascade_bs";
        switch (c) {
        case 16: launch_bs_t<16, 1, 1, 4, 1>(g, pts, gidx, grp, nwg, t, fh, flux, flux_fla, s, all_nr); break;
        case 32: launch_bs_t<32, 1, 1, 4, 1>(g, pts, gidx, grp, nwg, t, fh, flux, flux_fla, s, all_nr); break;
        case 48: launch_bs_t<48, 1, 1, 4, 1>(g, pts, gidx, grp, nwg, t, fh, flux, flux_fla, s, all_nr); break;
#if NUSI_BS_LONG32
        case 2032: launch_bs_t<32, 1, 1, 6, 1>(g, pts, gidx, grp, nwg, t, fh, flux, flux_fla, s, all_nr); break;
#endif
        default: launch_bs_t<16, 1, 1, 8, 1>(g, pts, gidx, grp, nwg, t, fh, flux, flux_fla, s, all_nr); break;
        }
    } else if (P == 2) {
        t_cascade_kernel = "k_cascade_bs_pairs";
        switch (c) {
        case 16: launch_bs_t<16, 2, 1, 2, 2>(g, pts, gidx, grp, nwg, t, fh, flux, flux_fla, s, all_nr); break;
        case 32: launch_bs_t<32, 2, 1, 2, 2>(g, pts, gidx, grp, nwg, t, fh, flux, flux_fla, s, all_nr); break;
        default: launch_bs_t<48, 2, 1, 2, 2>(g, pts, gidx, grp, nwg, t, fh, flux, flux_fla, s, all_nr); break;
        }
    } else {
        t_cascade_kernel = "k_cascade_bs_gamma";
        launch_bs_t<6, 16, 1, 2, 2>(g, pts, gidx, grp, nwg, t, fh, flux, flux_fla, s, all_nr);
    }
    return hipGetLastError();
}

// the bit-exact scalar cascade (NUSI_CASCADE_WAVEFRONT / REG / LDS): k_cascade, one wavefront per point, any N
hipError_t launch_cascade_exact(const GridDev& g, const Point* pts, int npts, TablesDev t, double* flux,
                                double* flux_fla, hipStream_t s)
{
    t_cascade_kernel = "k_cascade";
    const size_t lds = cascade_lds_bytes(g.N);
    hipLaunchKernelGGL(k_cascade, dim3(npts), dim3(64), lds, s, g, pts, t, flux, flux_fla);
    return hipGetLastError();
}

}  // namespace nusi

#ifdef NUSI_WS_TRACE
// diagnostic build: workgroup 0's block stamps of the latest k_cascade_bs launch, [wave][block][phase stamps]
extern "C" int nusi_debug_ws_trace(unsigned long long* out, int n)
{
    const int m = n < nusi::kTrWaves * nusi::kTrStages * 4 ? n : nusi::kTrWaves * nusi::kTrStages * 4;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(nusi::g_ws_trace), sizeof(unsigned long long) * m) == hipSuccess ? 0 : -5;
}
// HW_ID of every wave of the first kTrBlocks workgroups, [block][wave]
extern "C" int nusi_debug_ws_hwid(unsigned int* out, int n)
{
    const int m = n < nusi::kTrBlocks * nusi::kTrWaves ? n : nusi::kTrBlocks * nusi::kTrWaves;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(nusi::g_ws_hwid), sizeof(unsigned int) * m) == hipSuccess ? 0 : -5;
}
#endif
