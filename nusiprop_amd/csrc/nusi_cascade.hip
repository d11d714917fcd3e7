// nuSIprop MI355X -- Stage B: the implicit redshift cascade + finalisation
// (calculate_flux::evolve, nuSIprop.hpp:255-336).
//
//   k_cascade_ws<NJ, R>   warp-specialised wavefront, push on the fp64 matrix cores, R points sharing a
//                         table per workgroup (NUSI_CASCADE_AUTO / MFMA, Nz-1 <= 48)
//   k_cascade_wsp<NJ, NR> the same in passes of 16 redshift steps (Nz-1 > 48)
//   k_source_dsnb         the DSNB source terms those two read
//   k_cascade_wf<NJ>      bit-exact scalar wavefront (NUSI_CASCADE_WAVEFRONT)
//   k_cascade_reg<NQ, D>  bit-exact per-step chain in registers, N <= 64 NQ (NUSI_CASCADE_REG, fallback)
//   k_cascade             LDS-resident generic path, any N (NUSI_CASCADE_LDS, last fallback)
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

// The record of (step i, bin b) in two phases (k_cascade_ws runs them on different waves, one stage
// apart; cascade_record runs them back to back -- the same operations either way):
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

// ---------------------------------------------------------------------------
// Register-resident cascade (N <= 64 * 20 = 1280).
//
// Same arithmetic, in the same order, as k_cascade, but nothing on the
// per-bin chain touches memory:
//   * bin b is owned by lane b % 64, slot b / 64: F_k[b] and acc[b] live in
//     registers (F[k][q], acc[q]); uniform reads of one bin are readlanes;
//   * the per-bin precomputed fields of the current 64-bin chunk sit in the
//     owning lane's registers and are broadcast with readlane;
//   * the alpha column each bin pushes (alpha(b', b), b' < b) is prefetched D
//     bins ahead into a register ring, so the HBM latency of the table stream
//     is hidden behind D bins of the chain.
// The chunk loop is fully unrolled (NQ is a template parameter) so every
// register array is statically indexed.
// ---------------------------------------------------------------------------

__device__ __forceinline__ double rl(double v, int l)
{
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)x, l);
    const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// alpha(b', bn) for b' = lane + 64 q < bn (column r = bn + i - 1 of the packed transposed table),
// slots q <= qmax.  The loads are unconditional -- a masked (exec-branched) load would break the
// compiler's vmcnt bookkeeping and force a full drain every bin.  Slots q <= qmax - 2 lie entirely
// below bn (bn >= 64 qmax - D) and need no clamp; the top two slots clamp the row index into the
// column.  Lanes past the column read a valid neighbour that every consumer masks out.
template <int NQ>
__device__ __forceinline__ void load_col(double (&dst)[NQ], const double* __restrict__ Al, int bn, int i, int N,
                                         int lane, int qmax)
{
    const int bc = bn < 1 ? 1 : (bn > N - 1 ? N - 1 : bn);
    const int r = bc + i - 1;
    const double* col = Al + (size_t)r * (r - 1) / 2 + (i - 1);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if (q > qmax) continue;                // qmax is a compile-time constant after unrolling
        const int bp = lane + 64 * q;
        dst[q] = (q <= qmax - 2) ? col[bp] : col[bp < bc ? bp : bc - 1];
    }
}

// per-bin record of the current 64-bin chunk in LDS, read by every lane with broadcast
// ds_read_b128s: the 14 flux-independent fields, the LU permutation, and the bin's flux
// of the previous step (which the chain needs once, so it is staged with the fields)
constexpr int kRec = 18;   // doubles per record: PR_* (14), perm, F0, F1, F2
enum { RC_PERM = kPreFields, RC_F0, RC_F1, RC_F2 };

template <int NQ, int D>
__global__ __launch_bounds__(64) void k_cascade_reg(GridDev g, const Point* __restrict__ pts, TablesDev t,
                                                    double* __restrict__ flux, double* __restrict__ flux_fla)
{
    extern __shared__ __attribute__((aligned(16))) double sdiag[];   // resonant-only: alpha(b+i-1, b+i) [N]
    __shared__ __attribute__((aligned(16))) double rec[64 * kRec];
    double* rdE = sdiag + g.N;       // cascade_aux_init tables
    double* pw = rdE + g.N;
    const int N = g.N, Nz = g.Nz, T = g.T;
    const int p = blockIdx.x, lane = threadIdx.x;
    const Point& P = pts[p];
    const double u0 = P.u[0], u1 = P.u[1], u2 = P.u[2];
    const double* __restrict__ Gt = t.G + (size_t)P.tslot * T;
    const double* __restrict__ At = t.At + (size_t)P.tslot * T;
    const double* __restrict__ Al = t.A + (size_t)P.tslot * g.PT;
    const bool nonres = P.non_resonant;

    double F0[NQ], F1[NQ], F2[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) F0[q] = F1[q] = F2[q] = 0.0;
    cascade_aux_init(g, P, rdE, pw, lane, 64);

    for (int i = Nz - 1; i > 0; --i) {
        const double c = g.step_c[i], s = g.step_s[i];
        if (!nonres) {
            __syncthreads();
            for (int b = lane; b < N - 1; b += 64) sdiag[b] = Al[(size_t)(b + i) * (b + i - 1) / 2 + (b + i - 1)];
        }
        double acc[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
        double ring[D][NQ];   // loaded unconditionally (also when only the resonant chain uses none of it)
#pragma unroll
        for (int j = 0; j < D; ++j) load_col<NQ>(ring[j], Al, 64 * NQ - 1 - j, i, N, lane, NQ - 1);
        double next_acc = 0.0, racc = 0.0;
        double px0 = 0.0, px1 = 0.0, px2 = 0.0;
#pragma unroll
        for (int qc = NQ - 1; qc >= 0; --qc) {
            const int base = 64 * qc;
            __syncthreads();   // previous chunk's records consumed
            {   // ---- flux-independent fields of bin base + lane (one bin per lane) -> LDS record
                const int b = base + lane;
                double* R = rec + lane * kRec;
                if (b < N) {
                    cascade_record<false>(g, P, Gt, At, rdE, pw, i, b, R, 1);
                    R[RC_F0] = F0[qc];
                    R[RC_F1] = F1[qc];
                    R[RC_F2] = F2[qc];
                }
            }
            __syncthreads();
            for (int gq = 0; gq < 64 / D; ++gq) {
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const int l = 63 - (gq * D + j);
                    const int b = base + l;
                    if (b <= N - 1) {
                        const double2* R2 = reinterpret_cast<const double2*>(rec + l * kRec);
                        const double2 r01 = R2[0], r23 = R2[1], r45 = R2[2], r67 = R2[3], r89 = R2[4], r1011 = R2[5],
                                      r1213 = R2[6], r1415 = R2[7], r1617 = R2[8];
                        const double rz0 = r01.x, rz1 = r01.y, rz2 = r23.x, src0 = r23.y;
                        const double l10 = r45.x, l20 = r45.y, l21 = r67.x, u01 = r67.y, u02 = r89.x, u12 = r89.y;
                        const double ru00 = r1011.x, ru11 = r1011.y, ru22 = r1213.x, sde = r1213.y;
                        const int pmb = (int)r1415.x;
                        const double f0 = r1415.y, f1 = r1617.x, f2 = r1617.y;
                        double add;
                        if (nonres) {
                            add = c * next_acc;
                        } else {
                            if (b != N - 1) {
                                const double Sres = u0 * px0 + u1 * px1 + u2 * px2;
                                racc += Sres * (s * sdiag[b]) / (g.Emax[b + 1] - g.Emin[b + 1]) / sde;
                            }
                            add = c * racc * sde;
                        }
                        double x0, x1, x2;
                        cascade_solve(f0, f1, f2, add, src0, u0, u1, u2, rz0, rz1, rz2, pmb, l10, l20, l21, u01, u02,
                                      u12, ru00, ru11, ru22, x0, x1, x2);
                        if (lane == l) { F0[qc] = x0; F1[qc] = x1; F2[qc] = x2; }
                        px0 = x0; px1 = x1; px2 = x2;
                        if (nonres && b > 0) {
                            const double Tb = (u0 * x0 + u1 * x1 + u2 * x2) * sde;
                            double accb, diag;
                            if (l > 0) {
                                accb = rl(acc[qc], l - 1);
                                diag = rl(ring[j][qc], l - 1);
                            } else {
                                accb = rl(acc[qc > 0 ? qc - 1 : 0], 63);
                                diag = rl(ring[j][qc > 0 ? qc - 1 : 0], 63);
                            }
                            next_acc = fma(diag, Tb, accb);
                            // push T_b into every lower bin b' < b - 1 (bin b - 1 is carried in next_acc):
                            // slots below qc - 1 are entirely below b - 1; only the top two need a mask
#pragma unroll
                            for (int q = 0; q <= qc; ++q) {
                                if (q <= qc - 2) acc[q] = fma(ring[j][q], Tb, acc[q]);
                                else if (lane + 64 * q < b - 1) acc[q] = fma(ring[j][q], Tb, acc[q]);
                            }
                        }
                    }
                    load_col<NQ>(ring[j], Al, b - D, i, N, lane, qc);
                }
            }
        }
    }
    // finalise (nuSIprop.hpp:328-336)
    double* fo = flux + (size_t)p * 3 * N;
    double* fl = flux_fla + (size_t)p * 3 * N;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int b = lane + 64 * q;
        if (b < N) {
            const double dE = g.Emax[b] - g.Emin[b];
            const double f0 = F0[q] / dE, f1 = F1[q] / dE, f2 = F2[q] / dE;
            fo[b] = f0;
            fo[N + b] = f1;
            fo[2 * N + b] = f2;
            for (int f = 0; f < 3; ++f)
                fl[f * N + b] = P.U2[3 * f + 0] * f0 + P.U2[3 * f + 1] * f1 + P.U2[3 * f + 2] * f2;
        }
    }
}

// ---------------------------------------------------------------------------
// Wavefront cascade: all redshift steps of a point in flight at once.
//
// Step i may solve bin b as soon as step i+1 has finalised F[:, b] and step i
// has solved every bin above b.  Lagging step i by one bin behind step i+1
// (lane j = Nz-1-i solves bin b = N-1-sg+j at stage sg) meets both conditions,
// so the (Nz-1) N sequential solves of the reference's loop nest collapse into
// T = N+Nz-2 stages of up to Nz-1 independent solves.  Along a stage b + i is
// constant: every active step reads the SAME table column r = T-1-sg (the
// index-shift identity, nuSIprop.hpp:262-275), so each column of the packed
// alpha table is read from HBM once per point instead of once per step.
//
// A workgroup holds acc_j(rho) for every table row rho < T-1 and step j in
// registers: thread = (group of 4 rows, quarter of the steps), so each T_j
// broadcast read from LDS feeds 4 fma()s.  Per stage:
//   P1  wave 0, lane j: the 3x3 solve of its (step, bin) from LDS records and
//       the accumulator of row r (published by its owner), T_j -> LDS
//   P2  every row: the push of column r; the owner of row r-1 publishes its
//       accumulators for the next stage's chain
// The flux-independent records of K = threads/NJ stages are computed by all
// threads at once (one (stage, step) per thread) before those stages.
// Every accumulator receives the same fma()s in the same (descending column)
// order as in k_cascade_reg, and the solve is cascade_solve(): the two kernels
// agree bit for bit.  Rows rho < i-1 of step j are pushed too (no mask); they
// never feed a solve.
// ---------------------------------------------------------------------------
constexpr int kWfFields = kPreFields + 1;   // PR_* and the permutation
constexpr int kWfMaxThreads = 512;
constexpr int kWfRows = 4, kWfQuarters = 4;   // push: rows per thread, step groups per row group
constexpr int kWfPre = 2;           // alpha columns in flight (stages of prefetch)

template <int NJ, bool kPowerLaw>
__global__ __launch_bounds__(kWfMaxThreads) void k_cascade_wf(GridDev g, const Point* __restrict__ pts, TablesDev t,
                                                              double* __restrict__ flux, double* __restrict__ flux_fla,
                                                              int K)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int N = g.N, Nz = g.Nz, T = g.T, nst = Nz - 1;
    const int tid = threadIdx.x, nthr = blockDim.x;   // K: stages per record batch, K NJ <= nthr
    const int KR = K * NJ;                   // records per batch (field stride)
    double* F = lds;                         // [3][N]
    double* rec = F + 3 * N;                 // [kWfFields][K][NJ]
    double* Tp = rec + kWfFields * KR;       // [2][NJ]  T_j of the stage (double-buffered by stage parity)
    double* AX = Tp + 2 * NJ;                // [2][NJ]  accumulators B_j of the row the chain solves next
    double* rdE = AX + 2 * NJ;               // cascade_aux_init tables
    double* pw = rdE + N;
    // per-point and grid arrays the stage loop reads, staged in LDS: the loop's only global loads
    // are then the alpha-column prefetches, whose waits the compiler can count exactly
    double* sGt = pw + (T + 2);
    double* sAt = sGt + T;
    double* sdg = sAt + T;                   // alpha(r, r+1) (resonant-only chain)
    double* sEmin = sdg + T;
    double* sEmax = sEmin + N;
    double* sgz = sEmax + N;                 // z, step_c, step_s, sfr [Nz each]
    GridDev gl = g;
    gl.Emin = sEmin;
    gl.Emax = sEmax;
    gl.z = sgz;
    gl.step_c = sgz + Nz;
    gl.step_s = sgz + 2 * Nz;
    gl.sfr = sgz + 3 * Nz;
    const Point& P = pts[blockIdx.x];
    const double u0 = P.u[0], u1 = P.u[1], u2 = P.u[2];
    const double* __restrict__ Gt = t.G + (size_t)P.tslot * T;
    const double* __restrict__ At = t.At + (size_t)P.tslot * T;
    const double* __restrict__ Al = t.A + (size_t)P.tslot * g.PT;
    const bool nonres = P.non_resonant;

    for (int b = tid; b < 3 * N; b += nthr) F[b] = 0.0;
    for (int j = tid; j < 2 * NJ; j += nthr) AX[j] = Tp[j] = 0.0;
    for (int n = tid; n < T; n += nthr) {
        sGt[n] = Gt[n];
        sAt[n] = At[n];
        sdg[n] = (n + 1 < T) ? Al[(size_t)(n + 1) * n / 2 + n] : 0.0;
    }
    for (int b = tid; b < N; b += nthr) { sEmin[b] = g.Emin[b]; sEmax[b] = g.Emax[b]; }
    for (int i = tid; i < Nz; i += nthr) {
        sgz[i] = g.z[i];
        sgz[Nz + i] = g.step_c[i];
        sgz[2 * Nz + i] = g.step_s[i];
        sgz[3 * Nz + i] = g.sfr[i];
    }
    cascade_aux_init(g, P, rdE, pw, tid, nthr);
    // push geometry: thread = (row group, step quarter); kWfRows rows x JG steps of accumulators
    constexpr int JG = NJ / kWfQuarters;
    const int h = tid & (kWfQuarters - 1), row0 = (tid / kWfQuarters) * kWfRows;
    double acc[kWfRows][JG];
#pragma unroll
    for (int c = 0; c < kWfRows; ++c)
#pragma unroll
        for (int jj = 0; jj < JG; ++jj) acc[c][jj] = 0.0;
    // chain lane state (the last wave, lane = step slot j)
    const int cbase = nthr - 64, cj_lane = tid - cbase;
    const bool chain = cj_lane >= 0 && cj_lane < nst;
    const int ist = Nz - 1 - cj_lane;
    __syncthreads();   // staged arrays visible; the chain reads its step's c_i, s_i from LDS (a global load
                       // here would be waited for with vmcnt(0) inside the loop, draining the prefetches)
    const double cj = chain ? gl.step_c[ist] : 0.0, sj = chain ? gl.step_s[ist] : 0.0;
    double racc = 0.0, px0 = 0.0, px1 = 0.0, px2 = 0.0;
    double Tprev = 0.0;   // the lane's T_j of the previous stage
    // alpha(row, column) of the next kWfPre stages' columns (ring, [0] = this stage's), rows clamped
    // into the column; each load is issued kWfPre stages before its use (HBM latency > a stage)
    // The loads are unconditional (column clamped to >= 1, rows into the column; resonant-only
    // tables are allocated in full): a load skipped on some path would make the compiler wait for
    // every outstanding load (vmcnt(0)) at the next use.  Columns < 1 are never pushed.
    auto load_col = [&](int col, double (&dst)[kWfRows]) {
        const int cl = col < 1 ? 1 : (col > T - 1 ? T - 1 : col);
        const size_t cb = (size_t)cl * (cl - 1) / 2;
#pragma unroll
        for (int c = 0; c < kWfRows; ++c) {
            const int row = row0 + c;
            dst[c] = Al[cb + (row < cl - 1 ? row : cl - 1)];
        }
    };
    double a_ring[kWfPre][kWfRows];
#pragma unroll
    for (int d = 0; d < kWfPre; ++d) {   // issued in slot order (the loop's waits count on it)
        load_col(T - d, a_ring[d]);      // stage d pushes column T - d (none at stage 0)
        NUSI_PHASE();
    }
    // stage sg; ac = its alpha column (ring slot sg % kWfPre), reloaded with the column kWfPre
    // stages ahead after its use (the stage loop is unrolled by kWfPre, so the ring needs no
    // register moves, which would wait for the newest loads)
    for (int sg0 = 0; sg0 < T; sg0 += kWfPre)
#pragma unroll
    for (int d = 0; d < kWfPre; ++d) {
        const int sg = sg0 + d;
        if (sg >= T) break;
        double (&ac)[kWfRows] = a_ring[d];
        const int r = T - 1 - sg;
        const int ks = sg % K;
        if (ks == 0) {   // ---- records of stages sg .. sg+K-1, one (stage, step) per thread
            __syncthreads();
            const int q = tid / NJ, jj = tid - q * NJ, s2 = sg + q;
            if (q < K && jj < nst && s2 < T) {
                const int b = N - 1 - s2 + jj;
                if (b >= 0 && b < N) cascade_record<kPowerLaw>(gl, P, sGt, sAt, rdE, pw, Nz - 1 - jj, b, rec + q * NJ + jj, KR);
            }
            __syncthreads();
        }
        // ---- one phase per stage (one barrier):
        //   the chain (last wave) solves column r: its row's accumulator is the published B_j(r)
        //   (columns >= r+2) plus column r+1, which the lane adds itself from its own T_j(sg-1);
        //   the bulk push (other waves) adds column r+1 (T of stage sg-1) to the rows < r and
        //   publishes B(r-1) (columns >= r+1) for the next stage.  Every accumulator receives the
        //   same fma()s in the same descending-column order as before.
        const int cur = sg & 1, prv = cur ^ 1;
        if (chain) {
            const int tid = cj_lane;
            const int b = N - 1 - sg + tid;
            double T_j = 0.0;
            if (b >= 0 && b < N) {
                const double* R = rec + ks * NJ + tid;
                double add;
                if (nonres) {
                    add = cj * fma(sdg[r], Tprev, AX[prv * NJ + tid]);
                } else {
                    if (b != N - 1) {
                        const double Sres = u0 * px0 + u1 * px1 + u2 * px2;
                        const double sd = sdg[r];   // alpha(b+i-1, b+i)
                        racc += Sres * (sj * sd) / (sEmax[b + 1] - sEmin[b + 1]) / R[PR_SDE * KR];
                    }
                    add = cj * racc * R[PR_SDE * KR];
                }
                double x0 = add, x1 = add, x2 = add;
                cascade_solve(F[b], F[N + b], F[2 * N + b], add, R[PR_SRC * KR], u0, u1, u2, R[PR_RZ0 * KR],
                              R[PR_RZ1 * KR], R[PR_RZ2 * KR], (int)R[kPreFields * KR], R[PR_L10 * KR], R[PR_L20 * KR],
                              R[PR_L21 * KR], R[PR_U01 * KR], R[PR_U02 * KR], R[PR_U12 * KR], R[PR_RU00 * KR],
                              R[PR_RU11 * KR], R[PR_RU22 * KR], x0, x1, x2);
                F[b] = x0;
                F[N + b] = x1;
                F[2 * N + b] = x2;
                px0 = x0; px1 = x1; px2 = x2;
                if (nonres && b > 0) T_j = (u0 * x0 + u1 * x1 + u2 * x2) * R[PR_SDE * KR];
            }
            Tp[cur * NJ + tid] = T_j;
            Tprev = T_j;
        } else if (tid < cbase && nonres && r >= 1 && r + 1 <= T - 1 && row0 < r) {
            // push column r+1 (T of stage sg-1) into rows < r; rows >= r are consumed (row r through
            // the published copy), so a row group wholly at or above r stops pushing (whole waves drop
            // out as r falls); steps that have not started have T_j = 0, so nothing else is masked
            const double* Th = Tp + prv * NJ + h * JG;
#pragma unroll
            for (int jj = 0; jj < JG; ++jj) {
                const double tj = Th[jj];
#pragma unroll
                for (int c = 0; c < kWfRows; ++c) acc[c][jj] = fma(ac[c], tj, acc[c][jj]);
            }
            if (r - 1 >= row0 && r - 1 < row0 + kWfRows) {   // publish B(r-1) for the next stage's chain
                const int cp = r - 1 - row0;
#pragma unroll
                for (int c = 0; c < kWfRows; ++c)
                    if (c == cp) {
#pragma unroll
                        for (int jj = 0; jj < JG; ++jj) AX[cur * NJ + h * JG + jj] = acc[c][jj];
                    }
            }
        }
        load_col(r + 1 - kWfPre, ac);
        __syncthreads();
    }
    // finalise (nuSIprop.hpp:328-336)
    double* fo = flux + (size_t)blockIdx.x * 3 * N;
    double* fl = flux_fla + (size_t)blockIdx.x * 3 * N;
    for (int b = tid; b < N; b += nthr) {
        const double dE = g.Emax[b] - g.Emin[b];
        const double f0 = F[b] / dE, f1 = F[N + b] / dE, f2 = F[2 * N + b] / dE;
        fo[b] = f0;
        fo[N + b] = f1;
        fo[2 * N + b] = f2;
        for (int f = 0; f < 3; ++f) fl[f * N + b] = P.U2[3 * f + 0] * f0 + P.U2[3 * f + 1] * f1 + P.U2[3 * f + 2] * f2;
    }
}

typedef double nusi_f64x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// Warp-specialised MFMA cascade, R right-hand sides per workgroup (NUSI_CASCADE_MFMA / AUTO: every
// point kind -- power-law or DSNB source, non-resonant or resonant-only).
//
// The wavefront of k_cascade_wf (stage sg: step slot j solves bin N-1-sg+j, and every active step
// reads the same table column r = T-1-sg) with its push on the fp64 matrix cores.  k_cascade_wf adds
// one column per stage, ACC[rows, steps] += alpha[rows, r+1] T[r+1, steps], a rank-1 update; here the
// columns are pushed in blocks of four, once every four stages, as ACC[rows, steps] += alpha[rows, 4
// columns] . T[4 columns, steps] -- the transfer-matrix x flux-batch GEMM, whose batch is the set of
// redshift steps in flight -- with v_mfma_f64_16x16x4f64 on 16 x 16 tiles (row tile x step tile; C/D
// layout: step = lane & 15, row = (lane >> 4) + 4 reg).  Block q runs at stage 4q and pushes columns
// T-4q .. T-4q+3 (the T_j of stages 4q-1 .. 4q-4) into the rows below T-1-4q, then publishes the four
// rows the chain solves at stages 4q+1 .. 4q+4.  At stage sg the published row therefore lacks the
// columns r+1 .. r+n_u, n_u = sg - 4 ((sg-1) >> 2) in [1, 4]: the chain lane adds them itself from its
// last four T_j and alpha(r, r+k) (staged in LDS), in descending column order.  The matrix core sums
// each block of four columns in its own order, so the fluxes agree with k_cascade_wf to rounding (the
// tests' 1e-11 relative bound vs the oracle, the same exact zeros), not bit for bit.
//
// The waves are specialised, each kind in its own stage loop with one barrier per stage:
//   * push waves (0 .. nw-3) hold the accumulators of 16 RT rows and run only the block pushes;
//   * the flux-independent records (1/Z, the LU of M, the sources) come from a 3-slot ring in LDS,
//     two phases one stage apart: the record wave (nw-2) runs phase 1 (1/Z, M, sources) of stage
//     sg+2, the chain wave (or, R = 2, a wave of its own) phase 2 (the LU) of stage sg+1;
//   * the chain wave (nw-1) solves, lane j = step slot j.
// The registers of one kind's code are not live in another's, so the accumulators do not share a
// budget with the records' temporaries, and the kernel fits 128 VGPRs (4 waves per SIMD).
// Resonant-only points (non_resonant = false) read only alpha(b+i-1, b+i): their chain keeps the
// reference's running sum (nuSIprop.hpp:273-278, 285-287) and the push waves idle.  The DSNB source
// comes from k_source_dsnb's table, the power law is evaluated in the record wave.
//
// R = 1 (RT = 4): one point per workgroup, two workgroups per CU -- two independent chains share
//   a CU instead of one.
// R = 2 (RT = 2): two points that share one Stage-A table (a gamma batch: same m_phi, g, masses
//   and flags; nuSIprop.hpp:217-253 read neither si nor norm) in one workgroup -- the multi-RHS
//   transfer-matrix x flux-batch GEMM.  For fixed tables the cascade is linear in the source (Lum
//   enters only through src, nuSIprop.hpp:283): both points run the same triangular operator, so
//   the records are computed once (one source field per point), each alpha block is loaded once
//   and is the A operand of both points' MFMAs, and the chain lane solves both points' bins (two
//   independent solves that interleave).  groups[k] = (p0, p1); p1 < 0: a single point.
// Every accumulator, published row and solve of a point receives the same operations on the same
// operands whether it runs alone or paired (test_cascade_ws_*: R = 2 equals R = 1 bit for bit).
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
// lane's own solve of bin b+1 (x = F[:, b+1] of this step) -- k_cascade_wf's expression.  sde = dE_b.
NUSI_FN double resonant_add(double& racc, double u0, double u1, double u2, double px0, double px1, double px2,
                            double sj, double sd, double dEb1, double sde, double cj, bool top)
{
    if (!top) racc += (u0 * px0 + u1 * px1 + u2 * px2) * (sj * sd) / dEb1 / sde;
    return cj * racc * sde;
}

// push waves not publishing spread their block MFMAs over the block's stages: k_cascade_wsp yes (C3 cascade
// 37.3 -> 36.0 ms), k_cascade_ws no (C4 0.698 -> 0.728, C5 4.58 -> 4.93 ms; profiles/r2q)
constexpr bool kWsStagger = false, kWspStagger = true;
constexpr int kWsP2Wave = 1;   // R = 2: the LU phase of the records on a wave of its own (nw-3), not the chain (A/B: C5 cascade 5.75 -> 4.49 ms)
template <int R> struct WsCfg;
template <> struct WsCfg<1> { static constexpr int RT = 4, kMaxThreads = 512; };   // 6 push waves + 2
template <> struct WsCfg<2> { static constexpr int RT = 2, kMaxThreads = 832 + 64 * kWsP2Wave; };   // 11 push waves + 2 (3)

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
#define NUSI_WS_STAMP(sg, which)                                                                                   \
    do {                                                                                                           \
        if (which >= 2) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                               \
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (sg) < kTrStages)                                        \
            g_ws_trace[((threadIdx.x >> 6) * kTrStages + (sg)) * 4 + (which)] = __builtin_amdgcn_s_memtime();        \
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
#define NUSI_WS_STAMP(sg, which) do { } while (0)
#define NUSI_BS_STAMP(blk, which) do { } while (0)
#define NUSI_BS_CSTAMP(blk, which) do { } while (0)
#define NUSI_WS_HWID() do { } while (0)
#endif

template <int NJ, int R>
__global__ __launch_bounds__(WsCfg<R>::kMaxThreads) __attribute__((amdgpu_waves_per_eu(4, 4)))
void k_cascade_ws(GridDev g, const Point* __restrict__ pts, const int2* __restrict__ groups, TablesDev t,
                  double* __restrict__ flux, double* __restrict__ flux_fla)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    constexpr int RT = WsCfg<R>::RT, NST = NJ / 16;
    constexpr bool kP2 = R == 2 && kWsP2Wave;   // phase 2 on wave nw-3
    constexpr int FSRC = kWfFields, FM = kWfFields + R - 1, NF = FM + 6;   // other sources; phase-1 M entries
    const int N = g.N, Nz = g.Nz, T = g.T, nst = Nz - 1;
    const int tid = threadIdx.x, nthr = blockDim.x, lane = tid & 63, wave = tid >> 6, nw = nthr >> 6;
    int pid[R];
    bool single = false;
    if (R == 1) {
        pid[0] = blockIdx.x;
    } else {
        const int2 gp = groups[blockIdx.x];
        pid[0] = gp.x;
        pid[R - 1] = gp.y >= 0 ? gp.y : gp.x;
        single = gp.y < 0;
    }
    NUSI_WS_HWID();
    double* F = lds;                         // [R][3][N]
    double* rec = F + 3 * R * N;             // [NF][3][NJ]  records of stage sg in slot sg % 3
    double* Tp = rec + 3 * NF * NJ;          // [R][8][NJ]   T_j by stage (ring of 8)
    double* AX = Tp + 8 * R * NJ;            // [R][2][4][NJ] rows published by block q (parity q & 1)
    double* rdE = AX + 8 * R * NJ;           // [N]
    double* pw = rdE + N;                    // [R][T + 2]
    double* sGt = pw + R * (T + 2);
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
    const Point& P = pts[pid[0]];
    const double* __restrict__ Al = t.A + (size_t)P.tslot * g.PT;
    {
        const double* __restrict__ Gt = t.G + (size_t)P.tslot * T;
        const double* __restrict__ At = t.At + (size_t)P.tslot * T;
        for (int b = tid; b < 3 * R * N; b += nthr) F[b] = 0.0;
        for (int j = tid; j < 16 * R * NJ; j += nthr) Tp[j] = 0.0;   // Tp and AX
        for (int n = tid; n < T; n += nthr) {
            sGt[n] = Gt[n];
            sAt[n] = At[n];
#pragma unroll
            for (int k = 1; k <= 4; ++k) sdg[(k - 1) * T + n] = (n + k < T) ? Al[(size_t)(n + k) * (n + k - 1) / 2 + n] : 0.0;
        }
        for (int b = tid; b < N; b += nthr) { sEmin[b] = g.Emin[b]; sEmax[b] = g.Emax[b]; }
        for (int i = tid; i < Nz; i += nthr) {
            sgz[i] = g.z[i];
            sgz[Nz + i] = g.step_c[i];
            sgz[2 * Nz + i] = g.step_s[i];
            sgz[3 * Nz + i] = g.sfr[i];
        }
        cascade_aux_init(g, P, rdE, pw, tid, nthr);
#pragma unroll
        for (int p = 1; p < R; ++p) {   // the other points' pw[] (cascade_aux_init's expression)
            const double si = pts[pid[p]].si;
            for (int e = tid + 1; e <= T + 1; e += nthr) {
                const int i = min(Nz - 1, max(1, e - N + 1)), b = e - i;
                const double E = (b < N) ? g.Emin[b] : g.Emax[N - 1];
                pw[p * (T + 2) + e] = nm::pow(E / 1e14 * (1 + g.z[i]), -si);
            }
        }
    }
    __syncthreads();
    // records of stage s2 for step slot jj in ring slot s2 % 3 (fields spaced 3 NJ):
    //   phase 1 (record wave): 1/Z, the M entries, the sources of every point, sde
    //   phase 2 (chain wave, one stage later): the LU of M -- cascade_record's operations, split
    constexpr int S3 = 3 * NJ;
    const bool nonres = P.non_resonant;   // the points of a workgroup share a table, hence the flags
    SrcFactors sf[R];   // each point's source factors and kind (the record wave's)
    bool pl[R];
#pragma unroll
    for (int p = 0; p < R; ++p) {
        sf[p] = src_factors(pts[pid[p]]);
        pl[p] = pts[pid[p]].source == NUSI_SOURCE_POWER_LAW;
    }
    auto phase1 = [&](int s2, int jj) {
        const int b = N - 1 - s2 + jj, i = Nz - 1 - jj;
        if (jj < nst && b >= 0 && b < N) {
            double* Rw = rec + (s2 % 3) * NJ + jj;
            const RecM m = record_phase1(gl, P, sGt, sAt, rdE, i, b);
            Rw[PR_RZ0 * S3] = m.rz0;
            Rw[PR_RZ1 * S3] = m.rz1;
            Rw[PR_RZ2 * S3] = m.rz2;
            Rw[(FM + 0) * S3] = m.m01;
            Rw[(FM + 1) * S3] = m.m02;
            Rw[(FM + 2) * S3] = m.m10;
            Rw[(FM + 3) * S3] = m.m12;
            Rw[(FM + 4) * S3] = m.m20;
            Rw[(FM + 5) * S3] = m.m21;
            Rw[PR_SDE * S3] = nonres ? gl.step_s[i] * rdE[b] : (gl.Emax[b] - gl.Emin[b]);
#pragma unroll
            for (int p = 0; p < R; ++p)
                Rw[(p == 0 ? PR_SRC : FSRC + p - 1) * S3] =
                    pl[p] ? powerlaw_src_h(gl, sf[p], pw + p * (T + 2), i, b)
                          : t.Src[(size_t)pid[p] * T * nst + src_index(Nz, jj, b)];
        }
    };
    auto phase2 = [&](int s2, int jj) {
        const int b = N - 1 - s2 + jj;
        if (jj < nst && b >= 0 && b < N) {
            double* Rw = rec + (s2 % 3) * NJ + jj;
            RecM m;
            m.m01 = Rw[(FM + 0) * S3];
            m.m02 = Rw[(FM + 1) * S3];
            m.m10 = Rw[(FM + 2) * S3];
            m.m12 = Rw[(FM + 3) * S3];
            m.m20 = Rw[(FM + 4) * S3];
            m.m21 = Rw[(FM + 5) * S3];
            record_phase2<true>(m, Rw, S3);
        }
    };
    if (wave == nw - 2) {
        phase1(0, lane);
        if (1 < T) phase1(1, lane);
    }
    __syncthreads();
    if (wave == (kP2 ? nw - 3 : nw - 1)) phase2(0, lane);
    __syncthreads();

    // R = 1: phase 2 of stage sg+1 runs on the chain wave (on the top push wave once its rows were consumed, the
    // LU code entered the push branch and spilled its accumulators: C4 cascade 0.706 -> 2.93 ms, profiles/r3/r3f)
    if (wave == nw - 1) {
        // ---- chain: lane j solves (step j, bin N-1-sg+j) of every point at stage sg
        const int j = lane;
        const bool act = j < nst;
        const double u0 = P.u[0], u1 = P.u[1], u2 = P.u[2];
        const double cj = act ? gl.step_c[Nz - 1 - j] : 0.0, sj = act ? gl.step_s[Nz - 1 - j] : 0.0;
        // chain state in registers: px = the lane's last solve (F[:, b+1] of its step, which slot j+1 needs at
        // the next stage and the resonant-only sum reads), Th = its T_j of the last four stages (the columns the
        // published rows still lack); racc = the resonant-only running sum
        double racc[R], px0[R], px1[R], px2[R], Th[R][4];
#pragma unroll
        for (int p = 0; p < R; ++p) {
            racc[p] = px0[p] = px1[p] = px2[p] = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) Th[p][k] = 0.0;
        }
        for (int sg0 = 0; sg0 < T; sg0 += 4)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int sg = sg0 + d;
            if (sg >= T) break;
            NUSI_WS_STAMP(sg, 0);
            const int r = T - 1 - sg;
            const int b = N - 1 - sg + j;
            // F[:, b] of this step = slot j-1's solve of bin b at stage sg-1 (slot 0: the initial flux, 0)
            double f0[R], f1[R], f2[R];
#pragma unroll
            for (int p = 0; p < R; ++p) {
                f0[p] = wave_shr1(px0[p], 0.0);
                f1[p] = wave_shr1(px1[p], 0.0);
                f2[p] = wave_shr1(px2[p], 0.0);
            }
            double Tn[R];
#pragma unroll
            for (int p = 0; p < R; ++p) Tn[p] = 0.0;
            if (!kP2 && sg + 1 < T) phase2(sg + 1, j);   // independent of this stage's solve
            if (act && b >= 0 && b < N) {
                const double* Rc = rec + (sg % 3) * NJ + j;
                constexpr int S = S3;
                const double rz0 = Rc[PR_RZ0 * S], rz1 = Rc[PR_RZ1 * S], rz2 = Rc[PR_RZ2 * S];
                const int pmb = (int)Rc[kPreFields * S];
                const double l10 = Rc[PR_L10 * S], l20 = Rc[PR_L20 * S], l21 = Rc[PR_L21 * S];
                const double u01 = Rc[PR_U01 * S], u02 = Rc[PR_U02 * S], u12 = Rc[PR_U12 * S];
                const double ru00 = Rc[PR_RU00 * S], ru11 = Rc[PR_RU11 * S], ru22 = Rc[PR_RU22 * S];
                const double sde = Rc[PR_SDE * S];
                double srcv[R];
#pragma unroll
                for (int p = 0; p < R; ++p) srcv[p] = Rc[(p == 0 ? PR_SRC : FSRC + p - 1) * S];
                double add[R];   // c_i x (coupling of the bin to the bins above)
                if (nonres) {
                    const int qq = (sg - 1) >> 2;              // block whose publication serves stage sg
                    const int nu = (d == 0) ? 4 : d;           // columns r+1 .. r+nu not yet pushed
                    const int ax = ((qq & 1) * 4 + (sg - 1 - 4 * qq)) * NJ + j;
                    double s[R];
#pragma unroll
                    for (int p = 0; p < R; ++p) s[p] = AX[p * 8 * NJ + ax];
#pragma unroll
                    for (int k = 4; k >= 1; --k)
                        if (k <= nu) {
                            const double a = sdg[(k - 1) * T + r];
#pragma unroll
                            for (int p = 0; p < R; ++p) s[p] = fma(a, Th[p][k - 1], s[p]);
                        }
#pragma unroll
                    for (int p = 0; p < R; ++p) add[p] = cj * s[p];
                } else {
                    const double dEb1 = (b + 1 < N) ? sEmax[b + 1] - sEmin[b + 1] : 1.0;
#pragma unroll
                    for (int p = 0; p < R; ++p)
                        add[p] = resonant_add(racc[p], u0, u1, u2, px0[p], px1[p], px2[p], sj, sdg[r], dEb1, sde, cj,
                                              b == N - 1);
                }
                NUSI_WS_STAMP(sg, 2);
#pragma unroll
                for (int p = 0; p < R; ++p) {
                    double* Fp = F + 3 * N * p;
                    double x0, x1, x2;
                    cascade_solve(f0[p], f1[p], f2[p], add[p], srcv[p], u0, u1, u2, rz0, rz1, rz2, pmb, l10, l20, l21, u01,
                                  u02, u12, ru00, ru11, ru22, x0, x1, x2);
                    if (j == nst - 1) {   // the last step's flux (finalisation)
                        Fp[b] = x0;
                        Fp[N + b] = x1;
                        Fp[2 * N + b] = x2;
                    }
                    px0[p] = x0; px1[p] = x1; px2[p] = x2;
                    if (nonres && b > 0) Tn[p] = (u0 * x0 + u1 * x1 + u2 * x2) * sde;
                }
            }
            NUSI_WS_STAMP(sg, 3);
#pragma unroll
            for (int p = 0; p < R; ++p) {
                Th[p][3] = Th[p][2]; Th[p][2] = Th[p][1]; Th[p][1] = Th[p][0]; Th[p][0] = Tn[p];
            }
            if (act)
#pragma unroll
                for (int p = 0; p < R; ++p) Tp[(p * 8 + (sg & 7)) * NJ + j] = Tn[p];
            NUSI_WS_STAMP(sg, 1);
            __syncthreads();
        }
    } else if (kP2 && wave == nw - 3) {
        for (int sg = 0; sg < T; ++sg) {
            NUSI_WS_STAMP(sg, 0);
            if (sg + 1 < T) phase2(sg + 1, lane);
            NUSI_WS_STAMP(sg, 1);
            __syncthreads();
        }
    } else if (wave == nw - 2) {
        // ---- phase 1 of the records two stages ahead, while the chain solves this stage
        for (int sg = 0; sg < T; ++sg) {
            NUSI_WS_STAMP(sg, 0);
            if (sg + 2 < T) phase1(sg + 2, lane);
            NUSI_WS_STAMP(sg, 1);
            __syncthreads();
        }
    } else {
        // ---- push: block q (stage 4q) adds columns T-4q .. T-4q+3 (the T of stages 4q-1 .. 4q-4) into the
        // rows below r = T-1-4q, then publishes rows r-1 .. r-4 (the rows of stages 4q+1 .. 4q+4)
        const int rw0 = wave * 16 * RT;
        nusi_f64x4 acc[R][RT][NST];
#pragma unroll
        for (int p = 0; p < R; ++p)
#pragma unroll
            for (int a = 0; a < RT; ++a)
#pragma unroll
                for (int s = 0; s < NST; ++s) acc[p][a][s] = nusi_f64x4{0.0, 0.0, 0.0, 0.0};
        // A operands: alpha(row, column), row = tile row + (lane & 15), column = first block column + (lane >> 4);
        // rows clamped into the column (those rows are consumed)
        auto load_blk = [&](int q, double (&dst)[RT]) {
            int c = T - 4 * q + (lane >> 4);
            c = c < 1 ? 1 : (c > T - 1 ? T - 1 : c);
            const size_t cb = (size_t)c * (c - 1) / 2;
#pragma unroll
            for (int a = 0; a < RT; ++a) {
                const int row = rw0 + 16 * a + (lane & 15);
                dst[a] = Al[cb + (row < c - 1 ? row : c - 1)];
            }
        };
        double ablk[RT];
        load_blk(1, ablk);
        for (int sg = 0; sg < T; ++sg) {
            NUSI_WS_STAMP(sg, 0);
            // block q is pushed at stage 4q by the waves holding the rows it publishes, and one to three
            // stages later by the others (their rows are needed >= 5 stages on; the T_j ring keeps 8):
            // the matrix-core work of a block is spread over its four stages (kWsStagger)
            const int q = sg >> 2, r = T - 1 - 4 * q, hi = r - 1;
            const bool crit = rw0 <= hi && rw0 + 16 * RT - 1 >= hi - 3;
            const int dw = (!kWsStagger || crit) ? 0 : 1 + wave % 3;
            if ((sg & 3) == dw && nonres) {
                if (q >= 1) {
#pragma unroll
                    for (int s = 0; s < NST; ++s) {
                        const int bi = ((4 * q - 1 - (lane >> 4)) & 7) * NJ + 16 * s + (lane & 15);
                        double bop[R];
#pragma unroll
                        for (int p = 0; p < R; ++p) bop[p] = Tp[p * 8 * NJ + bi];
#pragma unroll
                        for (int a = 0; a < RT; ++a)
                            if (rw0 + 16 * a < r)   // tiles wholly at or above r hold consumed rows only
#pragma unroll
                                for (int p = 0; p < R; ++p)
                                    acc[p][a][s] = __builtin_amdgcn_mfma_f64_16x16x4f64(ablk[a], bop[p], acc[p][a][s], 0, 0, 0);
                    }
                    load_blk(q + 1, ablk);
                }
            }
            if ((sg & 3) == 0 && nonres) {
#pragma unroll
                for (int a = 0; a < RT; ++a)
                    if (rw0 + 16 * a <= hi && rw0 + 16 * a + 15 >= hi - 3)   // uniform: tiles holding those rows
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int row = rw0 + 16 * a + (lane >> 4) + 4 * e;
                            const int slot = hi - row;
                            if (slot >= 0 && slot < 4)
#pragma unroll
                                for (int s = 0; s < NST; ++s) {
                                    const int o = ((q & 1) * 4 + slot) * NJ + 16 * s + (lane & 15);
#pragma unroll
                                    for (int p = 0; p < R; ++p) AX[p * 8 * NJ + o] = acc[p][a][s][e];
                                }
                        }
            }
            NUSI_WS_STAMP(sg, 1);
            __syncthreads();
        }
    }
    // finalise (nuSIprop.hpp:328-336)
#pragma unroll
    for (int p = 0; p < R; ++p) {
        if (p > 0 && single) break;
        const Point& Q = pts[pid[p]];
        const double* Fp = F + 3 * N * p;
        double* fo = flux + (size_t)pid[p] * 3 * N;
        double* fl = flux_fla + (size_t)pid[p] * 3 * N;
        for (int b = tid; b < N; b += nthr) {
            const double dE = g.Emax[b] - g.Emin[b];
            const double f0 = Fp[b] / dE, f1 = Fp[N + b] / dE, f2 = Fp[2 * N + b] / dE;
            fo[b] = f0;
            fo[N + b] = f1;
            fo[2 * N + b] = f2;
            for (int f = 0; f < 3; ++f) fl[f * N + b] = Q.U2[3 * f + 0] * f0 + Q.U2[3 * f + 1] * f1 + Q.U2[3 * f + 2] * f2;
        }
    }
}

// ---------------------------------------------------------------------------
// Step passes: k_cascade_ws for grids with more redshift steps than the slots in flight (e.g.
// BASELINE C3: N = 1200, 134 steps).
//
// The wavefront keeps every step in flight, and its accumulators (T-1 rows x steps) outgrow a CU's
// registers.  The steps are therefore taken NJ = 16 at a time: pass p runs the wavefront of step
// slots [16 p, 16 p + 16) over N + 15 stages, its local stage 0 reading table column T-1-16p (along
// a stage b + i is constant within the pass as before).  F[3][N] stays in LDS from pass to pass --
// the first step of pass p starts from the last step of pass p-1, as step i starts from step i+1 in
// the reference's loop (nuSIprop.hpp:257-315) -- and the accumulators, the T_j ring and the
// published rows restart from zero.  Each pass reads its columns once (the table is read
// ceil(steps / 16) times).  Push waves own 16 RT = 128 rows; phase 2 of the records has a wave of
// its own.  Everything else -- records, solves, the rank-4 MFMA push -- is k_cascade_ws<NJ, 1>'s code;
// one pass (steps <= 16) gives that kernel's fluxes bit for bit (test_cascade_step_passes).  The body
// is a separate kernel rather than a mode of k_cascade_ws because the 48-slot instantiation of that
// kernel sits on the 128-VGPR edge and spills as soon as its code changes shape.
// ---------------------------------------------------------------------------
constexpr int kWsBigNJ = 16, kWsBigRT = 8;   // step slots per pass, 16-row tiles per push wave

// kNR: every point of the launch is non-resonant (the launcher checks), so the resonant-only chain code is not
// compiled in (C3 cascade 38.9 -> 37.3 ms, profiles/r3/r3w)
template <int NJ, bool kNR>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 4)))
void k_cascade_wsp(GridDev g, const Point* __restrict__ pts, TablesDev t, double* __restrict__ flux,
                   double* __restrict__ flux_fla)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    constexpr int R = 1, RT = kWsBigRT, NST = NJ / 16;
    constexpr bool kP2 = kWsP2Wave;   // phase 2 on wave nw-3
    constexpr int FSRC = kWfFields, FM = kWfFields + R - 1, NF = FM + 6;   // other sources; phase-1 M entries
    const int N = g.N, Nz = g.Nz, T = g.T, nst = Nz - 1;
    const int tid = threadIdx.x, nthr = blockDim.x, lane = tid & 63, wave = tid >> 6, nw = nthr >> 6;
    const int pid[R] = {(int)blockIdx.x};   // one point per workgroup
    constexpr bool single = true;
    double* F = lds;                         // [R][3][N]
    double* rec = F + 3 * R * N;             // [NF][3][NJ]  records of stage sg in slot sg % 3
    double* Tp = rec + 3 * NF * NJ;          // [R][8][NJ]   T_j by stage (ring of 8)
    double* AX = Tp + 8 * R * NJ;            // [R][2][4][NJ] rows published by block q (parity q & 1)
    double* rdE = AX + 8 * R * NJ;           // [N]
    double* pw = rdE + N;                    // [R][T + 2]
    double* sGt = pw + R * (T + 2);
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
    const Point& P = pts[pid[0]];
    const double* __restrict__ Al = t.A + (size_t)P.tslot * g.PT;
    {
        const double* __restrict__ Gt = t.G + (size_t)P.tslot * T;
        const double* __restrict__ At = t.At + (size_t)P.tslot * T;
        for (int b = tid; b < 3 * R * N; b += nthr) F[b] = 0.0;
        for (int j = tid; j < 16 * R * NJ; j += nthr) Tp[j] = 0.0;   // Tp and AX
        for (int n = tid; n < T; n += nthr) {
            sGt[n] = Gt[n];
            sAt[n] = At[n];
#pragma unroll
            for (int k = 1; k <= 4; ++k) sdg[(k - 1) * T + n] = (n + k < T) ? Al[(size_t)(n + k) * (n + k - 1) / 2 + n] : 0.0;
        }
        for (int b = tid; b < N; b += nthr) { sEmin[b] = g.Emin[b]; sEmax[b] = g.Emax[b]; }
        for (int i = tid; i < Nz; i += nthr) {
            sgz[i] = g.z[i];
            sgz[Nz + i] = g.step_c[i];
            sgz[2 * Nz + i] = g.step_s[i];
            sgz[3 * Nz + i] = g.sfr[i];
        }
        cascade_aux_init(g, P, rdE, pw, tid, nthr);
#pragma unroll
        for (int p = 1; p < R; ++p) {   // the other points' pw[] (cascade_aux_init's expression)
            const double si = pts[pid[p]].si;
            for (int e = tid + 1; e <= T + 1; e += nthr) {
                const int i = min(Nz - 1, max(1, e - N + 1)), b = e - i;
                const double E = (b < N) ? g.Emin[b] : g.Emax[N - 1];
                pw[p * (T + 2) + e] = nm::pow(E / 1e14 * (1 + g.z[i]), -si);
            }
        }
    }
    __syncthreads();
    // records of stage s2 for step slot jj in ring slot s2 % 3 (fields spaced 3 NJ):
    //   phase 1 (record wave): 1/Z, the M entries, the sources of every point, sde
    //   phase 2 (chain wave, one stage later): the LU of M -- cascade_record's operations, split
    constexpr int S3 = 3 * NJ;
    int jb = 0;   // first step slot of the current pass (step i = Nz-1-jb-j for slot j)
    const bool nonres = kNR || P.non_resonant;
    auto phase1 = [&](int s2, int jj) {
        const int b = N - 1 - s2 + jj, i = Nz - 1 - jb - jj;
        if (jj < NJ && jb + jj < nst && b >= 0 && b < N) {
            double* Rw = rec + (s2 % 3) * NJ + jj;
            const RecM m = record_phase1(gl, P, sGt, sAt, rdE, i, b);
            Rw[PR_RZ0 * S3] = m.rz0;
            Rw[PR_RZ1 * S3] = m.rz1;
            Rw[PR_RZ2 * S3] = m.rz2;
            Rw[(FM + 0) * S3] = m.m01;
            Rw[(FM + 1) * S3] = m.m02;
            Rw[(FM + 2) * S3] = m.m10;
            Rw[(FM + 3) * S3] = m.m12;
            Rw[(FM + 4) * S3] = m.m20;
            Rw[(FM + 5) * S3] = m.m21;
            Rw[PR_SDE * S3] = nonres ? gl.step_s[i] * rdE[b] : (gl.Emax[b] - gl.Emin[b]);
#pragma unroll
            for (int p = 0; p < R; ++p) {   // (the point's factors per record: hoisted they cost the kernel registers)
                const Point& Q = pts[pid[p]];
                Rw[(p == 0 ? PR_SRC : FSRC + p - 1) * S3] =
                    Q.source == NUSI_SOURCE_POWER_LAW ? powerlaw_src(gl, Q, pw + p * (T + 2), i, b)
                                                      : t.Src[(size_t)pid[p] * T * nst + src_index(Nz, jb + jj, b)];
            }
        }
    };
    auto phase2 = [&](int s2, int jj) {
        const int b = N - 1 - s2 + jj;
        if (jj < NJ && jb + jj < nst && b >= 0 && b < N) {
            double* Rw = rec + (s2 % 3) * NJ + jj;
            RecM m;
            m.m01 = Rw[(FM + 0) * S3];
            m.m02 = Rw[(FM + 1) * S3];
            m.m10 = Rw[(FM + 2) * S3];
            m.m12 = Rw[(FM + 3) * S3];
            m.m20 = Rw[(FM + 4) * S3];
            m.m21 = Rw[(FM + 5) * S3];
            record_phase2<true>(m, Rw, S3);
        }
    };
    const int npass = (nst + NJ - 1) / NJ;
#pragma unroll 1
    for (int pass = 0; pass < npass; ++pass) {
    jb = pass * NJ;
    const int Ts = N - 1 + (nst - jb < NJ ? nst - jb : NJ);   // stages of this pass
    const int c0 = T - 1 - jb;                                 // the table column of local stage 0
    if (pass > 0) {   // accumulators, T_j ring and published rows restart; F carries over
        __syncthreads();
        for (int j = tid; j < 16 * R * NJ; j += nthr) Tp[j] = 0.0;
        __syncthreads();
    }
    if (wave == nw - 2) {
        phase1(0, lane);
        if (1 < Ts) phase1(1, lane);
    }
    __syncthreads();
    if (wave == (kP2 ? nw - 3 : nw - 1)) phase2(0, lane);
    __syncthreads();

    if (wave == nw - 1) {
        // ---- chain: lane j solves (step jb+j, bin N-1-sg+j) of every point at stage sg
        const int j = lane;
        const bool act = j < NJ && jb + j < nst;
        const double u0 = P.u[0], u1 = P.u[1], u2 = P.u[2];
        const double cj = act ? gl.step_c[Nz - 1 - jb - j] : 0.0, sj = act ? gl.step_s[Nz - 1 - jb - j] : 0.0;
        // chain state: F[:, b] is updated in place in LDS (slot j reads slot j-1's solve of the previous stage),
        // the T_j of the last four stages come from the Tp ring.  (k_cascade_ws keeps both in registers -- a DPP
        // shift and a per-lane history; here that spilled loop invariants of the chain to scratch and the C3
        // cascade took 49.7 instead of 38.7 ms, profiles/r3/r3g.)
        double racc[R], px0[R], px1[R], px2[R];   // resonant-only chain state (per step: restarts every pass)
#pragma unroll
        for (int p = 0; p < R; ++p) racc[p] = px0[p] = px1[p] = px2[p] = 0.0;
        for (int sg0 = 0; sg0 < Ts; sg0 += 4)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int sg = sg0 + d;
            if (sg >= Ts) break;
            const int r = c0 - sg;
            const int b = N - 1 - sg + j;
            double Tn[R];
#pragma unroll
            for (int p = 0; p < R; ++p) Tn[p] = 0.0;
            if (!kP2 && sg + 1 < Ts) phase2(sg + 1, j);   // independent of this stage's solve
            if (act && b >= 0 && b < N) {
                const double* Rc = rec + (sg % 3) * NJ + j;
                constexpr int S = S3;
                const double rz0 = Rc[PR_RZ0 * S], rz1 = Rc[PR_RZ1 * S], rz2 = Rc[PR_RZ2 * S];
                const int pmb = (int)Rc[kPreFields * S];
                const double l10 = Rc[PR_L10 * S], l20 = Rc[PR_L20 * S], l21 = Rc[PR_L21 * S];
                const double u01 = Rc[PR_U01 * S], u02 = Rc[PR_U02 * S], u12 = Rc[PR_U12 * S];
                const double ru00 = Rc[PR_RU00 * S], ru11 = Rc[PR_RU11 * S], ru22 = Rc[PR_RU22 * S];
                const double sde = Rc[PR_SDE * S];
                double add[R];
                if (nonres) {
                    const int qq = (sg - 1) >> 2;              // block whose publication serves stage sg
                    const int nu = (d == 0) ? 4 : d;           // columns r+1 .. r+nu not yet pushed
                    const int ax = ((qq & 1) * 4 + (sg - 1 - 4 * qq)) * NJ + j;
                    double s[R];
#pragma unroll
                    for (int p = 0; p < R; ++p) s[p] = AX[p * 8 * NJ + ax];
#pragma unroll
                    for (int k = 4; k >= 1; --k)
                        if (k <= nu) {
                            const double a = sdg[(k - 1) * T + r];
#pragma unroll
                            for (int p = 0; p < R; ++p) s[p] = fma(a, Tp[(p * 8 + ((sg - k) & 7)) * NJ + j], s[p]);
                        }
#pragma unroll
                    for (int p = 0; p < R; ++p) add[p] = cj * s[p];
                } else {
                    const double dEb1 = (b + 1 < N) ? sEmax[b + 1] - sEmin[b + 1] : 1.0;
#pragma unroll
                    for (int p = 0; p < R; ++p)
                        add[p] = resonant_add(racc[p], u0, u1, u2, px0[p], px1[p], px2[p], sj, sdg[r], dEb1, sde, cj,
                                              b == N - 1);
                }
#pragma unroll
                for (int p = 0; p < R; ++p) {
                    double* Fp = F + 3 * N * p;
                    const double src = Rc[(p == 0 ? PR_SRC : FSRC + p - 1) * S];
                    double x0, x1, x2;
                    cascade_solve(Fp[b], Fp[N + b], Fp[2 * N + b], add[p], src, u0, u1, u2, rz0, rz1, rz2, pmb, l10,
                                  l20, l21, u01, u02, u12, ru00, ru11, ru22, x0, x1, x2);
                    Fp[b] = x0;
                    Fp[N + b] = x1;
                    Fp[2 * N + b] = x2;
                    px0[p] = x0; px1[p] = x1; px2[p] = x2;
                    if (nonres && b > 0) Tn[p] = (u0 * x0 + u1 * x1 + u2 * x2) * sde;
                }
            }
            if (act)
#pragma unroll
                for (int p = 0; p < R; ++p) Tp[(p * 8 + (sg & 7)) * NJ + j] = Tn[p];
            __syncthreads();
        }
    } else if (kP2 && wave == nw - 3) {
        for (int sg = 0; sg < Ts; ++sg) {
            if (sg + 1 < Ts) phase2(sg + 1, lane);
            __syncthreads();
        }
    } else if (wave == nw - 2) {
        // ---- phase 1 of the records two stages ahead, while the chain solves this stage
        for (int sg = 0; sg < Ts; ++sg) {
            if (sg + 2 < Ts) phase1(sg + 2, lane);
            __syncthreads();
        }
    } else {
        // ---- push: block q (stage 4q) adds columns c0+1-4q .. c0+4-4q (the T of stages 4q-1 .. 4q-4) into
        // the rows below r = c0-4q, then publishes rows r-1 .. r-4 (the rows of stages 4q+1 .. 4q+4)
        const int rw0 = wave * 16 * RT;
        nusi_f64x4 acc[R][RT][NST];
#pragma unroll
        for (int p = 0; p < R; ++p)
#pragma unroll
            for (int a = 0; a < RT; ++a)
#pragma unroll
                for (int s = 0; s < NST; ++s) acc[p][a][s] = nusi_f64x4{0.0, 0.0, 0.0, 0.0};
        // A operands: alpha(row, column), row = tile row + (lane & 15), column = first block column + (lane >> 4);
        // rows clamped into the column (those rows are consumed)
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
        double ablk[RT];
        load_blk(1, ablk);
        for (int sg = 0; sg < Ts; ++sg) {
            // block q is pushed at stage 4q by the waves holding the rows it publishes, and one to three
            // stages later by the others (their rows are needed >= 5 stages on; the T_j ring keeps 8):
            // the matrix-core work of a block is spread over its four stages (kWspStagger)
            const int q = sg >> 2, r = c0 - 4 * q, hi = r - 1;
            const bool crit = rw0 <= hi && rw0 + 16 * RT - 1 >= hi - 3;
            const int dw = (!kWspStagger || crit) ? 0 : 1 + wave % 3;
            if ((sg & 3) == dw && nonres) {
                if (q >= 1) {
#pragma unroll
                    for (int s = 0; s < NST; ++s) {
                        const int bi = ((4 * q - 1 - (lane >> 4)) & 7) * NJ + 16 * s + (lane & 15);
                        double bop[R];
#pragma unroll
                        for (int p = 0; p < R; ++p) bop[p] = Tp[p * 8 * NJ + bi];
#pragma unroll
                        for (int a = 0; a < RT; ++a)
                            if (rw0 + 16 * a < r)   // tiles wholly at or above r hold consumed rows only
#pragma unroll
                                for (int p = 0; p < R; ++p)
                                    acc[p][a][s] = __builtin_amdgcn_mfma_f64_16x16x4f64(ablk[a], bop[p], acc[p][a][s], 0, 0, 0);
                    }
                    load_blk(q + 1, ablk);
                }
            }
            if ((sg & 3) == 0 && nonres) {
#pragma unroll
                for (int a = 0; a < RT; ++a)
                    if (rw0 + 16 * a <= hi && rw0 + 16 * a + 15 >= hi - 3)   // uniform: tiles holding those rows
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int row = rw0 + 16 * a + (lane >> 4) + 4 * e;
                            const int slot = hi - row;
                            if (slot >= 0 && slot < 4)
#pragma unroll
                                for (int s = 0; s < NST; ++s) {
                                    const int o = ((q & 1) * 4 + slot) * NJ + 16 * s + (lane & 15);
#pragma unroll
                                    for (int p = 0; p < R; ++p) AX[p * 8 * NJ + o] = acc[p][a][s][e];
                                }
                        }
            }
            __syncthreads();
        }
    }
    }   // passes
    __syncthreads();   // the last pass's solves are in F
    // finalise (nuSIprop.hpp:328-336)
#pragma unroll
    for (int p = 0; p < R; ++p) {
        if (p > 0 && single) break;
        const Point& Q = pts[pid[p]];
        const double* Fp = F + 3 * N * p;
        double* fo = flux + (size_t)pid[p] * 3 * N;
        double* fl = flux_fla + (size_t)pid[p] * 3 * N;
        for (int b = tid; b < N; b += nthr) {
            const double dE = g.Emax[b] - g.Emin[b];
            const double f0 = Fp[b] / dE, f1 = Fp[N + b] / dE, f2 = Fp[2 * N + b] / dE;
            fo[b] = f0;
            fo[N + b] = f1;
            fo[2 * N + b] = f2;
            for (int f = 0; f < 3; ++f) fl[f * N + b] = Q.U2[3 * f + 0] * f0 + Q.U2[3 * f + 1] * f1 + Q.U2[3 * f + 2] * f2;
        }
    }
}

// ---------------------------------------------------------------------------
// k_cascade_gb: the gamma batch -- the north star's transfer-matrix x flux-batch GEMM at full batch width
// (SURVEY.md sec. 7 K_B').  For fixed tables the cascade is linear in the source, and the source is the only
// input that depends on gamma (Lum enters through src alone, nuSIprop.hpp:283; the power law :656): the up to 16
// points of a table slot (C5: the 16 gamma of one (m_phi, g)) share one triangular operator.  One workgroup takes
// all of them, gamma on the N dimension of v_mfma_f64_16x16x4f64:
//     ACC_j[16 rows, 16 gamma] += alpha[16 rows, 4 columns] . T_j[4 columns, 16 gamma]     (per row tile, step j)
// so each alpha block is loaded once for every point, and the records (1/Z, M and its LU, nuSIprop.hpp:289-310)
// are formed once per (step, bin) for all of them.  The accumulator state is rows x steps x gamma, so the steps
// are taken kGbNJ = 6 at a time, k_cascade_wsp's passes: 6 x 16 = 96 columns per CU, as the R = 2 kernel's 2 x 48.
//   * push waves: 16 kGbRT rows each, acc[RT][NJ] tiles, the block pushes of k_cascade_ws at stages 4q;
//   * two chain waves, lane = 3 p + jj (point p < 16, step jj of the wave's three): step j hands its solve to
//     j + 1 by a wave shift (DPP), across the two waves through LDS (hb), and across passes through a global FIFO
//     of the last step's F[:, b] (fh, loaded with non-temporal loads four stages ahead);
//   * the record wave: phase 1 / phase 2 of the records two / one stage ahead (6 lanes), and per point the power
//     law's pw at the stage's lower table edge (one exp per point and stage: along a stage b + i is constant, so
//     every step of the stage reads the same two edges; exp(-si log x) = nm::pow, the same bits as pw[]).
// Power-law points only (the DSNB source does not depend on gamma).  The solves and pushes are k_cascade_ws's
// operations on the same operands, so the fluxes agree with it to rounding (the MFMA sums a block in its own
// order; tests: test_cascade_gamma_batch, FLUX_RTOL against the oracle and the R = 1 kernel).
// ---------------------------------------------------------------------------
constexpr int kGbNJ = 6, kGbRT = 2, kGbSPW = 3, kGbChainWaves = kGbNJ / kGbSPW;
constexpr int kGbNF = kWfFields + 6;   // record fields + the phase-1 M entries
static_assert(kGbNJ % kGbSPW == 0 && 16 * kGbSPW <= 64, "chain lanes");

template <int NJ>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 4)))
void k_cascade_gb(GridDev g, const Point* __restrict__ pts, const int* __restrict__ gidx, const int2* __restrict__ grp,
                  TablesDev t, double* __restrict__ fh, double* __restrict__ flux, double* __restrict__ flux_fla)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    constexpr int RT = kGbRT, NF = kGbNF, FM = kWfFields, S3 = 3 * NJ;
    const int N = g.N, Nz = g.Nz, T = g.T, nst = Nz - 1;
    const int tid = threadIdx.x, nthr = blockDim.x, lane = tid & 63, wave = tid >> 6, nw = nthr >> 6;
    const int nwp = nw - kGbChainWaves - 2, recw = nw - 2;   // push waves, the chain waves, the two record waves
    const int2 gr = grp[blockIdx.x];
    const int R = gr.y;                                      // points of this workgroup (<= 16), one table
    const Point& P = pts[gidx[gr.x]];
    double* rec = lds;                       // [3][NF][NJ]     records of stage s in slot s % 3
    double* Tp = rec + 3 * NF * NJ;          // [8][NJ][16]     T_j of each point by stage
    double* AX = Tp + 8 * NJ * 16;           // [2][4][NJ][16]  rows published by block q (parity q & 1)
    double* hb = AX + 8 * NJ * 16;           // [2][3][16]      chain wave 0's top step -> wave 1 (stage parity)
    double* rdE = hb + 96;                   // [N]
    double* pw = rdE + N;                    // [T + 2][16]     each point's pw on table edge e (cascade_aux_init's)
    double* sGt = pw + 16 * (T + 2);
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
    const double* __restrict__ Al = t.A + (size_t)P.tslot * g.PT;
    {
        const double* __restrict__ Gt = t.G + (size_t)P.tslot * T;
        const double* __restrict__ At = t.At + (size_t)P.tslot * T;
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
        for (int q = tid; q < 16 * (T + 1); q += nthr) {   // cascade_aux_init's pw[e] of every point
            const int e = 1 + q / 16, p = q - 16 * (q / 16);
            if (p >= R) continue;
            const int i = min(Nz - 1, max(1, e - N + 1)), b = e - i;
            const double E = (b < N) ? g.Emin[b] : g.Emax[N - 1];
            pw[e * 16 + p] = nm::pow(E / 1e14 * (1 + g.z[i]), -pts[gidx[gr.x + p]].si);
        }
    }
    const bool nonres = P.non_resonant;
    int jb = 0;   // first step slot of the current pass (step i = Nz-1-jb-j for slot j)
    auto phase1 = [&](int s2, int jj) {
        const int b = N - 1 - s2 + jj, i = Nz - 1 - jb - jj;
        if (jj < NJ && jb + jj < nst && b >= 0 && b < N) {
            double* Rw = rec + (s2 % 3) * NJ + jj;
            const RecM m = record_phase1(gl, P, sGt, sAt, rdE, i, b);
            Rw[PR_RZ0 * S3] = m.rz0;
            Rw[PR_RZ1 * S3] = m.rz1;
            Rw[PR_RZ2 * S3] = m.rz2;
            Rw[(FM + 0) * S3] = m.m01;
            Rw[(FM + 1) * S3] = m.m02;
            Rw[(FM + 2) * S3] = m.m10;
            Rw[(FM + 3) * S3] = m.m12;
            Rw[(FM + 4) * S3] = m.m20;
            Rw[(FM + 5) * S3] = m.m21;
            Rw[PR_SDE * S3] = nonres ? gl.step_s[i] * rdE[b] : (gl.Emax[b] - gl.Emin[b]);
        }
    };
    auto phase2 = [&](int s2, int jj) {
        const int b = N - 1 - s2 + jj;
        if (jj < NJ && jb + jj < nst && b >= 0 && b < N) {
            double* Rw = rec + (s2 % 3) * NJ + jj;
            RecM m;
            m.m01 = Rw[(FM + 0) * S3];
            m.m02 = Rw[(FM + 1) * S3];
            m.m10 = Rw[(FM + 2) * S3];
            m.m12 = Rw[(FM + 3) * S3];
            m.m20 = Rw[(FM + 4) * S3];
            m.m21 = Rw[(FM + 5) * S3];
            record_phase2<true>(m, Rw, S3);
        }
    };
    // Every role runs the passes in its own loop (one loop around the role branches made the compiler spill the
    // push waves' accumulators), with the same barriers: pass start, records 0/1 written, record 0 complete, then
    // one per stage.
    const int npass = (nst + NJ - 1) / NJ;
    auto pass_geom = [&](int pass, int& njp, int& Ts, int& c0) {
        jb = pass * NJ;
        njp = nst - jb < NJ ? nst - jb : NJ;   // steps of this pass
        Ts = N - 1 + njp;                      // its stages
        c0 = T - 1 - jb;                       // the table column of its stage 0
    };
    auto pass_head = [&]() {   // the barriers and shared set-up every role runs at a pass start
        __syncthreads();       // (the previous pass is done with Tp, AX, hb and the records)
        for (int q = tid; q < 16 * NJ * 16; q += nthr) Tp[q] = 0.0;   // Tp and AX
    };
    if (wave >= nwp && wave < nwp + kGbChainWaves) {
        // ---- chain: lane (cp, cjj) of wave cw solves (step jb + j, bin N-1-sg+j) of point cp, j = 3 cw + cjj
        const int cw = wave - nwp, cp = lane / kGbSPW, cjj = lane - kGbSPW * (lane / kGbSPW);
        const bool clane = lane < 16 * kGbSPW && cp < R;
        const int cpid = clane ? gidx[gr.x + cp] : 0;
        const SrcFactors csf = clane ? src_factors(pts[cpid]) : SrcFactors{0.0, 0.0};
        double* const fhw = fh + (size_t)blockIdx.x * 3 * N * 16;   // this workgroup's F FIFO [3][N][16]
        const int j = kGbSPW * cw + cjj;
        const double u0 = P.u[0], u1 = P.u[1], u2 = P.u[2];
#pragma unroll 1
        for (int pass = 0; pass < npass; ++pass) {
            int njp, Ts, c0;
            pass_geom(pass, njp, Ts, c0);
            const bool last_pass = pass == npass - 1;
            pass_head();
            __syncthreads();
            __syncthreads();
            const bool act = clane && j < njp;
            const int i = Nz - 1 - jb - j;
            const double cj = act ? gl.step_c[i] : 0.0, sj = act ? gl.step_s[i] : 0.0, sfr = act ? gl.sfr[i] : 0.0;
            const bool top = j == njp - 1;   // the pass's last step: its solves feed the next pass or the output
            double racc = 0.0, px0 = 0.0, px1 = 0.0, px2 = 0.0, Th[4] = {0.0, 0.0, 0.0, 0.0};
            // slot 0 of wave 0 after the first pass: F[:, b] of the previous pass' last step from the FIFO, two
            // stages ahead (non-temporal: the FIFO's lines were rewritten since an earlier pass read them)
            const bool ffifo = pass > 0 && cw == 0 && cjj == 0 && clane;
            double fq0[2], fq1[2], fq2[2];
#pragma unroll
            for (int d = 0; d < 2; ++d) {
                fq0[d] = fq1[d] = fq2[d] = 0.0;
                const int bq = N - 1 - d;
                if (ffifo && d < Ts && bq >= 0) {
                    fq0[d] = __builtin_nontemporal_load(fhw + (0 * N + bq) * 16 + cp);
                    fq1[d] = __builtin_nontemporal_load(fhw + (1 * N + bq) * 16 + cp);
                    fq2[d] = __builtin_nontemporal_load(fhw + (2 * N + bq) * 16 + cp);
                }
            }
            for (int sg0 = 0; sg0 < Ts; sg0 += 4)
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const int sg = sg0 + d;
                if (sg >= Ts) break;
                NUSI_WS_STAMP(sg, 0);
                const int r = c0 - sg;
                const int b = N - 1 - sg + j;
                // F[:, b] of this step: step j-1's solve of bin b at stage sg-1 (the lane below; for the wave's
                // first step the other wave's top step through hb, or the previous pass through the FIFO)
                double f0 = wave_shr1(px0, 0.0), f1 = wave_shr1(px1, 0.0), f2 = wave_shr1(px2, 0.0);
                if (cjj == 0) {
                    if (cw == 0) {
                        f0 = fq0[d & 1];
                        f1 = fq1[d & 1];
                        f2 = fq2[d & 1];
                    } else if (sg >= 1 && clane) {
                        const double* h = hb + ((sg - 1) & 1) * 48 + cp;
                        f0 = h[0];
                        f1 = h[16];
                        f2 = h[32];
                    }
                }
                if (ffifo) {   // the FIFO entry of stage sg + 2 into the slot just consumed
                    const int bq = N - 3 - sg;
                    if (sg + 2 < Ts && bq >= 0) {
                        fq0[d & 1] = __builtin_nontemporal_load(fhw + (0 * N + bq) * 16 + cp);
                        fq1[d & 1] = __builtin_nontemporal_load(fhw + (1 * N + bq) * 16 + cp);
                        fq2[d & 1] = __builtin_nontemporal_load(fhw + (2 * N + bq) * 16 + cp);
                    }
                }
                double Tn = 0.0;
                if (act && b >= 0 && b < N) {
                    const double* Rc = rec + (sg % 3) * NJ + j;
                    constexpr int S = S3;
                    const double rz0 = Rc[PR_RZ0 * S], rz1 = Rc[PR_RZ1 * S], rz2 = Rc[PR_RZ2 * S];
                    const int pmb = (int)Rc[kPreFields * S];
                    const double l10 = Rc[PR_L10 * S], l20 = Rc[PR_L20 * S], l21 = Rc[PR_L21 * S];
                    const double u01 = Rc[PR_U01 * S], u02 = Rc[PR_U02 * S], u12 = Rc[PR_U12 * S];
                    const double ru00 = Rc[PR_RU00 * S], ru11 = Rc[PR_RU11 * S], ru22 = Rc[PR_RU22 * S];
                    const double sde = Rc[PR_SDE * S];
                    // the power-law source c_i Lum (powerlaw_src_h's expression): pw at b+i+1 and b+i = c0+1-sg
                    const double pwlo = pw[(c0 + 1 - sg) * 16 + cp], pwhi = pw[(c0 + 2 - sg) * 16 + cp];
                    const double src = cj * (csf.a3 * sfr * (sEmax[b] * pwhi - sEmin[b] * pwlo) * csf.rs);
                    double add;
                    if (nonres) {
                        const int qq = (sg - 1) >> 2;              // block whose publication serves stage sg
                        const int nu = (d == 0) ? 4 : d;           // columns r+1 .. r+nu not yet pushed
                        double sa = AX[(((qq & 1) * 4 + (sg - 1 - 4 * qq)) * NJ + j) * 16 + cp];
#pragma unroll
                        for (int k = 4; k >= 1; --k)
                            if (k <= nu) sa = fma(sdg[(k - 1) * T + r], Th[k - 1], sa);
                        add = cj * sa;
                    } else {
                        const double dEb1 = (b + 1 < N) ? sEmax[b + 1] - sEmin[b + 1] : 1.0;
                        add = resonant_add(racc, u0, u1, u2, px0, px1, px2, sj, sdg[r], dEb1, sde, cj, b == N - 1);
                    }
                    double x0, x1, x2;
                    cascade_solve(f0, f1, f2, add, src, u0, u1, u2, rz0, rz1, rz2, pmb, l10, l20, l21, u01, u02, u12,
                                  ru00, ru11, ru22, x0, x1, x2);
                    if (top) {
                        if (last_pass) {   // finalise (nuSIprop.hpp:328-336)
                            const Point& Q = pts[cpid];
                            const double dE = gl.Emax[b] - gl.Emin[b];
                            const double g0 = x0 / dE, g1 = x1 / dE, g2 = x2 / dE;
                            double* fo = flux + (size_t)cpid * 3 * N;
                            double* fl = flux_fla + (size_t)cpid * 3 * N;
                            fo[b] = g0;
                            fo[N + b] = g1;
                            fo[2 * N + b] = g2;
                            for (int f = 0; f < 3; ++f)
                                fl[f * N + b] = Q.U2[3 * f + 0] * g0 + Q.U2[3 * f + 1] * g1 + Q.U2[3 * f + 2] * g2;
                        } else {
                            fhw[(0 * N + b) * 16 + cp] = x0;
                            fhw[(1 * N + b) * 16 + cp] = x1;
                            fhw[(2 * N + b) * 16 + cp] = x2;
                        }
                    }
                    if (kGbChainWaves > 1 && cw == 0 && cjj == kGbSPW - 1) {
                        double* h = hb + (sg & 1) * 48 + cp;
                        h[0] = x0;
                        h[16] = x1;
                        h[32] = x2;
                    }
                    px0 = x0; px1 = x1; px2 = x2;
                    if (nonres && b > 0) Tn = (u0 * x0 + u1 * x1 + u2 * x2) * sde;
                }
                Th[3] = Th[2]; Th[2] = Th[1]; Th[1] = Th[0]; Th[0] = Tn;
                if (clane && j < njp) Tp[((sg & 7) * NJ + j) * 16 + cp] = Tn;
                NUSI_WS_STAMP(sg, 1);
                __syncthreads();
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the FIFO stores land before the next pass reads
        }
    } else if (wave == recw) {
        // ---- phase 1 of the records two stages ahead
#pragma unroll 1
        for (int pass = 0; pass < npass; ++pass) {
            int njp, Ts, c0;
            pass_geom(pass, njp, Ts, c0);
            pass_head();
            phase1(0, lane);
            if (1 < Ts) phase1(1, lane);
            __syncthreads();
            __syncthreads();
            for (int sg = 0; sg < Ts; ++sg) {
                NUSI_WS_STAMP(sg, 0);
                if (sg + 2 < Ts) phase1(sg + 2, lane);
                NUSI_WS_STAMP(sg, 1);
                __syncthreads();
            }
        }
    } else if (wave == recw + 1) {
        // ---- phase 2 (the LU of M) one stage ahead, on a wave of its own as in k_cascade_ws<NJ, 2>
#pragma unroll 1
        for (int pass = 0; pass < npass; ++pass) {
            int njp, Ts, c0;
            pass_geom(pass, njp, Ts, c0);
            pass_head();
            __syncthreads();
            phase2(0, lane);
            __syncthreads();
            for (int sg = 0; sg < Ts; ++sg) {
                NUSI_WS_STAMP(sg, 0);
                if (sg + 1 < Ts) phase2(sg + 1, lane);
                NUSI_WS_STAMP(sg, 1);
                __syncthreads();
            }
        }
    } else {
        // ---- push: block q (stage 4q) adds columns c0+1-4q .. c0+4-4q into the rows below r = c0-4q for every
        // step and point, then publishes rows r-1 .. r-4
        const int rw0 = wave * 16 * RT;
#pragma unroll 1
        for (int pass = 0; pass < npass; ++pass) {
            int njp, Ts, c0;
            pass_geom(pass, njp, Ts, c0);
            pass_head();
            __syncthreads();
            __syncthreads();
            nusi_f64x4 acc[RT][NJ];
#pragma unroll
            for (int a = 0; a < RT; ++a)
#pragma unroll
                for (int s = 0; s < NJ; ++s) acc[a][s] = nusi_f64x4{0.0, 0.0, 0.0, 0.0};
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
            double ablk[RT];
            load_blk(1, ablk);
            for (int sg = 0; sg < Ts; ++sg) {
                NUSI_WS_STAMP(sg, 0);
                const int q = sg >> 2, r = c0 - 4 * q, hi = r - 1;
                if ((sg & 3) == 0 && nonres) {
                    if (q >= 1) {
#pragma unroll
                        for (int s = 0; s < NJ; ++s) {
                            const double bop = Tp[(((4 * q - 1 - (lane >> 4)) & 7) * NJ + s) * 16 + (lane & 15)];
#pragma unroll
                            for (int a = 0; a < RT; ++a)
                                if (rw0 + 16 * a < r)   // tiles wholly at or above r hold consumed rows only
                                    acc[a][s] = __builtin_amdgcn_mfma_f64_16x16x4f64(ablk[a], bop, acc[a][s], 0, 0, 0);
                        }
                        load_blk(q + 1, ablk);
                    }
#pragma unroll
                    for (int a = 0; a < RT; ++a)
                        if (rw0 + 16 * a <= hi && rw0 + 16 * a + 15 >= hi - 3)   // uniform: tiles holding those rows
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const int row = rw0 + 16 * a + (lane >> 4) + 4 * e;
                                const int slot = hi - row;
                                if (slot >= 0 && slot < 4)
#pragma unroll
                                    for (int s = 0; s < NJ; ++s)
                                        AX[((((q & 1) * 4 + slot) * NJ) + s) * 16 + (lane & 15)] = acc[a][s][e];
                            }
                }
                NUSI_WS_STAMP(sg, 1);
                __syncthreads();
            }
        }
    }
}
// ---------------------------------------------------------------------------
// k_cascade_bs: the MFMA cascade with block-synchronous roles (round 4).  The wavefront, the rank-4 block
// pushes on v_mfma_f64_16x16x4f64, the records and the solves are k_cascade_ws / k_cascade_gb's operations on
// the same operands; what changes is when the waves meet.  k_cascade_ws / gb / wsp synchronise every wave of
// the workgroup once per STAGE, so a stage costs a barrier, an LDS round trip of the chain's records and its
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
//   <48, 1, 1, 4, 1>  one point per workgroup (C4; k_cascade_ws<48, 1>'s shape)
//   <48, 2, 1, 2, 2>  two points sharing a table (k_cascade_ws<48, 2>), a chain wave per point
//   <6, 16, 1, 2, 2>  the gamma batch, 16 power-law points of a table (k_cascade_gb), 8 per chain wave
//   <16, 1, 1, 8, 1>  step passes on long grids (C3; k_cascade_wsp)
// and the same points get the same fluxes as from those kernels (the MFMA sums each element's four columns in
// its own order whichever column it is).  Waves: push waves of 16 RT rows, the chain waves, the record wave.
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
size_t cascade_gb_scratch_doubles(const GridDev& g) { return (size_t)3 * g.N * 16; }

// launch geometry of the wavefront kernel: one thread per pushed row (T-1), whole waves; K stages
// of records per batch, as many as the threads cover and kWfMaxLds allows
constexpr size_t kWfMaxLds = 64 * 1024;
struct WfGeom { int nthr, K; size_t lds; };
static WfGeom wf_geom(const GridDev& g, int NJ)
{
    WfGeom w;
    w.nthr = ((((g.T - 1 + kWfRows - 1) / kWfRows) * kWfQuarters + 63) / 64) * 64 + 64;   // rows + the chain wave
    w.K = w.nthr / NJ;
    auto bytes = [&](int K) {
        return sizeof(double) * (3 * (size_t)g.N + (size_t)kWfFields * K * NJ + 4 * NJ + cascade_aux_doubles(g.N, g.T) +
                                 3 * (size_t)g.T + 2 * (size_t)g.N + 4 * (size_t)g.Nz);
    };
    while (w.K > 1 && bytes(w.K) > kWfMaxLds) --w.K;
    w.lds = bytes(w.K);
    return w;
}
// step slots: up to 48 (64 accumulators would spill at two waves per SIMD)
static int wf_nj(const GridDev& g) { const int n = g.Nz - 1; return n <= 16 ? 16 : n <= 32 ? 32 : n <= 48 ? 48 : 0; }
static bool wf_fits(const GridDev& g)
{
    const int nj = wf_nj(g);
    if (!nj || g.T < 2) return false;
    const WfGeom w = wf_geom(g, nj);
    if (w.nthr > kWfMaxThreads) return false;
    return w.lds <= kWfMaxLds;
}

// the warp-specialised kernel: push waves of 16 RT rows each, then the record and chain waves
// (R = 3 here: the step-pass kernel, one right-hand side, 128 rows per push wave)
constexpr size_t kWsMaxLds[4] = {0, 80 * 1024, 150 * 1024, 160 * 1024};   // R = 1: two workgroups per CU
static WfGeom ws_geom(const GridDev& g, int NJ, int R)
{
    WfGeom w;
    const bool big = R == 3;
    if (big) R = 1;
    const int rows = big ? 16 * kWsBigRT : R == 1 ? 64 : 32;
    w.nthr = ((g.T - 1 + rows - 1) / rows) * 64 + 128 + ((R == 2 || big) ? 64 * kWsP2Wave : 0);
    w.K = 2;
    w.lds = sizeof(double) * (3 * (size_t)R * g.N + 3 * (size_t)(kWfFields + R - 1 + 6) * NJ + 16 * (size_t)R * NJ + g.N +
                              (size_t)R * (g.T + 2) + 6 * (size_t)g.T + 2 * (size_t)g.N + 4 * (size_t)g.Nz);
    return w;
}
bool cascade_ws_fits(const GridDev& g, int R)
{
    const int nj = wf_nj(g);
    if (!nj || g.T < 2 || R < 1 || R > 2) return false;
    const WfGeom w = ws_geom(g, nj, R);
    return w.nthr <= (R == 1 ? WsCfg<1>::kMaxThreads : WsCfg<2>::kMaxThreads) && w.lds <= kWsMaxLds[R];
}
// the step-pass kernel: any number of redshift steps, T - 1 <= 13 x 128 rows
bool cascade_wsp_fits(const GridDev& g)
{
    if (g.T < 2 || g.Nz < 2) return false;
    const WfGeom w = ws_geom(g, kWsBigNJ, 3);
    return w.nthr <= 1024 && w.lds <= kWsMaxLds[3];
}

static thread_local const char* t_cascade_kernel = "";   // the kernel the latest launch on this thread chose
const char* last_cascade_kernel() { return t_cascade_kernel; }

template <int NJ, int R>
static void launch_ws_nj(const GridDev& g, const Point* pts, const int2* groups, int nwg, TablesDev t, double* flux,
                         double* flux_fla, hipStream_t s)
{
    const WfGeom w = ws_geom(g, NJ, R);
    hipLaunchKernelGGL((k_cascade_ws<NJ, R>), dim3(nwg), dim3(w.nthr), w.lds, s, g, pts, groups, t, flux, flux_fla);
}

hipError_t launch_cascade_ws(const GridDev& g, const Point* pts, int R, const int2* groups, int nwg, TablesDev t,
                             double* flux, double* flux_fla, hipStream_t s)
{
    if (!cascade_ws_fits(g, R)) return hipErrorInvalidValue;
    t_cascade_kernel = R == 2 ? "k_cascade_ws_mrhs" : "k_cascade_ws";
    const int nj = wf_nj(g);
    if (R == 1) {
        if (nj == 16) launch_ws_nj<16, 1>(g, pts, groups, nwg, t, flux, flux_fla, s);
        else if (nj == 32) launch_ws_nj<32, 1>(g, pts, groups, nwg, t, flux, flux_fla, s);
        else launch_ws_nj<48, 1>(g, pts, groups, nwg, t, flux, flux_fla, s);
    } else {
        if (nj == 16) launch_ws_nj<16, 2>(g, pts, groups, nwg, t, flux, flux_fla, s);
        else if (nj == 32) launch_ws_nj<32, 2>(g, pts, groups, nwg, t, flux, flux_fla, s);
        else launch_ws_nj<48, 2>(g, pts, groups, nwg, t, flux, flux_fla, s);
    }
    return hipGetLastError();
}

// the gamma-batch kernel: push waves of 16 kGbRT rows, two chain waves, two record waves; ~90 KB of LDS at N = 300
static int gb_push_waves(const GridDev& g) { return (g.T - 1 + 16 * kGbRT - 1) / (16 * kGbRT); }
static size_t gb_lds(const GridDev& g)
{
    return sizeof(double) * (3 * (size_t)kGbNF * kGbNJ + 16 * (size_t)kGbNJ * 16 + 96 + (size_t)g.N + 16 * (size_t)(g.T + 2) +
                             6 * (size_t)g.T + 2 * (size_t)g.N + 4 * (size_t)g.Nz);
}
bool cascade_gb_fits(const GridDev& g)
{
    return g.T >= 2 && g.Nz >= 2 && gb_push_waves(g) + kGbChainWaves + 2 <= 16 && gb_lds(g) <= 160 * 1024;
}
hipError_t launch_cascade_gb(const GridDev& g, const Point* pts, const int* gidx, const int2* grp, int nwg, TablesDev t,
                             double* fh, double* flux, double* flux_fla, hipStream_t s)
{
    if (!cascade_gb_fits(g)) return hipErrorInvalidValue;
    if (nwg <= 0) return hipSuccess;
    t_cascade_kernel = "k_cascade_gb";
    const int nthr = 64 * (gb_push_waves(g) + kGbChainWaves + 2);
    hipLaunchKernelGGL((k_cascade_gb<kGbNJ>), dim3(nwg), dim3(nthr), gb_lds(g), s, g, pts, gidx, grp, t, fh, flux,
                       flux_fla);
    return hipGetLastError();
}

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
// <= 14 x 128); P = 2: <wf_nj or 48, 2, 1, 2, 2>; P = 16 (the gamma batch): <6, 16, 1, 2, 2>
int cascade_bs_config(const GridDev& g, int P)
{
    const int nj = wf_nj(g);
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
                             TablesDev t, double* fh, double* flux, double* flux_fla, hipStream_t s, bool all_nr)
{
    if (nwg <= 0) return hipSuccess;
    const int c = cascade_bs_config(g, P);
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

hipError_t launch_cascade_wsp(const GridDev& g, const Point* pts, int npts, TablesDev t, double* flux, double* flux_fla,
                              hipStream_t s, bool all_nonres)
{
    if (!cascade_wsp_fits(g)) return hipErrorInvalidValue;
    t_cascade_kernel = "k_cascade_ws_passes";
    const WfGeom w = ws_geom(g, kWsBigNJ, 3);
    if (all_nonres)
        hipLaunchKernelGGL((k_cascade_wsp<kWsBigNJ, true>), dim3(npts), dim3(w.nthr), w.lds, s, g, pts, t, flux, flux_fla);
    else
        hipLaunchKernelGGL((k_cascade_wsp<kWsBigNJ, false>), dim3(npts), dim3(w.nthr), w.lds, s, g, pts, t, flux, flux_fla);
    return hipGetLastError();
}

template <int NJ>
static void launch_wf(const GridDev& g, const Point* pts, int npts, TablesDev t, double* flux, double* flux_fla,
                      hipStream_t s, bool power_law)
{
    const WfGeom w = wf_geom(g, NJ);
    if (power_law)
        hipLaunchKernelGGL((k_cascade_wf<NJ, true>), dim3(npts), dim3(w.nthr), w.lds, s, g, pts, t, flux, flux_fla, w.K);
    else
        hipLaunchKernelGGL((k_cascade_wf<NJ, false>), dim3(npts), dim3(w.nthr), w.lds, s, g, pts, t, flux, flux_fla, w.K);
}

template <int NQ>
static void launch_reg(const GridDev& g, const Point* pts, int npts, TablesDev t, double* flux, double* flux_fla,
                       hipStream_t s)
{
    constexpr int D = NQ <= 5 ? 8 : (NQ <= 10 ? 4 : 2);
    const size_t lds = sizeof(double) * ((size_t)g.N + cascade_aux_doubles(g.N, g.T));
    hipLaunchKernelGGL((k_cascade_reg<NQ, D>), dim3(npts), dim3(64), lds, s, g, pts, t, flux, flux_fla);
}

// instantiated chunk counts; a kernel built for NQ serves every N <= 64 NQ
template <int... Q>
static bool dispatch_reg(int nq, const GridDev& g, const Point* pts, int npts, TablesDev t, double* flux,
                         double* flux_fla, hipStream_t s, std::integer_sequence<int, Q...>)
{
    bool done = false;
    ((!done && nq <= Q ? (launch_reg<Q>(g, pts, npts, t, flux, flux_fla, s), done = true) : false), ...);
    return done;
}
using RegNQ = std::integer_sequence<int, 1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20>;

// the bit-exact scalar kernels (NUSI_CASCADE_WAVEFRONT / REG / LDS): k_cascade_wf where the grid fits it,
// else k_cascade_reg (N <= 1280), else k_cascade; a kind that does not fit falls back the same way
hipError_t launch_cascade_exact(const GridDev& g, const Point* pts, int npts, TablesDev t, double* flux,
                                double* flux_fla, hipStream_t s, int kind, bool all_power_law)
{
    const int nq = (g.N + 63) / 64;
    if (kind == NUSI_CASCADE_WAVEFRONT && wf_fits(g)) {
        t_cascade_kernel = "k_cascade_wf";
        switch (wf_nj(g)) {
        case 16: launch_wf<16>(g, pts, npts, t, flux, flux_fla, s, all_power_law); break;
        case 32: launch_wf<32>(g, pts, npts, t, flux, flux_fla, s, all_power_law); break;
        default: launch_wf<48>(g, pts, npts, t, flux, flux_fla, s, all_power_law); break;
        }
        return hipGetLastError();
    }
    t_cascade_kernel = "k_cascade_reg";
    if (kind != NUSI_CASCADE_LDS && dispatch_reg(nq, g, pts, npts, t, flux, flux_fla, s, RegNQ{}))
        return hipGetLastError();
    t_cascade_kernel = "k_cascade";
    const size_t lds = cascade_lds_bytes(g.N);
    hipLaunchKernelGGL(k_cascade, dim3(npts), dim3(64), lds, s, g, pts, t, flux, flux_fla);
    return hipGetLastError();
}

}  // namespace nusi

#ifdef NUSI_WS_TRACE
// diagnostic build: workgroup 0's stage stamps of the latest k_cascade_ws launch, [wave][stage][start, barrier]
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
