// nuSIprop MI355X -- HIP kernels for calculate_flux::evolve() (nuSIprop.hpp:176-337).
//
//   k_gamma_alphat  Stage A, absorption + same-bin regeneration tables   (:217-235)
//   k_alpha         Stage A, inter-bin regeneration table, one entry per
//                   work-item, packed transposed                          (:237-252)
//   (Stage B, the cascade, is in nusi_cascade.hip)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "nusi_internal.hpp"

namespace nusi {


// ---------------------------------------------------------------------------
// Stage A
// ---------------------------------------------------------------------------
// a warning w of entry (n, m) of table p: the table's word, and (shift-reuse base plans, wmin != nullptr) the
// row record TablesDev::Wmin.  Out of line: it runs only on a warning, and inlined its atomics cost the hot
// kernels' register allocation (k_alpha_batch: 39 -> 41 VGPR spills)
__device__ __attribute__((noinline)) void warn_entry(int* warn, int* wmin, int T, int p, int w, int n, int m)
{
    atomicOr(&warn[p], w);
    if (wmin)
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if ((w >> b) & 1) atomicMin(&wmin[((size_t)p * 4 + b) * T + n], m);
}

#ifndef NUSI_GA_WAVES   // Gamma / alphaTilde kernel waves per SIMD (A/B)
#define NUSI_GA_WAVES 4   // with Gamma / alphaTilde split over work-items: 4 0.525, 3 0.535 ms (was 0.572 unsplit at 3)
#endif
// Gamma and alphaTilde: grid (T / 64, points, 2 quantities), 3 kParts waves per workgroup of 64 bins -- wave
// (k, part) runs mass state k (gamma_k / alphat_k; kParts = 2: part 1 the s-t / s-u interference, part 0 every other
// channel; kParts = 1: all), its channel terms go to LDS by slot, and wave 0 sums them in the reference's order
// (state after state, channel after channel: gamma_entry's additions, the same bits).  A wave per mass state: three
// times the waves of one work-item per entry, each a third as long (C4 reference order 2.1 -> 1.6 ms, spills 202 ->
// 26).  Calls of few tables (a single propagation: a few dozen waves in all) split the channels too (kParts = 2:
// 0.34 -> 0.29 ms for one table); on scans that split measured slower (C4 1.6 -> 2.4 ms: the parts repeat the state's
// common leaves).  With kParts = 2 the warnings, which read several channels, are formed on wave 0 from the
// unscaled values (gamma_warn, alphat_warn: the per-entry path's own predicates).  kRef: NUSI_OPT_REFERENCE_ORDER.
constexpr int kGaTerms = kAlphatSlots;   // >= kGammaSlots
struct LdsSink {
    double* v;   // this lane's column of [kGaTerms][64]: the scaled terms
    double* r;   // ... the unscaled channel values
    NUSI_FN void put(int slot, double x, double raw) { v[slot * 64] = x; r[slot * 64] = raw; }
};
// Edge sharing (round 6): the dilogarithms Gamma and alphaTilde take of one bin edge (gamma_edge_vals,
// alphat_edge_vals) are evaluated once per edge -- lane l of a wave holds the lower edge of bin n0 + l and hands it to
// bin n0 + l - 1 as its upper edge (a lane shift; hi[n] == lo[n + 1] bitwise for the first N bins), so a workgroup
// takes 63 bins and lane 63 only supplies bin n0 + 62's upper edge; a bin whose upper edge is not shared (the
// redshift-extended bins) evaluates it itself.  The same functions on the same arguments: the same bits.
NUSI_FN double shfl_dn(double x) { return __shfl_down(x, 1, 64); }
NUSI_FN double shfl_upd(double x) { return __shfl_up(x, 1, 64); }
NUSI_FN cd shfl_dn(cd z) { return cd{__shfl_down(z.r, 1, 64), __shfl_down(z.i, 1, 64)}; }
// kPre (reference order, calls of few tables): every dilogarithm value from k_ga_dilogs' block pre (ga_pre_load)
// instead of the lanes' own GSL calls
template <bool kRef, int kParts, bool kPre = false>
__global__ __launch_bounds__(192 * kParts) __attribute__((amdgpu_waves_per_eu(NUSI_GA_WAVES, NUSI_GA_WAVES))) void k_gamma_alphat(GridDev g, const Point* __restrict__ pts, const SplineSet* __restrict__ splp,
                                                     double* __restrict__ G, double* __restrict__ At,
                                                     int* __restrict__ warn, int* __restrict__ wmin,
                                                     const double* __restrict__ pre = nullptr)
{
    __shared__ double v[3][kGaTerms][64], raw[kParts == 2 ? 3 : 1][kGaTerms][64];
    __shared__ int wk[3 * kParts][64];
    const SplineSet& spl = *splp;   // (in global memory: a by-value copy would live in scratch)
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), k = wv / kParts, part = wv - k * kParts;
    const int p = blockIdx.y;
    const int n = blockIdx.x * 63 + lane, T = g.T;
    const bool act = lane < 63 && n < T;
    const Point& P = pts[p];
    const bool gam = blockIdx.z == 0;
    // this lane's edge: the lower edge of bin n, or (n == T) the last bin's upper edge
    const double elo = n < T ? g.lo[n] : n == T ? g.hi[T - 1] : 0.0;
    const double lo = act ? g.lo[n] : 0.0, hi = act ? g.hi[n] : 0.0;
    const bool up_sh = act && (n + 1 == T || g.hi[n] == g.lo[n + 1]);   // bin n's upper edge is lane + 1's
    int w = 0;
    LdsSink sk{&v[k][0][lane], &raw[kParts == 2 ? k : 0][0][lane]};
    if (kPre) {
        if (act) {
            GammaEdgePair ge;
            AlphatEdgePair ae;
            AlphatBinVals bv;
            ga_pre_load(pre + (size_t)(p * 3 + k) * kGaPreFields * T, T, n, ge, ae, bv);
            if (gam) {
                if (part == 0) gamma_k<kRef, 0>(P, k, lo, hi, sk, w, &ge);
                else gamma_k<kRef, 1>(P, k, lo, hi, sk, w, &ge);
            } else {
                if (part == 0) alphat_k<kRef, 0>(P, spl, k, lo, hi, sk, w, &ae, &bv);
                else alphat_k<kRef, 1>(P, spl, k, lo, hi, sk, w, &ae, &bv);
            }
        }
    } else if (gam) {
        GammaEdgePair ge{};
        unsigned need = 0;
        if (act) need = kParts == 1 ? gamma_edge_need<-1>(P, k, lo, hi) : part == 0 ? gamma_edge_need<0>(P, k, lo, hi)
                                                                                    : gamma_edge_need<1>(P, k, lo, hi);
        const unsigned from_prev = (unsigned)__shfl_up((int)(up_sh ? need : 0u), 1, 64);
        const unsigned need_lo = need | (lane > 0 ? from_prev : 0u);
        gamma_edge_vals<kRef>(P, k, elo, need_lo, ge.lo);
        ge.hi.ls = shfl_dn(ge.lo.ls);
        ge.hi.l1s = shfl_dn(ge.lo.l1s);
        ge.hi.cz = shfl_dn(ge.lo.cz);
        if (!kRef) ge.hi.czc = shfl_dn(ge.lo.czc);
        if (act && !up_sh) gamma_edge_vals<kRef>(P, k, hi, need, ge.hi);
        if (act) {
            if (kParts == 1) gamma_k<kRef, -1>(P, k, lo, hi, sk, w, &ge);
            else if (part == 0) gamma_k<kRef, 0>(P, k, lo, hi, sk, w, &ge);
            else gamma_k<kRef, 1>(P, k, lo, hi, sk, w, &ge);
        }
    } else {
        AlphatEdgePair ae{};
        unsigned need = 0;
        if (act) need = kParts == 1 ? alphat_edge_need<-1>(P, k, lo, hi) : part == 0 ? alphat_edge_need<0>(P, k, lo, hi)
                                                                                     : alphat_edge_need<1>(P, k, lo, hi);
        const unsigned from_prev = (unsigned)__shfl_up((int)(up_sh ? need : 0u), 1, 64);
        const unsigned need_lo = need | (lane > 0 ? from_prev : 0u);
        alphat_edge_vals<kRef>(P, k, elo, need_lo, ae.lo);
        ae.hi.e78 = shfl_dn(ae.lo.e78);
        ae.hi.e51 = shfl_dn(ae.lo.e51);
        ae.hi.e1o = shfl_dn(ae.lo.e1o);
        ae.hi.e1p = shfl_dn(ae.lo.e1p);
        if (act && !up_sh) alphat_edge_vals<kRef>(P, k, hi, need, ae.hi);
        if (act) {
            if (kParts == 1) alphat_k<kRef, -1>(P, spl, k, lo, hi, sk, w, &ae);
            else if (part == 0) alphat_k<kRef, 0>(P, spl, k, lo, hi, sk, w, &ae);
            else alphat_k<kRef, 1>(P, spl, k, lo, hi, sk, w, &ae);
        }
    }
    if (act) wk[wv][lane] = w;
    __syncthreads();
    if (wv != 0 || !act) return;
    const int ns = !P.non_resonant ? 1 : gam ? kGammaSlots : kAlphatSlots;
    SumSink tot;
    w = 0;
    for (int kk = 0; kk < 3; ++kk) {
        for (int i = 0; i < ns; ++i) tot.put(i, v[kk][i][lane], 0.0);
        for (int pp = 0; pp < kParts; ++pp) w |= wk[kk * kParts + pp][lane];
        if (kParts == 2 && P.non_resonant) {
            const double* x = &raw[kParts == 2 ? kk : 0][0][lane];
            w |= gam ? gamma_warn(x[0], x[64], x[128], x[192], x[256])
                     : alphat_warn(x[0], x[64], x[128], x[192], x[256], x[320], P.a_nrm);
        }
    }
    (gam ? G : At)[(size_t)p * g.T + n] = tot.tot;
    if (w) warn_entry(warn, wmin, g.T, p, w, n, n);
}

// 4 x 4 windows of a 3-D spline table (nusi_spline.hpp): fw[16 node + 4 a1 + a2] = f[i0][i1 + a1][i2 + a2]
__global__ __launch_bounds__(256) void k_spline_windows(const float* __restrict__ f, int n0, int n1, int n2,
                                                        float* __restrict__ fw)
{
    const size_t node = (size_t)blockIdx.x * 256 + threadIdx.x, nn = (size_t)n0 * n1 * n2;
    if (node >= nn) return;
    const int i2 = (int)(node % n2), i1 = (int)((node / n2) % n1);
    const size_t row = node - (size_t)i1 * n2 - i2;   // (i0, 0, 0)
    float4 out[4];
#pragma unroll
    for (int a1 = 0; a1 < 4; ++a1) {
        const size_t r = row + (size_t)min(i1 + a1, n1 - 1) * n2;
        out[a1] = make_float4(f[r + min(i2, n2 - 1)], f[r + min(i2 + 1, n2 - 1)], f[r + min(i2 + 2, n2 - 1)],
                              f[r + min(i2 + 3, n2 - 1)]);
    }
    float4* dst = reinterpret_cast<float4*>(fw + 16 * node);
#pragma unroll
    for (int a1 = 0; a1 < 4; ++a1) dst[a1] = out[a1];
}

hipError_t spline_windows_build(const float* f, int n0, int n1, int n2, float* fw)
{
    const size_t nn = (size_t)n0 * n1 * n2;
    hipLaunchKernelGGL(k_spline_windows, dim3((unsigned)((nn + 255) / 256)), dim3(256), 0, 0, f, n0, n1, n2, fw);
    hipError_t e = hipGetLastError();
    return e != hipSuccess ? e : hipDeviceSynchronize();
}

// one entry per work-item over the bins [nlo, T) x [nlo, T), n < m (nlo = 0: the whole table)
#ifndef NUSI_PE_WAVES   // per-entry kernel waves per SIMD (A/B)
#define NUSI_PE_WAVES 3   // 3: 20.05 vs 20.24 ms alpha stage (profiles/r1i/ab_occ_*)
#endif
template <bool kRef>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NUSI_PE_WAVES, NUSI_PE_WAVES)))
void k_alpha(GridDev g, const Point* __restrict__ pts, const SplineSet* __restrict__ splp, int nlo,
                                               double* __restrict__ A, int* __restrict__ warn, int* __restrict__ wmin)
{
    const SplineSet& spl = *splp;
    const int p = blockIdx.y;
    const long long L = g.T - nlo;
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    if (e >= L * (L - 1) / 2) return;
    // packed transposed index e = m'(m'-1)/2 + n', n' < m', within the sub-triangle
    int m = (int)((1.0 + sqrt(1.0 + 8.0 * (double)e)) * 0.5);
    while ((long long)m * (m - 1) / 2 > e) --m;
    while ((long long)(m + 1) * m / 2 <= e) ++m;
    int n = (int)(e - (long long)m * (m - 1) / 2);
    n += nlo;
    m += nlo;
    const Point& P = pts[p];
    int w = 0;
    double v = 0.0;
    // without non-s channels the cascade reads only alpha(n, n+1) (nuSIprop.hpp:273-275)
    if (P.non_resonant || m == n + 1) v = alpha_entry<kRef>(P, spl, g.lo[n], g.hi[n], g.lo[m], g.hi[m], w);
    A[(size_t)p * g.PT + (size_t)m * (m - 1) / 2 + n] = v;
    if (w) warn_entry(warn, wmin, g.T, p, w, n, m);
}

// Calls of few tables in the reference order: every GSL dilogarithm of Gamma / alphaTilde, one per work-item
// (ga_pre_slot; grid (bins / 64, points, 3 mass states x kGaPreSlots)) into pre [point][k][kGaPreFields][T], before
// k_gamma_alphat<true, 2, true> combines them: a lane no longer walks its bin's six GSL series one after the other
__global__ __launch_bounds__(64) void k_ga_dilogs(GridDev g, const Point* __restrict__ pts, double* __restrict__ pre)
{
    const int n = blockIdx.x * 64 + threadIdx.x, p = blockIdx.y, T = g.T;
    const int k = blockIdx.z / kGaPreSlots, slot = blockIdx.z - k * kGaPreSlots;   // (wave-uniform slot)
    if (n >= T) return;
    const Point& P = pts[p];
    if (!P.non_resonant) return;   // (gamma_k / alphat_k return before any dilogarithm)
    double v[2];
    int f;
    const int nv = ga_pre_slot(P, k, g.lo[n], g.hi[n], slot, v, &f);
    double* o = pre + ((size_t)(p * 3 + k) * kGaPreFields + f) * T + n;
    o[0] = v[0];
    if (nv == 2) o[T] = v[1];
}

#ifndef NUSI_GA_PRE_ALL   // A/B: 1 = scans too take the dilogarithm pre-pass (k_ga_dilogs)
#define NUSI_GA_PRE_ALL 0
#endif
size_t gamma_alphat_pre_doubles(int T, int npts) { return (size_t)3 * kGaPreFields * T * npts; }

hipError_t launch_gamma_alphat(const GridDev& g, const Point* pts, int npts, const SplineSet* spl, TablesDev t,
                               int* warn, hipStream_t s, bool ref)
{
    dim3 grid((g.T + 62) / 63, npts, 2);   // (63 bins per workgroup: the edge-shared lanes)
    if (ref && t.Gpre && (npts <= 16 || NUSI_GA_PRE_ALL)) {   // (the dilogarithms one per work-item first)
        hipLaunchKernelGGL(k_ga_dilogs, dim3((g.T + 63) / 64, npts, 3 * kGaPreSlots), dim3(64), 0, s, g, pts, t.Gpre);
        hipLaunchKernelGGL((k_gamma_alphat<true, 2, true>), grid, dim3(384), 0, s, g, pts, spl, t.G, t.At, warn, t.Wmin,
                           t.Gpre);
        return hipGetLastError();
    }
    if (npts <= 16) {   // (a few tables: the channels split too, kParts = 2)
        if (ref) hipLaunchKernelGGL((k_gamma_alphat<true, 2>), grid, dim3(384), 0, s, g, pts, spl, t.G, t.At, warn, t.Wmin);
        else hipLaunchKernelGGL((k_gamma_alphat<false, 2>), grid, dim3(384), 0, s, g, pts, spl, t.G, t.At, warn, t.Wmin);
    } else {
        if (ref) hipLaunchKernelGGL((k_gamma_alphat<true, 1>), grid, dim3(192), 0, s, g, pts, spl, t.G, t.At, warn, t.Wmin);
        else hipLaunchKernelGGL((k_gamma_alphat<false, 1>), grid, dim3(192), 0, s, g, pts, spl, t.G, t.At, warn, t.Wmin);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// k_alpha_tile: one workgroup per (kAlphaTile x kAlphaTile bin tile, point).
//
//   1. the distinct bin edges of the tile's n side (t) and m side (S');
//   2. edge and m-bin leaves of all three mass states -> LDS (one round);
//   3. per mass state k: every (S', t) corner leaf -> LDS (one corner per
//      work-item: a core tile has 16 x 16 = 256 corners), then every entry of
//      the tile combines its four corners, four edges and its m bin
//      (alpha_k<TileLeaves>), accumulating the k sum in a register.
// A core tile evaluates 256 corners for its 225 entries where the per-entry
// path evaluates 4 per entry: the dilogarithms, complex dilogarithms and
// mixed logarithms that dominate the table cost are ~3.5x fewer.
// ---------------------------------------------------------------------------
constexpr int kTileThreads = 256;
static_assert(kAlphaTile * kAlphaTile <= kTileThreads, "one entry per work-item");

// dynamic LDS of a tile for batches of up to G points: corner block, edge blocks, per-point sums
__host__ __device__ constexpr int alpha_tile_lds_doubles(int cs, int ct, int G)
{
    return alpha_tile_corner_block(cs, ct, G) + alpha_tile_edge_doubles(cs, ct, G) + (G > 1 ? G * kTileThreads : 0);
}

// 3 waves per SIMD (<= 168 VGPRs): measured 38.5 ms vs 42.0 (2 waves, 222 VGPRs) and 42.4 (4 waves,
// spills) per 1024-point table build (profiles/r1e/ab3_*.log); override with -DNUSI_TILE_WAVES=n
#ifndef NUSI_TILE_WAVES
#define NUSI_TILE_WAVES 3
#endif
#define NUSI_TILE_ATTR __attribute__((amdgpu_waves_per_eu(NUSI_TILE_WAVES, NUSI_TILE_WAVES)))
// One workgroup per (tile, batch).  A batch is 1..G tables whose points share m_phi, the masses and
// the channel flags (nusi_capi.cpp orders the tables so): the leaves of (S', t) alone -- the real
// dilogarithms and most logarithms -- are evaluated once for the batch, the leaves that read
// gr = Gamma_phi / m_phi once per point.  batches[y] = first table | count << 24 (nullptr: table y alone).
template <int G, bool kRef>   // batch capacity (compile time, so that G = 1 keeps its sum in a register);
                              // kRef: NUSI_OPT_REFERENCE_ORDER member corners
__global__ __launch_bounds__(kTileThreads) NUSI_TILE_ATTR void k_alpha_tile(GridDev g, const Point* __restrict__ pts, const SplineSet* __restrict__ splp,
                                                           const int* __restrict__ tiles, int cs_max, int ct_max,
                                                           const int* __restrict__ batches,
                                                           double* __restrict__ A, int* __restrict__ warn,
                                                           int* __restrict__ wmin)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const SplineSet& spl = *splp;
    __shared__ double tE[2 * kAlphaTile], sE[2 * kAlphaTile];
    __shared__ int tl[kAlphaTile], th[kAlphaTile], sl[kAlphaTile], sh[kAlphaTile];
    __shared__ int cnt[2];
    __shared__ double elo[2][kAlphaTile], ehi[2][kAlphaTile];   // bin edges of both sides, staged in parallel
    const int tid = threadIdx.x, T = g.T;
    const int bw = batches ? batches[blockIdx.y] : (int)blockIdx.y | (1 << 24);
    const int p0 = bw & 0xffffff, nb = (G == 1) ? 1 : bw >> 24;   // tables p0 .. p0 + nb - 1 (nb <= G)
    const int tw = tiles[blockIdx.x];
    // tile word: tn | tm << 14 | mhalf << 28 | nhalf << 30; half 1 / 2 = the first 8 / last 7 bins of
    // that side of the tile only (redshift-extended sides are split so that their at most 16 edges fit
    // the core tiles' LDS)
    const unsigned tu = (unsigned)tw;
    const int half = (tu >> 28) & 3, nhalf = (tu >> 30) & 3;
    const int n0 = (tu & 0x3fff) * kAlphaTile + (nhalf == 2 ? 8 : 0);
    const int m0 = ((tu >> 14) & 0x3fff) * kAlphaTile + (half == 2 ? 8 : 0);
    const int mcnt = half == 0 ? kAlphaTile : (half == 1 ? 8 : kAlphaTile - 8);
    const int ncnt = nhalf == 0 ? kAlphaTile : (nhalf == 1 ? 8 : kAlphaTile - 8);
    const int Tm = (m0 + mcnt < T) ? m0 + mcnt : T;   // bins of the m side: [m0, Tm)
    const int Tn = (n0 + ncnt < T) ? n0 + ncnt : T;   // bins of the n side: [n0, Tn)
    const Point& P = pts[p0];   // the batch's shared fields (m_phi, masses, flags)
    if (tid < 2 * kAlphaTile) {
        const int side = tid / kAlphaTile, j = tid - side * kAlphaTile, b = (side ? m0 : n0) + j;
        if (b < (side ? Tm : Tn)) { elo[side][j] = g.lo[b]; ehi[side][j] = g.hi[b]; }
    }
    __syncthreads();
    if (tid == 0) cnt[0] = alpha_edge_list(elo[0], ehi[0], 0, Tn - n0, tE, tl, th);
    if (tid == 64) cnt[1] = alpha_edge_list(elo[1], ehi[1], 0, Tm - m0, sE, sl, sh);
    __syncthreads();
    const int ct = cnt[0], cs = cnt[1], cc = cs * ct;
    const int ln = tid % kAlphaTile, lm = tid / kAlphaTile;
    const int n = n0 + ln, m = m0 + lm;
    const bool valid = tid < kAlphaTile * kAlphaTile && n < m && m < Tm && n < Tn;
    if (cs > cs_max || ct > ct_max || nb > G) {   // host classification guarantees this never happens
        if (valid)
            for (int q = 0; q < nb; ++q) A[(size_t)(p0 + q) * g.PT + (size_t)m * (m - 1) / 2 + n] = __builtin_nan("");
        return;
    }
    const bool nonres = P.non_resonant, maj = P.majorana;
    const bool needed = valid && (nonres || m == n + 1);
    double* cor = sm;
    double* edg = sm + alpha_tile_corner_block(cs, ct, G);
    double* tsum = edg + alpha_tile_edge_doubles(cs, ct, G);   // [G][kTileThreads] per-point sums (G > 1)
    double tot1 = 0.0;                                          // the sum of a batch of one
    // ---- 2. edge and m-bin leaves, all k: shared jobs, one round
    {
        // one job kind per wave (t edges: wave 0, S' edges: waves 1-2, m bins: wave 3), so no wave runs
        // two kinds' code one after the other; other tile shapes take the jobs in order
        const int per = ct + cs + kAlphaTile, w = tid >> 6, l = tid & 63;
        int job = -1;
        if (3 * ct <= 64 && 3 * cs <= 128) {
            if (w == 0) { if (l < 3 * ct) job = (l / ct) * per + l % ct; }
            else if (w <= 2) { const int q = tid - 64; if (q < 3 * cs) job = (q / cs) * per + ct + q % cs; }
            else if (l < 3 * kAlphaTile) job = (l / kAlphaTile) * per + ct + cs + l % kAlphaTile;
        } else if (tid < 3 * per) {
            job = tid;
        }
        if (job >= 0) {   // the shared leaves, then the same edge's member leaves of every batch point
            alpha_tile_edge_job(P, job, tE, ct, sE, cs, g.lo, g.hi, m0, Tm, edg);
#pragma unroll 1
            for (int q = 0; q < nb; ++q)
                alpha_tile_edge_member_job(pts[p0 + q], q, G, job, tE, ct, sE, cs, g.lo, g.hi, m0, Tm, edg);
        }
        if (G > 1)
            for (int q = 0; q < nb; ++q) tsum[q * kTileThreads + tid] = 0.0;
    }
    for (int k = 0; k < 3; ++k) {
        __syncthreads();   // edge leaves written / previous k's corners consumed
        if (nonres && maj) {
            const double* edgk = edg + k * alpha_tile_edge_stride(cs, ct);
            for (int j = tid; j < cc; j += kTileThreads) {   // corner j: shared leaves, then each point's
                alpha_tile_corner_job<kRef>(j, edgk, ct, cs, cor);
#pragma unroll 1
                for (int q = 0; q < nb; ++q) alpha_tile_corner_member_job<kRef>(pts[p0 + q], q, j, edgk, ct, cs, cor);
            }
            for (int j = tid; j < kAlphaTile * (cs + ct); j += kTileThreads)
                alpha_tile_mixed_job(j, edgk, ct, cs, G, tl, th, sl, sh, n0, m0, Tn, Tm, cor);
        }
        __syncthreads();
        if (needed) {
            // the t and tu channels' brackets depend on the shared leaves only: once per entry
            AlphaPre pre;
            const bool share = G > 1 && nb > 1 && nonres && maj;
            if (share) {
                const TileLeaves lv0 = alpha_tile_leaves(cor, edg, k, 0, G, cs, ct, lm, sl, sh, tl, th, ln);
                alpha_k_pre(P, k, g.lo[n], g.hi[n], g.lo[m], g.hi[m], lv0, pre);
            }
#pragma unroll 1
            for (int q = 0; q < nb; ++q) {
                double tot = (G > 1) ? tsum[q * kTileThreads + tid] : tot1;
                int w = 0;
                const TileLeaves lv = alpha_tile_leaves(cor, edg, k, q, G, cs, ct, lm, sl, sh, tl, th, ln);
                alpha_k(pts[p0 + q], spl, k, g.lo[n], g.hi[n], g.lo[m], g.hi[m], lv, tot, w, share ? &pre : nullptr);
                if (G > 1) tsum[q * kTileThreads + tid] = tot;
                else tot1 = tot;
                if (w) warn_entry(warn, wmin, T, p0 + q, w, n, m);
            }
        }
    }
    if (valid)
        for (int q = 0; q < nb; ++q)
            A[(size_t)(p0 + q) * g.PT + (size_t)m * (m - 1) / 2 + n] =
                needed ? ((G > 1) ? tsum[q * kTileThreads + tid] : tot1) : 0.0;
}

// ---------------------------------------------------------------------------
// k_alpha_batch: one workgroup per (class-0 tile, batch of up to 255 tables sharing m_phi, the masses
// and the channel flags).  Mass state by mass state, the leaves of (S', t) alone -- and from them the
// t / t-u / phi-phi brackets and the Taylor coefficients of the member complex dilogarithms about their
// gr-free real points -- are formed ONCE per batch; then the batch's points run through their member
// leaves (edge leaves for kBatchQC points at a time, one job per thread; per corner one Taylor
// evaluation) and the per-point combine.  The shared work per table falls as 1 / batch (C4: 32
// couplings per m_phi, C5: 64).  A point's entry accumulates over the mass states in the output array
// (the reference's k order and term order: bit-identical to k_alpha_tile and to the oracle).
//
// LDS (doubles; cs, ct <= kAlphaTile + 1, cc = cs ct; offsets for the largest tile):
//   P3   [3][cc]   L, Drr, Dri of the current k
//   X    [10][cc]  the current k's member coefficients (alpha_batch_xshared_job); while the brackets are
//                  formed it holds LL, TU1, TU2, G [4][cc] and the mixed logs [kAlphaTile (cs + ct)]
//   mem  [2][cc]   member corner leaves Dcr, Dci of the current (point, k)
//   edg  [alpha_tile_edge_stride]  shared edge / m-bin leaves of the current k
//   memb [kBatchQC][alpha_batch_memb_doubles]  member edge leaves of a chunk of points
// ---------------------------------------------------------------------------
#ifndef NUSI_BATCH_QC   // points per member-edge round (5: C4 alpha 6.05 -> 5.95 ms vs 4, profiles/r2q)
#define NUSI_BATCH_QC 5
#endif
constexpr int kBatchQC = NUSI_BATCH_QC;   // kBatchQC (ct + cs + kAlphaTile) <= 256 jobs
// NUSI_BATCH_PIPE (A/B): the member corners of point q + 1 are formed while point q combines (two mem buffers),
// one barrier per point instead of two
#ifndef NUSI_BATCH_PIPE
#define NUSI_BATCH_PIPE 0
#endif
constexpr bool kBatchPipe = NUSI_BATCH_PIPE != 0;
// NUSI_REFO_PREFETCH (A/B): the reference-order member corners of point q + 1 are loaded while point q combines
#ifndef NUSI_REFO_PREFETCH
#define NUSI_REFO_PREFETCH 1
#endif
constexpr bool kRefPrefetch = NUSI_REFO_PREFETCH != 0;
#ifndef NUSI_BATCH_KLAUNCH   // A/B: 1 = the non-phi-phi batch kernels as one launch per mass state (kOneK)
#define NUSI_BATCH_KLAUNCH 0
#endif
constexpr bool kBatchKLaunch = NUSI_BATCH_KLAUNCH != 0;
#ifndef NUSI_REFO_BSTUB   // timing A/B only (wrong tables): bit 1 the batch kernel without the block's loads, bit 2
                          // without the chunk's A (atan2 of the member quotient), bit 3 without the per-point combine
#define NUSI_REFO_BSTUB 0
#endif
__host__ __device__ inline int alpha_batch_lds_doubles()
{
    const int c1 = kAlphaTile + 1;
    return (3 + kXFields + (kBatchPipe ? 4 : 2)) * c1 * c1 + alpha_tile_edge_stride(c1, c1) +
           kBatchQC * alpha_batch_memb_doubles(c1, c1);
}
static_assert(kXFields * (kAlphaTile + 1) * (kAlphaTile + 1) >= 4 * (kAlphaTile + 1) * (kAlphaTile + 1) + kAlphaTile * 2 * (kAlphaTile + 1),
              "the bracket phase's blocks fit X");
static_assert(kBatchQC * (2 * (kAlphaTile + 1) + kAlphaTile) <= kTileThreads, "one member-edge round per chunk");
static_assert(3 + kBatchQC <= kXFields, "(kRef) the chunk's A fields fit X beside Dcr, Dci");

#ifndef NUSI_BATCH_WAVES
#define NUSI_BATCH_WAVES 4
#endif
// waves per SIMD of k_alpha_batch: 4 (128 VGPRs; the LDS holds four workgroups per CU), and 3 for the reference-order
// instance without phi-phi (NUSI_BATCH_WAVES_REFO, 168 VGPRs): spills 82 -> 35, C4 7.28 -> 6.76 ms (profiles/r5/r6u,
// r6v; shipped in round 6).  The default-order instance is equal at 3 and 4, the phi-phi reference-order one slower at
// 3 (C3 11.1 -> 12.0 ms per chunk)
#ifndef NUSI_BATCH_WAVES_REFO
#define NUSI_BATCH_WAVES_REFO 3
#endif
constexpr int batch_waves(bool pp, bool ref) { return ref && !pp ? NUSI_BATCH_WAVES_REFO : NUSI_BATCH_WAVES; }
// the batch-shared phases out of line: they run once per batch, and inlined their working sets raise the register
// pressure of the per-point loop (measured slower: round 1 profiles/r1e, round 2 profiles/r2s, r2aa)
#define NUSI_BCOLD __device__ __attribute__((noinline))
template <bool kRef>
NUSI_BCOLD void b_corner(int j, const double* edgk, int ct, int cs, double* per, double* tmp)
{
#ifdef NUSI_REFO_SHARED_FAST   // timing A/B only: the reference-order batches' shared corners in the default arithmetic
    alpha_batch_corner_job<false>(j, edgk, ct, cs, per, tmp);
#else
    alpha_batch_corner_job<kRef>(j, edgk, ct, cs, per, tmp);
#endif
}
// (kRef, kPP) A of a member corner, out of line (the phi-phi instance's point loop spills more with it inline)
NUSI_BCOLD double b_marg(double S, double t, double gr) { return alpha_member_ref_arg(S, t, gr); }
NUSI_BCOLD void b_xshared(int j, const double* edgk, int ct, int cs, double* X) { alpha_batch_xshared_job(j, edgk, ct, cs, X); }
// The leaves the batch's shared brackets read (alpha_k_pre, alpha_k_pp): the shared corner blocks P3 | tmp, the
// edge block edgk and the mixed logs; no member leaf
NUSI_FN SplitLeaves batch_bracket_leaves(const double* P3, const double* tmp, const double* mix, const double* edgk,
                                         int cs, int ct, int lm, int ln, int s0, int s1, int t0, int t1)
{
    const int cc = cs * ct;
    SplitLeaves lv;
    lv.cf[0] = P3; lv.cf[1] = tmp; lv.cf[2] = tmp + kCC; lv.cf[3] = tmp + 2 * kCC; lv.cf[4] = tmp + 3 * kCC;
    lv.cf[5] = P3 + kCC; lv.cf[6] = P3 + 2 * kCC;
    lv.corm = P3;   // (not read by the brackets)
    lv.cc = cc; lv.ct = ct; lv.cs = cs; lv.mb = lm; lv.nb = ln;
    lv.sidx[0] = s0; lv.sidx[1] = s1; lv.tidx[0] = t0; lv.tidx[1] = t1;
    lv.ted = edgk; lv.sed = edgk + kTEdgeFields * ct; lv.mbv = lv.sed + kSEdgeFields * cs;
    lv.tedm = P3; lv.sedm = P3; lv.mbm = P3; lv.marg = P3;   // (not read)
    lv.xl = mix; lv.yl = mix + kAlphaTile * cs;
    return lv;
}
// (returned by value: an out parameter's address would keep the caller's copy in scratch, reloaded by every
// point's combine; the leaves are built here from scalars -- a SplitLeaves argument is passed in memory, and its
// per-lane copy was ~200 B of scratch stores per thread and mass state)
NUSI_BCOLD AlphaPre b_pre(const Point& P, int k, double Em, double Ep, double Emp, double Epp, const double* P3,
                          const double* tmp, const double* mix, const double* edgk, int cs, int ct, int lm, int ln,
                          int s0, int s1, int t0, int t1)
{
    const SplitLeaves lv = batch_bracket_leaves(P3, tmp, mix, edgk, cs, ct, lm, ln, s0, s1, t0, t1);
    AlphaPre pre;
    alpha_k_pre(P, k, Em, Ep, Emp, Epp, lv, pre);
    return pre;
}

// member edge leaves of every (table, k, bin edge) -> t.Med (alpha_medge_job); grid (jobs / 256, tables, 3)
__global__ __launch_bounds__(256) void k_alpha_medge(GridDev g, const Point* __restrict__ pts, double* __restrict__ med)
{
    const int j = blockIdx.x * 256 + threadIdx.x, p = blockIdx.y, k = blockIdx.z, T = g.T;
    if (j >= 5 * T) return;
    alpha_medge_job(pts[p], k, j, T, g.lo, g.hi, med + ((size_t)p * 3 + k) * kMedFields * T);
}

// NUSI_OPT_REFERENCE_ORDER: the member corners of every table of the batches [0, gridDim.y) -> mc (MCornerDev's
// layout); grid (NC / cb, batches, 3 mass states), cb = jobs / nb corners of a batch of nb tables per workgroup (the grid
// sized for the chunk's largest batch).  A workgroup takes corners [c0, c0 + cb): job j (up to 4 per work-item) is
// corner c0 + j / nb of table q = j % nb,
// so a wavefront's lanes hold the batch's tables at a few neighbouring corners, whose quotients -- differing in gr
// only -- take similar GSL branches and series lengths (in the tile's corner order the lanes of a wave diverge: 0.21
// ns per call against 0.06, scripts/dev/gsl_bench.hip).  The values pass through LDS to leave as runs of cb corners
// per (field, table), the layout the batch kernel reads a tile's corner rows from.
#ifndef NUSI_MC_JOBS   // A/B: jobs (corner x point) per k_alpha_mcorner workgroup on scans, a multiple of 256
#define NUSI_MC_JOBS 1024
#endif
constexpr int kMcJobs = NUSI_MC_JOBS;
#ifndef NUSI_MC_WAVES   // A/B: waves per SIMD the member-corner kernel is built for (0: the compiler's choice)
#define NUSI_MC_WAVES 0
#endif
__global__ __launch_bounds__(256)
#if NUSI_MC_WAVES
__attribute__((amdgpu_waves_per_eu(NUSI_MC_WAVES, NUSI_MC_WAVES)))
#endif
void k_alpha_mcorner(const Point* __restrict__ pts, const int* __restrict__ batches,
                                                       MCornerDev mc, int pc0, int jobs)
{
    __shared__ double v[2 * kMcJobs];   // [q][cl][Dcr, Dci]
    __shared__ double cst[2][kMcJobs];           // S', t of corner c0 + cl (shared by the batch's tables)
    const int bw = batches[blockIdx.y], k = blockIdx.z, tid = threadIdx.x;
    const int p0 = bw & 0xffffff, nb = (int)((unsigned)bw >> 24);
    const Point& P = pts[p0];
    if (!(P.non_resonant && P.majorana)) return;   // (no member corners)
    const int cb = jobs / nb;   // this batch's corners per workgroup (jobs <= kMcJobs)
    const long long c0 = (long long)blockIdx.x * cb;
    if (c0 >= mc.NC) return;   // (the grid is sized for the chunk's largest batch)
    const int nj = cb * nb;
    for (int cl = tid; cl < cb && c0 + cl < mc.NC; cl += 256) alpha_mcorner_st(P, k, c0 + cl, mc.ue, cst[0][cl], cst[1][cl]);
    __syncthreads();
    for (int j = tid; j < nj; j += 256) {
        const int cl = j / nb, q = j - cl * nb;
        if (c0 + cl >= mc.NC) break;
        const double S = cst[0][cl], t = cst[1][cl], gr = pts[p0 + q].a_gr;
        const cd Dc = NUSI_REFO_STUB == 2 ? C(0.0) : alpha_member_ref_dc_inl(S, t, gr);
        v[2 * (q * cb + cl)] = Dc.r;
        v[2 * (q * cb + cl) + 1] = Dc.i;
    }
    __syncthreads();
    double* const o = mc.buf + (size_t)(p0 - pc0) * 6 * mc.NC + (size_t)k * 2 * nb * mc.NC;
    for (int e = tid; e < 2 * nj; e += 256) {   // runs of 2 cb doubles per table q
        const int q = e / (2 * cb), r = e - q * 2 * cb;
        if (c0 + r / 2 < mc.NC) o[((size_t)q * mc.NC + c0) * 2 + r] = v[e];
    }
}

void mcorner_edges(int T, const double* lo, const double* hi, std::vector<int>& eu, std::vector<double>& ue)
{
    eu.assign(2 * (size_t)T, 0);
    ue.clear();
    for (int b = 0; b < T; ++b) {
        if (b == 0 || !(lo[b] == hi[b - 1])) ue.push_back(lo[b]);   // else the previous bin's upper edge
        eu[2 * b] = (int)ue.size() - 1;
        ue.push_back(hi[b]);
        eu[2 * b + 1] = (int)ue.size() - 1;
    }
}


// Diagnostic build only (-DNUSI_BATCH_TRACE, scripts/build_variant.sh): s_memtime stamps of the reference-order batch
// kernel's phases in workgroups (x < 4, y < 4), per wave, in program order (per mass state: its start, the edge
// leaves' barrier, the shared corners' barrier, the brackets' barrier; per chunk: its start, its member edges and A
// done; per point: its two barriers and its combine done).  nusi_debug_batch_trace() copies them out; compiled out of
// the product.
#ifdef NUSI_BATCH_TRACE
constexpr int kBtWg = 16, kBtN = 512;
__device__ unsigned long long g_bt[kBtWg * 4 * kBtN];
#define NUSI_BT()                                                                                                   \
    do {                                                                                                            \
        if (kRef && !kPP && !kSplit && blockIdx.x < 4 && blockIdx.y < 4 && (threadIdx.x & 63) == 0 && bt_i < kBtN) \
            g_bt[((blockIdx.y * 4 + blockIdx.x) * 4 + (threadIdx.x >> 6)) * kBtN + bt_i] = __builtin_amdgcn_s_memtime(); \
        ++bt_i;                                                                                                     \
    } while (0)
#else
#define NUSI_BT() do { } while (0)
#endif
// kPP: the batches' tables have the phi-phi channel (its shared term per k).  kRef: NUSI_OPT_REFERENCE_ORDER -- each
// point's member corners in the reference's operation order, read from k_alpha_mcorner's block mc (Dcr, Dci, A into
// the X block, which then holds no Taylor coefficients; pc0: the first table of the launch chunk), the rest of the
// batch structure unchanged.  kSplit (calls of few tables, a single propagation): mass state k = blockIdx.z only,
// its terms of every entry recorded into kt ([table][3][PT][8]: up to 7 terms, then their count, -1 for an entry
// the resonant-only table does not compute) for k_alpha_ksum -- three times the workgroups, each a third as long
// kOneK (NUSI_BATCH_KLAUNCH A/B): one mass state per launch, kone, the launches k = 0, 1, 2 in order on the stream
// (the running sum through A as in the loop): no state lives across the k loop
template <bool kPP, bool kRef, bool kSplit = false, bool kOneK = false>
__global__ __launch_bounds__(kTileThreads) __attribute__((amdgpu_waves_per_eu(batch_waves(kPP, kRef), batch_waves(kPP, kRef))))
void k_alpha_batch(GridDev g, const Point* __restrict__ pts, const SplineSet* __restrict__ splp, const int* __restrict__ tiles,
                   const int* __restrict__ batches, double* __restrict__ A, const double* __restrict__ med,
                   int* __restrict__ warn, int* __restrict__ wmin, MCornerDev mc, int pc0, double* __restrict__ kt,
                   int kone = 0)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const SplineSet& spl = *splp;
    __shared__ double tE[2 * kAlphaTile], sE[2 * kAlphaTile];
    __shared__ int tl[kAlphaTile], th[kAlphaTile], sl[kAlphaTile], sh[kAlphaTile];
    __shared__ int cnt[2];
    __shared__ double elo[2][kAlphaTile], ehi[2][kAlphaTile];
    const int tid = threadIdx.x, T = g.T;
    // (an XCD-contiguous remap of the blocks measured slower than the dealt order: C4 alpha 5.97 -> 6.09 ms,
    // profiles/r2s)
    const int bx = blockIdx.x, by = blockIdx.y;
    const int bw = batches[by];
    const int p0 = bw & 0xffffff, nb = (int)((unsigned)bw >> 24);   // tables p0 .. p0 + nb - 1
    const unsigned tu = (unsigned)tiles[bx];                         // tile word, as in k_alpha_tile
    const int half = (tu >> 28) & 3, nhalf = (tu >> 30) & 3;
    const int n0 = (tu & 0x3fff) * kAlphaTile + (nhalf == 2 ? 8 : 0);
    const int m0 = ((tu >> 14) & 0x3fff) * kAlphaTile + (half == 2 ? 8 : 0);
    const int mcnt = half == 0 ? kAlphaTile : (half == 1 ? 8 : kAlphaTile - 8);
    const int ncnt = nhalf == 0 ? kAlphaTile : (nhalf == 1 ? 8 : kAlphaTile - 8);
    const int Tm = (m0 + mcnt < T) ? m0 + mcnt : T;
    const int Tn = (n0 + ncnt < T) ? n0 + ncnt : T;
    const Point& P = pts[p0];
    if (tid < 2 * kAlphaTile) {
        const int side = tid / kAlphaTile, j = tid - side * kAlphaTile, b = (side ? m0 : n0) + j;
        if (b < (side ? Tm : Tn)) { elo[side][j] = g.lo[b]; ehi[side][j] = g.hi[b]; }
    }
    __syncthreads();
    if (tid == 0) cnt[0] = alpha_edge_list(elo[0], ehi[0], 0, Tn - n0, tE, tl, th);
    if (tid == 64) cnt[1] = alpha_edge_list(elo[1], ehi[1], 0, Tm - m0, sE, sl, sh);
    __syncthreads();
    const int ct = cnt[0], cs = cnt[1], cc = cs * ct;
    __shared__ int tsrc[2 * kAlphaTile], ssrc[2 * kAlphaTile];   // bin edge (2 b + side) behind each list slot
    if (tid < 2 * kAlphaTile) {
        const int side = tid / kAlphaTile, j = tid - side * kAlphaTile, b0 = side ? m0 : n0;
        const int* il = side ? sl : tl;
        const int* ih = side ? sh : th;
        int* src = side ? ssrc : tsrc;
        if (b0 + j < (side ? Tm : Tn)) {
            src[ih[j]] = 2 * (b0 + j) + 1;
            if (j == 0 || il[j] != ih[j - 1]) src[il[j]] = 2 * (b0 + j);   // else the previous bin's upper edge
        }
    }
    const int ln = tid % kAlphaTile, lm = tid / kAlphaTile;
    const int n = n0 + ln, m = m0 + lm;
    const bool valid = tid < kAlphaTile * kAlphaTile && n < m && m < Tm && n < Tn;
    const size_t eidx = (size_t)m * (m - 1) / 2 + n;
    if (cs > kAlphaTile + 1 || ct > kAlphaTile + 1) {   // host classification guarantees this never happens
        if (valid)
            for (int q = 0; q < nb; ++q) A[(size_t)(p0 + q) * g.PT + eidx] = __builtin_nan("");
        return;
    }
    const bool nonres = P.non_resonant, maj = P.majorana, cornered = nonres && maj;
    const bool needed = valid && (nonres || m == n + 1);
    constexpr int ccmax = kCC;
    double* P3 = sm;                           // [3][cc]
    double* X = P3 + 3 * ccmax;                // [kXFields][cc] | LL TU1 TU2 G [4][cc] + mixed
    double* mem = X + kXFields * ccmax;        // [2][cc] (kBatchPipe: [2][2][cc], by point parity)
    double* edgk = mem + (kBatchPipe ? 4 : 2) * ccmax;   // [estride]
    double* membq = edgk + alpha_tile_edge_stride(kAlphaTile + 1, kAlphaTile + 1);   // [kBatchQC][mbd]
    const int mbd = alpha_batch_memb_doubles(cs, ct);
    double* tmp = X;
    double* mix = X + 4 * kCC;
    const int mjobs = ct + cs + kAlphaTile;
    int wsh = 0;
    const int kb = kSplit ? (int)blockIdx.z : kOneK ? kone : 0, ke = (kSplit || kOneK) ? kb + 1 : 3;
#ifdef NUSI_BATCH_TRACE
    int bt_i = 0;
#endif
#pragma unroll 1
    for (int k = kb; k < ke; ++k) {
        NUSI_BT();
        __syncthreads();   // the previous k's points are done with P3, X, mem, edgk, membq
        if (tid < mjobs) alpha_tile_edge_job_k(P, k, tid, tE, ct, sE, cs, g.lo, g.hi, m0, Tm, edgk);
        __syncthreads();
        NUSI_BT();
        // ---- the batch's shared leaves and brackets of mass state k
        AlphaPre pre{};
        PPTerm ppt{0.0, 1.0, 1.0};
        if (cornered) {
            for (int j = tid; j < cc; j += kTileThreads) b_corner<kRef>(j, edgk, ct, cs, P3, tmp);
            for (int j = tid; j < kAlphaTile * (cs + ct); j += kTileThreads)
                alpha_batch_mixed_job(j, edgk, ct, cs, tl, th, sl, sh, n0, m0, T, Tm, mix, mix + kAlphaTile * cs);
            __syncthreads();
            NUSI_BT();
            if (needed) {
                pre = b_pre(P, k, g.lo[n], g.hi[n], g.lo[m], g.hi[m], P3, tmp, mix, edgk, cs, ct, lm, ln, sl[lm], sh[lm],
                            tl[ln], th[ln]);
                if (kPP) {
                    const SplitLeaves lv = batch_bracket_leaves(P3, tmp, mix, edgk, cs, ct, lm, ln, sl[lm], sh[lm],
                                                                tl[ln], th[ln]);
                    ppt = alpha_k_pp(P, spl, k, g.lo[n], g.hi[n], g.lo[m], g.hi[m], lv, wsh);
                }
            }
            __syncthreads();   // X is rewritten with the member coefficients (kRef: with the member corners)
            NUSI_BT();
            if (!kRef)
                for (int j = tid; j < cc; j += kTileThreads) b_xshared(j, edgk, ct, cs, X);
        }
        // ---- the points, kBatchQC at a time: their member edge leaves in one round, then point by point.
        // (Two points per pair of barriers -- 512-thread workgroups whose halves share the batch's leaves -- measured
        // slower too: C4 alpha 8.0 ms, profiles/r3/r3u.)
        // (Each wave owning 4 m rows of the tile, with its own block of member corners and no workgroup barrier in
        // the point loop, measured slower: C4 alpha 9.6 ms, the per-wave corner rows and the values live across the
        // loop spill at 4 waves per SIMD, 6.7 ms at 3; profiles/r3/r3q.)
        // A point's entry accumulates over the mass states in A; the sum of the states < k is loaded one
        // point ahead (timed equal to loading it in place, profiles/r2m: four blocks per CU already hide it).
        const bool reload = !kSplit && k > 0 && needed;
        double tnext = reload ? A[(size_t)p0 * g.PT + eidx] : 0.0;
        // member edges: thread (mq, mjob) copies job mjob of point mq of each chunk (loading the next chunk's
        // values a chunk ahead measured slower: their registers stay live through the combine)
        const int mq = tid / mjobs, mjob = tid - mq * mjobs;
        // (kRef) thread tid < cc carries corner tid's member leaves one point ahead, from k_alpha_mcorner's block:
        // the corner's numbering c (only corners with ut <= us are read by the entries n < m; the others stay unset)
        const double2* const mcb =   // (uniform: the block of this batch and mass state, [q][c] of (Dcr, Dci))
            kRef ? reinterpret_cast<const double2*>(mc.buf + (size_t)(p0 - pc0) * 6 * mc.NC + (size_t)k * 2 * nb * mc.NC)
                 : nullptr;
        int moff = -1;   // this thread's corner c, or -1 (point q's pair at q NC + c)
        double2 mcv = make_double2(0.0, 0.0);
        if (kRef && cornered && tid < cc) {
            const int si = tid / ct, ti = tid - si * ct;
            const int us = mc.eu[ssrc[si]], ut = mc.eu[tsrc[ti]];
            if (ut <= us) {
                moff = us * (us + 1) / 2 + ut;
                if (kRefPrefetch && !(NUSI_REFO_BSTUB & 2)) mcv = mcb[moff];
            }
        }
#pragma unroll 1
        for (int q0 = 0; q0 < nb; q0 += kBatchQC) {
            const int nq = (nb - q0 < kBatchQC) ? nb - q0 : kBatchQC;
            __syncthreads();   // the previous chunk is done with membq (and mem)
            NUSI_BT();
            if (mq < nq) {
                MedVals mv{};
                alpha_batch_medge_load(nonres, mjob, tsrc, ct, ssrc, cs, m0, Tm, T,
                                       med + ((size_t)(p0 + q0 + mq) * 3 + k) * kMedFields * T, mv);
                alpha_batch_medge_store(nonres, mjob, ct, cs, m0, Tm, mv, membq + mq * mbd);
            }
            // (kRef) A of this thread's corner for the chunk's points, into X's fields 3 .. 3 + nq - 1 (free in the
            // point loop): the reference's carg of the member quotient, out of the per-point phases (formed per point
            // between their barriers, out of line, it cost 1.23 ms of C4's 7.96; here 7.28 ms in all, profiles/r5/r6p)
            if (kRef && moff >= 0) {
                const int si = tid / ct, ti = tid - si * ct;
                const double S = edgk[kTEdgeFields * ct + kSEdgeVal * cs + si], t = edgk[kTEdgeVal * ct + ti];
#pragma unroll 1
                for (int qq = 0; qq < nq; ++qq)   // (inline: C4 7.42 -> 7.28 ms, r6p; kPP, whose point loop holds
                    X[(3 + qq) * kCC + tid] =     // the phi-phi term too, as a call: C3 12.33 -> 11.24 ms, r6q)
                        (NUSI_REFO_BSTUB & 4) ? S + t : kPP ? b_marg(S, t, pts[p0 + q0 + qq].a_gr)
                                                            : alpha_member_ref_arg(S, t, pts[p0 + q0 + qq].a_gr);
            }
            constexpr bool pipe = kBatchPipe && !kRef;
            NUSI_BT();
            if (pipe) {
                __syncthreads();   // member edges written
                if (cornered)
                    for (int j = tid; j < cc; j += kTileThreads)
                        alpha_batch_mcorner_job(pts[p0 + q0], j, edgk, ct, cs, X, membq, mem);
            }
#pragma unroll 1
            for (int qq = 0; qq < nq; ++qq) {
                const int q = q0 + qq;
                const Point& Q = pts[p0 + q];
                const double* memb = membq + qq * mbd;
                double tot = tnext;   // after states < k
                if (reload && q + 1 < nb) tnext = A[(size_t)(p0 + q + 1) * g.PT + eidx];
                double* memq = mem;
                if (pipe) {
                    memq = mem + (qq & 1) * 2 * ccmax;
                    __syncthreads();   // mem of q written / the previous point's combine is done with the other buffer
                    if (cornered && qq + 1 < nq)
                        for (int j = tid; j < cc; j += kTileThreads)
                            alpha_batch_mcorner_job(pts[p0 + q + 1], j, edgk, ct, cs, X, memb + mbd,
                                                    mem + ((qq + 1) & 1) * 2 * ccmax);
                } else {
                    __syncthreads();   // member edges written / the previous point's combine is done with mem
                    NUSI_BT();
                    if (cornered) {
                        if (kRef) {
                            if (moff >= 0) {
                                const size_t o = (size_t)q * mc.NC + moff;
                                if (!kRefPrefetch) mcv = mcb[o];
                                X[tid] = mcv.x; X[kCC + tid] = mcv.y;
                                if (kRefPrefetch && q + 1 < nb && !(NUSI_REFO_BSTUB & 2)) mcv = mcb[o + mc.NC];
                            }
                        }
                        else
                            for (int j = tid; j < cc; j += kTileThreads) alpha_batch_mcorner_job(Q, j, edgk, ct, cs, X, memb, mem);
                    }
                    __syncthreads();   // mem of q written
                    NUSI_BT();
                }
                int w = 0;
                TermRec rec;
                if (needed && !(kRef && (NUSI_REFO_BSTUB & 8))) {
                    SplitLeavesT<kRef> lv;
                    lv.cf[0] = P3; lv.cf[1] = P3; lv.cf[2] = P3; lv.cf[3] = P3; lv.cf[4] = P3;
                    lv.cf[5] = P3 + kCC; lv.cf[6] = P3 + 2 * kCC;   // (LL, TU1, TU2, G are not read with pre)
                    lv.corm = kRef ? X : memq;
                    lv.cc = cc; lv.ct = ct; lv.cs = cs; lv.mb = lm; lv.nb = ln;
                    lv.sidx[0] = sl[lm]; lv.sidx[1] = sh[lm]; lv.tidx[0] = tl[ln]; lv.tidx[1] = th[ln];
                    lv.ted = edgk; lv.sed = edgk + kTEdgeFields * ct; lv.mbv = lv.sed + kSEdgeFields * cs;
                    lv.tedm = memb; lv.sedm = memb + ct; lv.mbm = memb + ct + 2 * cs;
                    lv.marg = kRef ? X + (3 + qq) * kCC : memb + ct + 2 * cs + kAlphaTile + 2 * ct;   // sT | fT | sS | fS
                    lv.xl = mix; lv.yl = mix;   // (not read with pre)
                    if (kSplit)
                        alpha_k<SplitLeavesT<kRef>, kPP>(Q, spl, k, g.lo[n], g.hi[n], g.lo[m], g.hi[m], lv, rec, w,
                                                         cornered ? &pre : nullptr, kPP && cornered ? &ppt : nullptr);
                    else
                        alpha_k<SplitLeavesT<kRef>, kPP>(Q, spl, k, g.lo[n], g.hi[n], g.lo[m], g.hi[m], lv, tot, w,
                                                         cornered ? &pre : nullptr, kPP && cornered ? &ppt : nullptr);
                }
                if (kSplit) {
                    if (valid) {
                        double* o = kt + ((((size_t)(p0 + q) * 3 + k) * g.PT + eidx) << 3);
#pragma unroll
                        for (int j = 0; j < 7; ++j) o[j] = rec.v[j];
                        o[7] = needed ? (double)rec.n : -1.0;
                    }
                } else if (valid) A[(size_t)(p0 + q) * g.PT + eidx] = needed ? tot : 0.0;
                if (w) warn_entry(warn, wmin, T, p0 + q, w, n, m);
                NUSI_BT();
            }
        }
    }
    if (wsh)   // (the batch-shared phi-phi term of this thread's entry)
        for (int q = 0; q < nb; ++q) warn_entry(warn, wmin, T, p0 + q, wsh, n, m);
}

// The k-split path's sums (k_alpha_batch<.., kSplit>): every class-0 entry of the batches' tables, its mass states'
// recorded terms added in order from 0.0 -- k_alpha_batch's own additions (tot starts at 0.0 for k = 0 and at the
// previous states' sum after), so the same bits; 0.0 for entries a resonant-only table does not compute.  Grid and
// tile decode as k_alpha_batch's
__global__ __launch_bounds__(kTileThreads) void k_alpha_ksum(GridDev g, const int* __restrict__ tiles,
                                                             const int* __restrict__ batches, const double* __restrict__ kt,
                                                             double* __restrict__ A)
{
    const int tid = threadIdx.x, T = g.T;
    const int bw = batches[blockIdx.y];
    const int p0 = bw & 0xffffff, nb = (int)((unsigned)bw >> 24);
    const unsigned tu = (unsigned)tiles[blockIdx.x];
    const int half = (tu >> 28) & 3, nhalf = (tu >> 30) & 3;
    const int n0 = (tu & 0x3fff) * kAlphaTile + (nhalf == 2 ? 8 : 0);
    const int m0 = ((tu >> 14) & 0x3fff) * kAlphaTile + (half == 2 ? 8 : 0);
    const int mcnt = half == 0 ? kAlphaTile : (half == 1 ? 8 : kAlphaTile - 8);
    const int ncnt = nhalf == 0 ? kAlphaTile : (nhalf == 1 ? 8 : kAlphaTile - 8);
    const int Tm = (m0 + mcnt < T) ? m0 + mcnt : T, Tn = (n0 + ncnt < T) ? n0 + ncnt : T;
    const int n = n0 + tid % kAlphaTile, m = m0 + tid / kAlphaTile;
    if (!(tid < kAlphaTile * kAlphaTile && n < m && m < Tm && n < Tn)) return;
    const size_t eidx = (size_t)m * (m - 1) / 2 + n;
    for (int q = 0; q < nb; ++q) {
        double tot = 0.0;
        bool skip = false;
        for (int k = 0; k < 3; ++k) {
            const double* o = kt + ((((size_t)(p0 + q) * 3 + k) * g.PT + eidx) << 3);
            const int cnt = (int)o[7];
            if (cnt < 0) skip = true;
            for (int j = 0; j < cnt; ++j) tot += o[j];
        }
        A[(size_t)(p0 + q) * g.PT + eidx] = skip ? 0.0 : tot;
    }
}

// NUSI_OPT_SHIFT_REUSE: table slot s0 + q <- base table map[q].x of the extended axis (Tb bins),
// read map[q].y = o bins higher.  A copy, HBM-bound: 2 x 8 B per entry.  The slot reads the base's entries (n', m')
// with o <= n' <= m' <= T - 1 + o, so it takes warning bit b iff some row n' in [o, T + o) has an entry of column
// <= T - 1 + o that raised it (tb.Wmin, the base's row records): the bits of the base's bins outside the slot's
// range -- below o and above T - 1 + o -- are not passed on.
__global__ __launch_bounds__(256) void k_table_shift(int T, long long PT, int Tb, long long PTb, const int2* __restrict__ map,
                                                     int s0, TablesDev tb, TablesDev t, int* __restrict__ warn)
{
    const int q = blockIdx.y, s = s0 + q;
    const int bi = map[q].x, o = map[q].y;
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    if (e < T) {
        t.G[(size_t)s * T + e] = tb.G[(size_t)bi * Tb + e + o];
        t.At[(size_t)s * T + e] = tb.At[(size_t)bi * Tb + e + o];
        int bits = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if (tb.Wmin[((size_t)bi * 4 + b) * Tb + e + o] <= T - 1 + o) bits |= 1 << b;
        if (bits) atomicOr(&warn[s], bits);
    }
    if (e >= PT) return;
    int m = (int)((1.0 + sqrt(1.0 + 8.0 * (double)e)) * 0.5);   // packed index e = m (m - 1) / 2 + n, n < m
    while ((long long)m * (m - 1) / 2 > e) --m;
    while ((long long)(m + 1) * m / 2 <= e) ++m;
    const long long n = e - (long long)m * (m - 1) / 2, mb = m + o;
    t.A[(size_t)s * PT + e] = tb.A[(size_t)bi * PTb + mb * (mb - 1) / 2 + n + o];
}

hipError_t launch_table_shift(const GridDev& g, const GridDev& gb, const int2* map, int s0, int nshift, TablesDev tb,
                              TablesDev t, int* warn, hipStream_t s)
{
    if (nshift <= 0) return hipSuccess;
    if (!tb.Wmin) return hipErrorInvalidValue;
    const long long ne = std::max<long long>(g.PT, g.T);
    hipLaunchKernelGGL(k_table_shift, dim3((unsigned)((ne + 255) / 256), nshift), dim3(256), 0, s, g.T, g.PT, gb.T, gb.PT,
                       map, s0, tb, t, warn);
    return hipGetLastError();
}

hipError_t alpha_tiles_create(int T, const unsigned char* shared, AlphaTilesDev* out)
{
    const int nt = (T + kAlphaTile - 1) / kAlphaTile;
    // distinct edges of each tile side, exactly as alpha_edge_list counts them on the device
    std::vector<int> ne(nt, 0);
    for (int t = 0; t < nt; ++t)
        for (int j = t * kAlphaTile; j < (t + 1) * kAlphaTile && j < T; ++j)
            ne[t] += (j > t * kAlphaTile && shared[j - 1]) ? 1 : 2;
    // class 0: both sides <= 16 edges; 1: t side <= 16, S' side <= 30; 2: both <= 30.  From the
    // first tile t0 whose bins do not share edges (the redshift-extended bins) on, tiles of class 2
    // save no corner (4 per entry, like the per-entry path) and their 80-KB LDS footprint halves the
    // occupancy: the bins [15 t0, T) x [15 t0, T) go to the per-entry kernel instead (ext_lo).
    const int cap_core = kAlphaTile + 1, cap_ext = 2 * kAlphaTile;
    int t0 = nt;
    for (int t = 0; t < nt; ++t)
        if (ne[t] > cap_core) { t0 = t; break; }
    bool tail_ext = true;   // no bin from tile t0 on shares an edge with its neighbour
    for (int n = t0 * kAlphaTile; n + 1 < T; ++n) tail_ext = tail_ext && !shared[n];
    // the extended triangle runs as quarter tiles (8 x 8 bins, batched with the core tiles; round 1: alpha
    // stage 14.68 -> 14.55 ms per 1024 points against the per-entry kernel)
    constexpr bool ext_tiles = true;
    out->ext_lo = (tail_ext && t0 < nt && !ext_tiles) ? t0 * kAlphaTile : T;
    const int qlo = (tail_ext && t0 < nt && ext_tiles) ? t0 : nt;   // tiles from qlo on: split on both sides
    // Class-1 tiles (t side core, S' side extended: 30 S' edges) are split into their first 8 and last
    // 7 m bins (16 / 14 S' edges): the halves fit the core tiles' LDS footprint and join class 0,
    // whose launch builds batches of tables (16.0 -> 14.8 ms when introduced).
    constexpr bool split_ext = true;
    std::vector<int> cls[3];
    for (int tm = 0; tm < nt; ++tm)
        for (int tn = 0; tn <= tm; ++tn) {
            const int c = (ne[tn] <= cap_core && ne[tm] <= cap_core) ? 0 : (ne[tn] <= cap_core) ? 1 : 2;
            if (tn * kAlphaTile >= out->ext_lo) continue;   // per-entry region
            const int w = tn | (tm << 14);
            if (tn >= qlo) {   // both sides extended: up to 4 quarter tiles (n half, m half)
                for (int nh = 1; nh <= 2; ++nh)
                    for (int mh = 1; mh <= 2; ++mh) {
                        const int nb0 = tn * kAlphaTile + (nh == 2 ? 8 : 0), mb0 = tm * kAlphaTile + (mh == 2 ? 8 : 0);
                        const int mb1 = std::min(T, tm * kAlphaTile + (mh == 1 ? 8 : kAlphaTile));
                        if (nb0 >= T || mb0 >= T || nb0 >= mb1 - 1) continue;   // no entry n < m
                        cls[0].push_back((int)((unsigned)w | ((unsigned)mh << 28) | ((unsigned)nh << 30)));
                    }
            } else if (c == 1 && split_ext && tn < tm) {
                cls[0].push_back(w | (1 << 28));
                if (tm * kAlphaTile + 8 < T) cls[0].push_back(w | (2 << 28));
            } else {
                cls[c].push_back(w);
            }
        }
    const int csm[3] = {cap_core, cap_ext, cap_ext}, ctm[3] = {cap_core, cap_core, cap_ext};
    std::vector<int> all;
    for (int c = 0; c < 3; ++c) {
        out->ncls[c] = (int)cls[c].size();
        out->cs_max[c] = csm[c];
        out->ct_max[c] = ctm[c];
        all.insert(all.end(), cls[c].begin(), cls[c].end());
    }
    hipError_t e = hipMalloc(&out->tiles, sizeof(int) * all.size());
    if (e != hipSuccess) return e;
    return hipMemcpy(out->tiles, all.data(), sizeof(int) * all.size(), hipMemcpyHostToDevice);
}

void alpha_tiles_destroy(AlphaTilesDev* t)
{
    if (t->tiles) (void)hipFree(t->tiles);
    t->tiles = nullptr;
}

static thread_local const char* t_alpha_kernel = "";   // the main kernel of the latest launch on this thread
const char* last_alpha_kernel() { return t_alpha_kernel; }

template <bool kRef>
static hipError_t launch_alpha_t(const GridDev& g, const Point* pts, int npts, const SplineSet* spl,
                                 const AlphaTilesDev& at, TablesDev t, int* warn, hipStream_t s, const int* batches,
                                 int nbatches, int gmax, int kernel, int nb_plain, const int* h_batches,
                                 const MCornerDev* mc)
{
    t_alpha_kernel = kRef ? "k_alpha_tile[refo]" : "k_alpha_tile";
    if (kernel == 0 && batches) {
        t_alpha_kernel = kRef ? "k_alpha_mcorner + k_alpha_batch[refo]" : "k_alpha_batch";
        // class 0 on the big-batch kernel (batches of up to gmax tables), classes 1 / 2 per table
        if (at.ext_lo < g.T) {
            const long long L = g.T - at.ext_lo, ne = L * (L - 1) / 2;
            hipLaunchKernelGGL(k_alpha<kRef>, dim3((unsigned)((ne + 255) / 256), npts), dim3(256), 0, s, g, pts, spl,
                               at.ext_lo, t.A, warn, t.Wmin);
        }
        int off = 0;
        for (int c = 0; c < 3; ++c) {
            if (at.ncls[c] == 0) continue;
            const int cs = at.cs_max[c], ct = at.ct_max[c];
            if (c == 0) {   // batches [0, nb_plain) without the phi-phi channel, then those with it
                const size_t lds = sizeof(double) * (size_t)alpha_batch_lds_doubles();
                if (cs > kAlphaTile + 1 || ct > kAlphaTile + 1) return hipErrorInvalidValue;
                {
                    if (!t.Med) return hipErrorInvalidValue;
                    hipLaunchKernelGGL(k_alpha_medge, dim3((unsigned)((5 * g.T + 255) / 256), npts, 3), dim3(256), 0, s,
                                       g, pts, t.Med);
                }
                // (NUSI_BATCH_KLAUNCH: the non-phi-phi batches as three launches, one per mass state)
                // t.Kt (calls of few tables, no phi-phi channel): the k-split instance, its mass states' workgroups at
                // once, and k_alpha_ksum's ordered sums
                const bool split = t.Kt && nb_plain == nbatches;
                if (!kRef) {
                    if (split) {
                        hipLaunchKernelGGL((k_alpha_batch<false, false, true>), dim3(at.ncls[0], nbatches, 3),
                                           dim3(kTileThreads), lds, s, g, pts, spl, at.tiles, batches, t.A, t.Med, warn,
                                           t.Wmin, MCornerDev{}, 0, t.Kt);
                        hipLaunchKernelGGL(k_alpha_ksum, dim3(at.ncls[0], nbatches), dim3(kTileThreads), 0, s, g, at.tiles,
                                           batches, t.Kt, t.A);
                    } else if (nb_plain > 0 && kBatchKLaunch) {
                        for (int kk = 0; kk < 3; ++kk)
                            hipLaunchKernelGGL((k_alpha_batch<false, false, false, true>), dim3(at.ncls[0], nb_plain),
                                               dim3(kTileThreads), lds, s, g, pts, spl, at.tiles, batches, t.A, t.Med, warn,
                                               t.Wmin, MCornerDev{}, 0, nullptr, kk);
                    } else if (nb_plain > 0)
                        hipLaunchKernelGGL((k_alpha_batch<false, false>), dim3(at.ncls[0], nb_plain), dim3(kTileThreads),
                                           lds, s, g, pts, spl, at.tiles, batches, t.A, t.Med, warn, t.Wmin, MCornerDev{}, 0, nullptr);
                    if (nbatches > nb_plain)
                        hipLaunchKernelGGL((k_alpha_batch<true, false>), dim3(at.ncls[0], nbatches - nb_plain),
                                           dim3(kTileThreads), lds, s, g, pts, spl, at.tiles, batches + nb_plain, t.A,
                                           t.Med, warn, t.Wmin, MCornerDev{}, 0, nullptr);
                } else {
                    // the member corners of a chunk of whole batches (<= mc->cap_tables tables, the phi-phi batches
                    // in chunks of their own), then the chunk's tiles.  (k_alpha_mcorner of chunk c + 1 on a second
                    // stream beside k_alpha_batch of chunk c, in two halves of the block, measured no gain: C4 18.25
                    // -> 18.26 ms, the two kernels' workgroups sharing the CUs each ran slower by the other's share.)
                    if (!mc || !mc->buf || !h_batches) return hipErrorInvalidValue;
                    for (int b = 0; b < nbatches;) {
                        const int lim = b < nb_plain ? nb_plain : nbatches, pc0 = h_batches[b] & 0xffffff;
                        int e = b, ntb = 0, nbmax = 0;
                        while (e < lim) {
                            const int nbe = (int)((unsigned)h_batches[e] >> 24);
                            if (e > b && ntb + nbe > mc->cap_tables) break;
                            ntb += nbe;
                            nbmax = std::max(nbmax, nbe);
                            ++e;
                        }
                        if (ntb > mc->cap_tables) return hipErrorInvalidValue;
                        // jobs per workgroup: 4 per work-item on scans, 1 when the chunk is too small to fill ~2048
                        // workgroups (a single propagation: one GSL call per work-item, not four in a row)
                        const long long tot = mc->NC * 3 * ntb;
                        const int jobs = 256 * (int)std::max(1LL, std::min<long long>(kMcJobs / 256, tot / (2048 * 256)));
                        const int cbmin = jobs / nbmax;
                        hipLaunchKernelGGL(k_alpha_mcorner, dim3((unsigned)((mc->NC + cbmin - 1) / cbmin), e - b, 3),
                                           dim3(256), 0, s, pts, batches + b, *mc, pc0, jobs);
                        if (split) {
                            hipLaunchKernelGGL((k_alpha_batch<false, true, true>), dim3(at.ncls[0], e - b, 3),
                                               dim3(kTileThreads), lds, s, g, pts, spl, at.tiles, batches + b, t.A, t.Med,
                                               warn, t.Wmin, *mc, pc0, t.Kt);
                            hipLaunchKernelGGL(k_alpha_ksum, dim3(at.ncls[0], e - b), dim3(kTileThreads), 0, s, g,
                                               at.tiles, batches + b, t.Kt, t.A);
                        } else if (b < nb_plain && kBatchKLaunch) {
                            for (int kk = 0; kk < 3; ++kk)
                                hipLaunchKernelGGL((k_alpha_batch<false, true, false, true>), dim3(at.ncls[0], e - b),
                                                   dim3(kTileThreads), lds, s, g, pts, spl, at.tiles, batches + b, t.A,
                                                   t.Med, warn, t.Wmin, *mc, pc0, nullptr, kk);
                        } else if (b < nb_plain)
                            hipLaunchKernelGGL((k_alpha_batch<false, true>), dim3(at.ncls[0], e - b), dim3(kTileThreads),
                                               lds, s, g, pts, spl, at.tiles, batches + b, t.A, t.Med, warn, t.Wmin, *mc,
                                               pc0, nullptr);
                        else
                            hipLaunchKernelGGL((k_alpha_batch<true, true>), dim3(at.ncls[0], e - b), dim3(kTileThreads),
                                               lds, s, g, pts, spl, at.tiles, batches + b, t.A, t.Med, warn, t.Wmin, *mc,
                                               pc0, nullptr);
                        b = e;
                    }
                }
            } else {
                const size_t lds = sizeof(double) * (size_t)alpha_tile_lds_doubles(cs, ct, 1);
                hipLaunchKernelGGL((k_alpha_tile<1, kRef>), dim3(at.ncls[c], npts), dim3(kTileThreads), lds, s, g, pts,
                                   spl, at.tiles + off, cs, ct, nullptr, t.A, warn, t.Wmin);
            }
            off += at.ncls[c];
        }
        return hipGetLastError();
    }
    const bool per_entry = kernel == 2;
    auto per_entry_region = [&](int nlo) {
        const long long L = g.T - nlo, ne = L * (L - 1) / 2;
        if (ne <= 0) return;
        dim3 grid((unsigned)((ne + 255) / 256), npts);
        hipLaunchKernelGGL(k_alpha<kRef>, grid, dim3(256), 0, s, g, pts, spl, nlo, t.A, warn, t.Wmin);
    };
    if (per_entry) {
        t_alpha_kernel = kRef ? "k_alpha[refo]" : "k_alpha";
        per_entry_region(0);
        return hipGetLastError();
    }
    per_entry_region(at.ext_lo);
    int off = 0;
    for (int c = 0; c < 3; ++c) {
        if (at.ncls[c] == 0) continue;
        const int cs = at.cs_max[c], ct = at.ct_max[c];
        // class 0 (core tiles) runs on batches of tables sharing their (S', t) leaves; the others per table
        // (batching class 1 too measured slower: its LDS then allows 2 workgroups/CU, profiles/r1l).  The
        // reference-order mode takes this kernel one table per workgroup (its A/B role needs no batches).
        const bool batched = !kRef && c == 0 && batches && gmax > 1;
        const int G = batched ? (gmax < 4 ? gmax : 4) : 1;
        const size_t lds = sizeof(double) * (size_t)alpha_tile_lds_doubles(cs, ct, G);
        const dim3 grid(at.ncls[c], batched ? nbatches : npts), blk(kTileThreads);
        const int* bt = batched ? batches : nullptr;
        if (kRef) {
            hipLaunchKernelGGL((k_alpha_tile<1, true>), grid, blk, lds, s, g, pts, spl, at.tiles + off, cs, ct, bt, t.A,
                               warn, t.Wmin);
        } else {
            switch (G) {
            case 1: hipLaunchKernelGGL((k_alpha_tile<1, false>), grid, blk, lds, s, g, pts, spl, at.tiles + off, cs, ct, bt, t.A, warn, t.Wmin); break;
            case 2: hipLaunchKernelGGL((k_alpha_tile<2, false>), grid, blk, lds, s, g, pts, spl, at.tiles + off, cs, ct, bt, t.A, warn, t.Wmin); break;
            case 3: hipLaunchKernelGGL((k_alpha_tile<3, false>), grid, blk, lds, s, g, pts, spl, at.tiles + off, cs, ct, bt, t.A, warn, t.Wmin); break;
            default: hipLaunchKernelGGL((k_alpha_tile<4, false>), grid, blk, lds, s, g, pts, spl, at.tiles + off, cs, ct, bt, t.A, warn, t.Wmin); break;
            }
        }
        off += at.ncls[c];
    }
    return hipGetLastError();
}

hipError_t launch_alpha(const GridDev& g, const Point* pts, int npts, const SplineSet* spl, const AlphaTilesDev& at,
                        TablesDev t, int* warn, hipStream_t s, const int* batches, int nbatches, int gmax,
                        int kernel, int nb_plain, bool ref, const int* h_batches, const MCornerDev* mc)
{
    if (ref)
        return launch_alpha_t<true>(g, pts, npts, spl, at, t, warn, s, batches, nbatches, gmax, kernel, nb_plain,
                                    h_batches, mc);
    return launch_alpha_t<false>(g, pts, npts, spl, at, t, warn, s, batches, nbatches, gmax, kernel, nb_plain, h_batches,
                                 mc);
}

}  // namespace nusi

#ifdef NUSI_BATCH_TRACE
// diagnostic build: the batch kernel's phase stamps of the latest launch, [workgroup][wave][stamp]
extern "C" int nusi_debug_batch_trace(unsigned long long* out, int n)
{
    const int m = n < nusi::kBtWg * 4 * nusi::kBtN ? n : nusi::kBtWg * 4 * nusi::kBtN;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(nusi::g_bt), sizeof(unsigned long long) * m) == hipSuccess ? 0 : -5;
}
#endif
