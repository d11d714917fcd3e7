// nuSIprop MI355X -- HIP kernels for calculate_flux::evolve() (nuSIprop.hpp:176-337).
//
//   k_gamma_alphat  Stage A, absorption + same-bin regeneration tables   (:217-235)
//   k_alpha         Stage A, inter-bin regeneration table, one entry per
//                   work-item, packed transposed                          (:237-252)
//   (Stage B, the cascade, is in nusi_cascade.hip)
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

}  // namespace nusi
