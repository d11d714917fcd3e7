// nuSIprop MI355X -- device evaluator for interp::spline_ND<N> (interp.hpp:13-638).
//
// The phi-phi regeneration tables (xsec/alphatilde_phiphi.bin, 2-D 5000x100;
// xsec/alpha_phiphi.bin, 3-D 1000x1000x100; x0 logarithmic, non-regular nodes)
// stay resident in HBM for the lifetime of a plan.  Node values are kept as
// float32 (exactly the file's bytes; the reference promotes them to double on
// load, interp.hpp:258-276, so the promoted values are identical); nodes and
// the 4x4 Hermite weights (interp.hpp:576-636) are fp64, computed on the host.
// eval() follows f_eval (interp.hpp:345-467): bounds check (the reference
// exits on a miss -- here eval returns false and the caller raises a warning
// bit that the host turns into an error), node search per axis, 3- or
// 4-point stencil, tensor product summed with axis 0 fastest.
//
// Node search.  The reference binary-searches every axis (isRegular = false,
// nuSIprop.hpp:168-169): 10 + 10 + 7 dependent loads per lookup, which made
// the phi-phi alpha table latency-bound at the real 1000x1000x100 geometry.
// Here each axis carries a guide table over 4 (n-1) equal buckets of its
// (log'd) range: gd[u] = the last node <= the bucket's lower end.  A query
// starts from the guide of the bucket BELOW its own (a valid lower bound even
// when the bucket index rounds up) and steps up while the next node is <= x0.
// The result is the last node <= x0 -- exactly the index the binary search
// returns on sorted nodes -- in one guide load and about two node loads.
// The 16 weights of node k sit together (wt[16 k + 4 a + b], one 128-B line).
// Without a guide (gd == nullptr) the reference's binary search runs.
//
// Windows (3-D table).  A lookup reads a 4 x 4 x 4 stencil: with the values
// in the file's order (last index fastest) that is 16 runs of 16 B, each in
// its own cache line, and at C3 these gathers were ~80 % of the alpha
// kernel's HBM traffic.  The plan therefore keeps, for every node
// (i0, i1, i2), the 4 x 4 window fw[16 node + 4 a1 + a2] = f[i0][i1 + a1][i2 + a2]
// (indices clamped at the table's end; those entries are never read): a
// lookup reads 4 aligned 64-B windows.  16 x the table (6.4 GB at
// {1000,1000,100}), built on the GPU from f at load.  The same floats are
// summed in the same order (axis 0 fastest), so the value is unchanged.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

#include "nusi_libm.hpp"

#ifndef NUSI_FN
#define NUSI_FN __host__ __device__ inline
#endif

namespace nusi {

constexpr int kSplMaxDim = 3;

struct SplineDev {
    int ndim = 0;
    int n[kSplMaxDim] = {0, 0, 0};
    const double* x[kSplMaxDim] = {nullptr, nullptr, nullptr};  // nodes, log'd where islog
    const double* w[kSplMaxDim] = {nullptr, nullptr, nullptr};  // w[i][16 node + 4 a + b]
    const int* gd[kSplMaxDim] = {nullptr, nullptr, nullptr};     // guide: gd[i][bucket], ng[i] buckets
    int ng[kSplMaxDim] = {0, 0, 0};
    double ginv[kSplMaxDim] = {0.0, 0.0, 0.0};                   // buckets per unit of the axis
    const float* f = nullptr;                                    // values, last index fastest
    const float* fw = nullptr;                                   // 3-D: 4 x 4 windows per node (or nullptr)
    int islog[kSplMaxDim + 1] = {0, 0, 0, 0};

    // the last node <= x0 (x[0] < x0 < x[n-1])
    NUSI_FN int search(int i, double x0) const
    {
        const double* xi = x[i];
        if (gd[i]) {
            int u = (int)((x0 - xi[0]) * ginv[i]) - 1;
            u = u < 0 ? 0 : (u >= ng[i] ? ng[i] - 1 : u);
            int kk = gd[i][u];
            while (xi[kk + 1] <= x0) ++kk;
            return kk;
        }
        int L = 0, R = n[i] - 1, kk = 0;
        while (L <= R) {
            const int m = (L + R) / 2;
            if (x0 < xi[m]) R = m - 1;
            else {
                kk = m;
                L = m + 1;
            }
        }
        return kk;
    }

    // ND = ndim (2: alphaTilde_phiphi, 3: alpha_phiphi) at compile time: every per-axis array is statically
    // indexed (registers, not the per-lane scratch a runtime dimension loop puts them in) and each descriptor
    // field is read once; the same operations in the same order as the reference's loops (interp.hpp:425-460)
    template <int ND>
    NUSI_FN bool eval(const double* x0in, double& out) const
    {
        double x0[ND], t[ND], fac[ND][4];
        int k[ND], lo[ND], cnt[ND];
#pragma unroll
        for (int i = 0; i < ND; ++i) {
            x0[i] = islog[i] ? nm::log(x0in[i]) : x0in[i];
            const double* xi = x[i];
            const int ni = n[i];
            if (x0[i] <= xi[0] || x0[i] >= xi[ni - 1]) {
                out = 0.0;
                return false;
            }
            const int kk = search(i, x0[i]);
            k[i] = kk;
            if (kk == 0) { lo[i] = 0; cnt[i] = 3; }
            else if (kk == ni - 2) { lo[i] = kk - 1; cnt[i] = 3; }
            else { lo[i] = kk - 1; cnt[i] = 4; }
            t[i] = (x0[i] - xi[kk]) / (xi[kk + 1] - xi[kk]);
        }
        // per-axis stencil factors (t^3 w0 + t^2 w1 + t w2 + w3), interp.hpp:453-454
#pragma unroll
        for (int i = 0; i < ND; ++i)
#pragma unroll
            for (int a = 0; a < 4; ++a)
                if (a < cnt[i]) {
                    const double* wk = w[i] + 16 * k[i] + 4 * a;
                    fac[i][a] = t[i] * t[i] * t[i] * wk[0] + (t[i] * t[i]) * wk[1] + t[i] * wk[2] + wk[3];
                } else {
                    fac[i][a] = 0.0;
                }
        double res = 0;   // the reference's order: axis 0 fastest (loops of 4 with guards: static indices)
        if constexpr (ND == 3) {
            if (fw) {
                struct alignas(16) F4 { float v[4]; };
                F4 win[4][4];   // win[idx0][a1].v[a2] = f[lo0 + idx0][lo1 + a1][lo2 + a2]
#pragma unroll
                for (int i0 = 0; i0 < 4; ++i0) {
                    const int r0 = lo[0] + (i0 < cnt[0] ? i0 : 0);
                    const F4* src = reinterpret_cast<const F4*>(fw + 16 * (((size_t)r0 * n[1] + lo[1]) * n[2] + lo[2]));
#pragma unroll
                    for (int a1 = 0; a1 < 4; ++a1) win[i0][a1] = src[a1];
                }
#pragma unroll
                for (int i2 = 0; i2 < 4; ++i2)
#pragma unroll
                    for (int i1 = 0; i1 < 4; ++i1)
#pragma unroll
                        for (int i0 = 0; i0 < 4; ++i0)
                            if (i2 < cnt[2] && i1 < cnt[1] && i0 < cnt[0]) {
                                double v = (double)win[i0][i1].v[i2];
                                v *= fac[0][i0];
                                v *= fac[1][i1];
                                v *= fac[2][i2];
                                res += v;
                            }
            } else {
#pragma unroll 1
                for (int i2 = 0; i2 < cnt[2]; ++i2)
#pragma unroll 1
                    for (int i1 = 0; i1 < cnt[1]; ++i1)
#pragma unroll
                        for (int i0 = 0; i0 < 4; ++i0)
                            if (i0 < cnt[0]) {
                                double v = (double)f[((long long)(lo[0] + i0) * n[1] + (lo[1] + i1)) * n[2] + (lo[2] + i2)];
                                v *= fac[0][i0];
                                v *= fac[1][i1];
                                v *= fac[2][i2];
                                res += v;
                            }
            }
        } else {
#pragma unroll
            for (int i1 = 0; i1 < 4; ++i1)
#pragma unroll
                for (int i0 = 0; i0 < 4; ++i0)
                    if (i1 < cnt[1] && i0 < cnt[0]) {
                        double v = (double)f[(long long)(lo[0] + i0) * n[1] + (lo[1] + i1)];
                        v *= fac[0][i0];
                        v *= fac[1][i1];
                        res += v;
                    }
        }
        out = islog[ND] ? nm::exp(res) : res;
        return true;
    }
};

struct SplineSet {
    SplineDev at;  // alphaTilde_phiphi, 2-D
    SplineDev a;   // alpha_phiphi, 3-D
};

}  // namespace nusi
