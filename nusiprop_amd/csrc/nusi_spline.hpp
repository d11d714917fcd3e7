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
// bit that the host turns into an error), binary search per axis, 3- or
// 4-point stencil, tensor product summed with axis 0 fastest.
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
    const double* w[kSplMaxDim] = {nullptr, nullptr, nullptr};  // w[i][(a*4+b)*n[i] + node]
    const float* f = nullptr;                                    // values, last index fastest
    int islog[kSplMaxDim + 1] = {0, 0, 0, 0};

    NUSI_FN bool eval(const double* x0in, double& out) const
    {
        double x0[kSplMaxDim];
        int k[kSplMaxDim], lo[kSplMaxDim], cnt[kSplMaxDim];
        double t[kSplMaxDim];
        for (int i = 0; i < ndim; ++i) {
            x0[i] = islog[i] ? nm::log(x0in[i]) : x0in[i];
            const double* xi = x[i];
            if (x0[i] <= xi[0] || x0[i] >= xi[n[i] - 1]) {
                out = 0.0;
                return false;
            }
            int L = 0, R = n[i] - 1, kk = 0;
            while (L <= R) {
                const int m = (L + R) / 2;
                if (x0[i] < xi[m]) R = m - 1;
                else {
                    kk = m;
                    L = m + 1;
                }
            }
            k[i] = kk;
            if (kk == 0) { lo[i] = 0; cnt[i] = 3; }
            else if (kk == n[i] - 2) { lo[i] = kk - 1; cnt[i] = 3; }
            else { lo[i] = kk - 1; cnt[i] = 4; }
            t[i] = (x0[i] - xi[kk]) / (xi[kk + 1] - xi[kk]);
        }
        // per-axis stencil factors (t^3 w0 + t^2 w1 + t w2 + w3), interp.hpp:453-454
        double fac[kSplMaxDim][4];
        for (int i = 0; i < ndim; ++i)
            for (int a = 0; a < cnt[i]; ++a) {
                const double* wi = w[i];
                const int ni = n[i], kk = k[i];
                fac[i][a] = t[i] * t[i] * t[i] * wi[(a * 4 + 0) * ni + kk] + (t[i] * t[i]) * wi[(a * 4 + 1) * ni + kk]
                            + t[i] * wi[(a * 4 + 2) * ni + kk] + wi[(a * 4 + 3) * ni + kk];
            }
        int idx[kSplMaxDim] = {0, 0, 0};
        double res = 0;
        for (;;) {
            long long off = 0;
            for (int i = 0; i < ndim; ++i) off = off * n[i] + (lo[i] + idx[i]);
            double v = (double)f[off];
            for (int i = 0; i < ndim; ++i) v *= fac[i][idx[i]];
            res += v;
            int p = 0;
            while (p < ndim && ++idx[p] == cnt[p]) {
                idx[p] = 0;
                ++p;
            }
            if (p == ndim) break;
        }
        out = islog[ndim] ? nm::exp(res) : res;
        return true;
    }
};

struct SplineSet {
    SplineDev at;  // alphaTilde_phiphi, 2-D
    SplineDev a;   // alpha_phiphi, 3-D
};

}  // namespace nusi
