// Development timing (not part of the product): gsl_cli2 (nusi_gsl.hpp, NUSI_OPT_REFERENCE_ORDER's complex
// dilogarithm) in isolation on the alpha table's member-corner quotients z = (1 + S + t) / (2 + t - i gr) of a C4-like
// scan (N_E = 300, lE 12 -> 17, Sum m = 0.1 NO; every corner of the unique bin edges for 11 m_phi x 8 g x 3 mass
// states), against the shared-algorithm cli2 -- in tile-like order, shuffled, and sorted by gsl_cli2_cost; the
// member-corner order (a batch's points fastest) as it is and with each workgroup's 1024 jobs sorted by cost.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I nusiprop_amd/csrc scripts/dev/gsl_bench.hip -o gsl_bench
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "nusi_math.hpp"

using namespace nusi;

template <int V>
__global__ __launch_bounds__(256) void kbench(const double2* __restrict__ z, double2* __restrict__ o, int n)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const cd r = V == 1 ? cli2(z[i].x, z[i].y) : gsl_cli2(z[i].x, z[i].y);
    o[i] = make_double2(r.r, r.i);
}

int main()
{
    const int N = 300;
    const double lEmin = 12, lEmax = 17, d = (lEmax - lEmin) / N;
    std::vector<double> E;
    for (int b = 0; b <= N; ++b) E.push_back(pow(10.0, lEmin + b * d));
    const double r = E[1] / E[0];
    const int Nz = (int)(log(1 + 5.0) / log(r) + 2);
    for (int i = 1; i < Nz - 1; ++i) { E.push_back(E[N - 1] * pow(r, i)); E.push_back(E[N] * pow(r, i)); }
    std::sort(E.begin(), E.end());
    const double mn[3] = {0.02183689, 0.02347445, 0.05468866};
    std::vector<double2> h, hp;   // point-major (tile-like) and corner-major, the batch's 32 points fastest
    for (int im = 0; im < 32; im += 3) {
        const double mphi = pow(10.0, 5.5 + 2.5 * im / 31.0);
        for (int ig = 0; ig < 32; ig += 4) {
            const double g = pow(10.0, -3.0 + 3.0 * ig / 31.0), gr = g * g / (16 * M_PI);
            for (int k = 0; k < 3; ++k)
                for (size_t a = 0; a < E.size(); ++a)          // t edge
                    for (size_t b = a + 1; b < E.size(); b += 4) {   // S edge (every 4th)
                        const double t = -2 * mn[k] * E[a] / (mphi * mphi), S = 2 * mn[k] * E[b] / (mphi * mphi);
                        const cd zz = (1 + S + t) / C(2 + t, -gr);
                        h.push_back(make_double2(zz.r, zz.i));
                    }
        }
        for (int k = 0; k < 3; ++k)
            for (size_t a = 0; a < E.size(); ++a)
                for (size_t b = a + 1; b < E.size(); b += 4)
                    for (int ig = 0; ig < 32; ++ig) {
                        const double g = pow(10.0, -3.0 + 3.0 * ig / 31.0), gr = g * g / (16 * M_PI);
                        const double t = -2 * mn[k] * E[a] / (mphi * mphi), S = 2 * mn[k] * E[b] / (mphi * mphi);
                        const cd zz = (1 + S + t) / C(2 + t, -gr);
                        hp.push_back(make_double2(zz.r, zz.i));
                    }
    }
    const int n = (int)h.size();
    std::vector<double2> hs = h, hr = h;
    std::sort(hs.begin(), hs.end(), [](const double2& x, const double2& y) {
        return gsl_cli2_cost(x.x, x.y) > gsl_cli2_cost(y.x, y.y);
    });
    std::shuffle(hr.begin(), hr.end(), std::mt19937(1));
    const int np = (int)hp.size();
    // the member-corner kernel's workgroup sets (1024 consecutive jobs of hp) sorted locally by cost, and in 16
    // cost buckets (a counting sort's order)
    std::vector<double2> hl = hp, hb = hp, hc = hp, hk = hp;
    auto cls = [](const double2& z) {   // GSL's branches: inversion, reflection, series_1 / series_2 / series_3
        const double x = z.x, y = z.y, r2 = x * x + y * y;
        if (y == 0.0) return 0;
        const bool inv = !(r2 < 1.0);
        const double ux = inv ? x / r2 : x, uy = inv ? -y / r2 : y;
        const bool refl = ux > 0.732;
        const double fx = refl ? 1.0 - ux : ux, r = sqrt(fx * fx + uy * uy);
        const int ser = r > 0.98 ? 2 : r > 0.25 ? 1 : 0;
        return 1 + ser + 3 * (refl + 2 * inv);
    };
    for (int s0 = 0; s0 < np; s0 += 1024) {
        const int s1 = std::min(np, s0 + 1024);
        auto cost = [](const double2& x) { return gsl_cli2_cost(x.x, x.y); };
        std::stable_sort(hl.begin() + s0, hl.begin() + s1, [&](const double2& x, const double2& y) { return cost(x) > cost(y); });
        std::stable_sort(hb.begin() + s0, hb.begin() + s1, [&](const double2& x, const double2& y) {
            auto bk = [&](const double2& z) { const double c = cost(z); return c >= 8.0 && c < 8.5 ? 0 : std::min(15, 1 + (int)(c / 8.0)); };
            return bk(x) > bk(y); });
        std::stable_sort(hc.begin() + s0, hc.begin() + s1, [&](const double2& x, const double2& y) { return cls(x) < cls(y); });
        std::stable_sort(hk.begin() + s0, hk.begin() + s1, [&](const double2& x, const double2& y) {
            const int a = cls(x), b = cls(y);
            return a != b ? a < b : cost(x) > cost(y); });
    }
    double2 *dz, *dzs, *dzr, *dzp, *dout;
    hipMalloc(&dzp, sizeof(double2) * np);
    hipMemcpy(dzp, hp.data(), sizeof(double2) * np, hipMemcpyHostToDevice);
    double2 *dzl, *dzb;
    hipMalloc(&dzl, sizeof(double2) * np);
    hipMalloc(&dzb, sizeof(double2) * np);
    hipMemcpy(dzl, hl.data(), sizeof(double2) * np, hipMemcpyHostToDevice);
    hipMemcpy(dzb, hb.data(), sizeof(double2) * np, hipMemcpyHostToDevice);
    double2 *dzc, *dzk;
    hipMalloc(&dzc, sizeof(double2) * np);
    hipMalloc(&dzk, sizeof(double2) * np);
    hipMemcpy(dzc, hc.data(), sizeof(double2) * np, hipMemcpyHostToDevice);
    hipMemcpy(dzk, hk.data(), sizeof(double2) * np, hipMemcpyHostToDevice);
    hipMalloc(&dz, sizeof(double2) * n);
    hipMalloc(&dzs, sizeof(double2) * n);
    hipMalloc(&dzr, sizeof(double2) * n);
    hipMalloc(&dout, sizeof(double2) * (n > np ? n : np));
    hipMemcpy(dz, h.data(), sizeof(double2) * n, hipMemcpyHostToDevice);
    hipMemcpy(dzs, hs.data(), sizeof(double2) * n, hipMemcpyHostToDevice);
    hipMemcpy(dzr, hr.data(), sizeof(double2) * n, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, auto kern, const double2* src, int n) {
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kern, dim3((n + 255) / 256), dim3(256), 0, 0, src, dout, n);
        hipEventRecord(e0);
        const int reps = 5;
        for (int rep = 0; rep < reps; ++rep) hipLaunchKernelGGL(kern, dim3((n + 255) / 256), dim3(256), 0, 0, src, dout, n);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-30s %8.3f ms per %d calls = %.4f ns/call (device)\n", name, ms / reps, n, ms / reps * 1e6 / n);
        fflush(stdout);
    };
    run("gsl_cli2 tile order", kbench<0>, dz, n);
    run("gsl_cli2 shuffled", kbench<0>, dzr, n);
    run("gsl_cli2 cost-sorted", kbench<0>, dzs, n);
    run("gsl_cli2 points fastest", kbench<0>, dzp, np);
    run("points fastest, 1024-sets sorted", kbench<0>, dzl, np);
    run("points fastest, 1024-sets bucketed", kbench<0>, dzb, np);
    run("points fastest, 1024-sets by branch", kbench<0>, dzc, np);
    run("1024-sets by branch, then cost", kbench<0>, dzk, np);
    {   // the branch mix of the set
        long long nc[13] = {};
        for (const double2& z : hp) nc[cls(z)]++;
        for (int c = 0; c < 13; ++c) if (nc[c]) printf("class %2d (inv %d refl %d series %d): %.3f\n", c, c ? (c - 1) / 6 : 0, c ? ((c - 1) / 3) % 2 : 0, c ? (c - 1) % 3 + 1 : 0, (double)nc[c] / hp.size());
    }
    run("cli2 (shared algorithm)", kbench<1>, dz, n);
    return (int)hipDeviceSynchronize();
}
