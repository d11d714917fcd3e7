// TEST INFRASTRUCTURE ONLY -- the host build of the device physics headers (tests/hostcheck) under
// ASan/UBSan: per-entry tables and the host emulation of the tile kernel (k_alpha_tile's edge lists,
// jobs and LDS leaf layout) for Majorana / Dirac / resonant-only points; the two must agree bit for bit.
#include <cstdio>
#include <cstring>
#include <vector>

#include "../hostcheck/hostcheck.cpp"

int main()
{
    int fails = 0;
    const int N = 31, Nz = 12, T = N + Nz - 2;
    std::vector<double> lo(T), hi(T);
    for (int n = 0; n < T; ++n) {   // log grid, the first N bins sharing edges, the extended ones not
        lo[n] = pow(10.0, 12.0 + 5.0 * n / N);
        hi[n] = (n + 1 < N) ? pow(10.0, 12.0 + 5.0 * (n + 1) / N) : lo[n] * pow(10.0, 5.0 / N) * (1 + 1e-15 * n);
        if (n > 0 && n < N) lo[n] = hi[n - 1];
    }
    const double pts[2][13] = {{6e5, 0.01, 0.1, 2.5, 6, 1, 6e5 * 1e-4 / (16 * M_PI), 0.02, 0.022, 0.055, 0.3, 0.3, 0.4},
                               {2e6, 0.3, 0.1, 2.5, 6, 1, 2e6 * 0.09 / (16 * M_PI), 0.02, 0.022, 0.055, 0.3, 0.3, 0.4}};
    const int flags[3][4] = {{1, 1, 0, 1}, {0, 1, 0, 1}, {1, 0, 0, 1}};
    for (const auto& pt : pts)
        for (const auto& fl : flags) {
            std::vector<double> G(T), At(T), A(T * T, 0.0), B(T * T, 0.0);
            for (int ref = 0; ref < 2; ++ref) {   // the default and the reference-order (GSL) arithmetic
                if (ref) {
                    hc_tables_ref(pt, fl, T, lo.data(), hi.data(), G.data(), At.data(), A.data());
                    hc_alpha_tiled_ref(pt, fl, T, lo.data(), hi.data(), B.data());
                } else {
                    hc_tables(pt, fl, T, lo.data(), hi.data(), G.data(), At.data(), A.data());
                    hc_alpha_tiled(pt, fl, T, lo.data(), hi.data(), B.data());
                }
                for (int n = 0; n < T; ++n)
                    for (int m = n + 1; m < T; ++m)
                        if ((fl[1] || m == n + 1) && memcmp(&A[n * T + m], &B[n * T + m], sizeof(double)) != 0) {
                            if (fails < 5) fprintf(stderr, "tile != entry at (%d, %d) ref %d\n", n, m, ref);
                            ++fails;
                        }
            }
        }
    if (fails) return 1;
    printf("hostcheck_asan OK\n");
    return 0;
}
