/* TEST INFRASTRUCTURE ONLY -- runs the CPU oracle under ASan/UBSan (tests/test_sanitizers.py).
 * Small configurations of every branch the parity tests use: Majorana / Dirac, normal / inverted
 * ordering, resonant-only, DSNB / power-law source, the phi-phi spline path on small tables written
 * here (interp.hpp's binary layout), out-of-range lookups, and the energy-conservation diagnostic. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "nusi_oracle.h"

static int fails = 0;
#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } } while (0)

static ora_params base(void)
{
    ora_params p = {6e5, 0.01, 0.1, 2.5, 6.0, 1, 1, 1, 40, 12.0, 17.0, 5.0, 2, 0, 1};
    return p;
}

static void run(ora_params p, const char *at, const int *n2, const char *a, const int *n3, int expect_err)
{
    int err = 0;
    ora_state *S = ora_create(&p, &err);
    CHECK(S && err == 0);
    if (!S) return;
    if (at) CHECK(ora_load_phiphi_dims(S, at, n2, a, n3) == 0);
    const int N = ora_N(S);
    double *f = calloc(3 * (size_t)N, sizeof(double)), *fl = calloc(3 * (size_t)N, sizeof(double));
    const int r = ora_evolve(S, f, fl);
    if (expect_err) CHECK(r != 0);
    else {
        CHECK(r == 0);
        for (int i = 0; i < 3 * N; ++i) CHECK(isfinite(fl[i]));
        const double e = ora_check_energy_conservation(S, f, fl);
        CHECK(isfinite(e));
    }
    free(f);
    free(fl);
    ora_destroy(S);
}

/* float32 records {x0.., f}, last index fastest */
static void write_table(const char *path, int nd, const int *n, double x0lo, double x0hi)
{
    FILE *fp = fopen(path, "wb");
    int idx[3] = {0, 0, 0};
    long tot = 1;
    for (int d = 0; d < nd; ++d) tot *= n[d];
    for (long r = 0; r < tot; ++r) {
        long q = r;
        for (int d = nd - 1; d >= 0; --d) { idx[d] = (int)(q % n[d]); q /= n[d]; }
        float rec[4];
        rec[0] = (float)(x0lo * pow(x0hi / x0lo, idx[0] / (double)(n[0] - 1)));
        if (nd == 2) rec[1] = (float)(0.003 + 0.057 * idx[1] / (double)(n[1] - 1));
        else {
            rec[1] = (float)(idx[1]);
            rec[2] = (float)(0.003 + 0.057 * idx[2] / (double)(n[2] - 1));
        }
        rec[nd] = (float)(1e-7 * (1 + rec[0]) * (1 + idx[nd - 1]));
        fwrite(rec, sizeof(float), (size_t)nd + 1, fp);
    }
    fclose(fp);
}

int main(void)
{
    ora_params p = base();
    run(p, NULL, NULL, NULL, NULL, 0);                                  /* Majorana, non-resonant, power law */
    p.majorana = 0; run(p, NULL, NULL, NULL, NULL, 0);                  /* Dirac */
    p = base(); p.non_resonant = 0; run(p, NULL, NULL, NULL, NULL, 0);  /* resonant only */
    p = base(); p.normal_ordering = 0; p.mntot = 0.2; run(p, NULL, NULL, NULL, NULL, 0);
    p = base(); p.source = 0; p.lEmin = 4; p.lEmax = 9; p.mphi = 3e3; p.g = 0.03; run(p, NULL, NULL, NULL, NULL, 0);
    p = base(); p.mphi = 1e7; p.g = 0.5; p.flav = 0; run(p, NULL, NULL, NULL, NULL, 0);
    /* reference order: GSL's dilogarithm algorithms (ora_gsl.c) at every call site */
    ora_set_reference_order(1);
    p = base(); run(p, NULL, NULL, NULL, NULL, 0);
    p = base(); p.mphi = 1e7; p.g = 1.0; run(p, NULL, NULL, NULL, NULL, 0);
    p = base(); p.source = 0; p.lEmin = 4; p.lEmax = 9; p.mphi = 3e3; p.g = 0.03; run(p, NULL, NULL, NULL, NULL, 0);
    p = base(); p.majorana = 0; run(p, NULL, NULL, NULL, NULL, 0);
    ora_set_reference_order(0);
    /* phi-phi on small tables */
    char dir[] = "/tmp/nusi_asan_XXXXXX";
    CHECK(mkdtemp(dir) != NULL);
    char at[256], a[256];
    snprintf(at, sizeof at, "%s/at.bin", dir);
    snprintf(a, sizeof a, "%s/a.bin", dir);
    const int n2[2] = {40, 6}, n3[3] = {12, 60, 5};
    write_table(at, 2, n2, 1.0, 2e4);
    write_table(a, 3, n3, 1.0, 2e4);
    p = base(); p.phiphi = 1; p.mphi = 1e4; p.g = 0.05; p.lEmin = 10; p.lEmax = 12;
    run(p, at, n2, a, n3, 0);
    write_table(at, 2, n2, 1.0, 50.0);   /* lookups beyond the nodes: the reference's exit(1), an error here */
    write_table(a, 3, n3, 1.0, 50.0);
    run(p, at, n2, a, n3, 1);
    unlink(at);
    unlink(a);
    rmdir(dir);
    if (fails) { fprintf(stderr, "%d checks failed\n", fails); return 1; }
    printf("oracle_asan OK\n");
    return 0;
}
