/*
 * nuSIprop oracle -- restatement of interp::spline_ND<N>.  TEST INFRASTRUCTURE ONLY.
 * Cubic-Hermite (Catmull-Rom-like, non-uniform) tensor-product interpolation.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ora_spline.h"
#include "ora_libm.h"

#define SQ(a) ((a) * (a))

/* interp.hpp:576-636.  Weights of the last node are never read (k <= n-2);
 * the reference computes them from x[j+1], x[j+2] past the end (UB) -- we
 * leave them at zero. */
static void compute_weights(ora_spline *s)
{
    for (int i = 0; i < s->ndim; ++i) {
        const int n = s->n[i];
        const double *x = s->x[i];
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b) s->w[i][a][b] = (double *)calloc((size_t)n, sizeof(double));
        for (int j = 0; j + 1 < n; ++j) {
            double *w00 = &s->w[i][0][0][j], *w01 = &s->w[i][0][1][j], *w02 = &s->w[i][0][2][j], *w03 = &s->w[i][0][3][j];
            double *w10 = &s->w[i][1][0][j], *w11 = &s->w[i][1][1][j], *w12 = &s->w[i][1][2][j], *w13 = &s->w[i][1][3][j];
            double *w20 = &s->w[i][2][0][j], *w21 = &s->w[i][2][1][j], *w22 = &s->w[i][2][2][j], *w23 = &s->w[i][2][3][j];
            double *w30 = &s->w[i][3][0][j], *w31 = &s->w[i][3][1][j], *w32 = &s->w[i][3][2][j], *w33 = &s->w[i][3][3][j];
            const double xm = (j > 0) ? x[j - 1] : 0.0, x0 = x[j], x1 = x[j + 1];
            const double x2 = (j + 2 < n) ? x[j + 2] : 0.0;
            if (j == 0) {
                *w00 = 0;
                *w01 = (x0 - x1) / (x0 - x2);
                *w02 = (-1 + (x1 - x0) / (x0 - x2));
                *w03 = 1;
                *w10 = 0;
                *w11 = (x1 - x0) / (x1 - x2);
                *w12 = (x0 - x2) / (x1 - x2);
                *w13 = 0;
                *w20 = 0;
                *w21 = SQ(x1 - x0) / ((x2 - x1) * (x2 - x0));
                *w22 = SQ(x1 - x0) / ((x2 - x1) * (x0 - x2));
                *w23 = 0;
            } else if (j == n - 2) {
                *w00 = 0;
                *w01 = SQ(x1 - x0) / ((xm - x0) * (xm - x1));
                *w02 = SQ(x1 - x0) / ((x0 - xm) * (xm - x1));
                *w03 = 0;
                *w10 = 0;
                *w11 = (x1 - x0) / (xm - x0);
                *w12 = (2 * x0 - x1 - xm) / (xm - x0);
                *w13 = 1;
                *w20 = 0;
                *w21 = (x0 - x1) / (xm - x1);
                *w22 = (xm - x0) / (xm - x1);
                *w23 = 0;
            } else {
                *w00 = SQ(x1 - x0) / ((x0 - xm) * (xm - x1));
                *w01 = 2 * SQ(x1 - x0) / ((xm - x0) * (xm - x1));
                *w02 = SQ(x1 - x0) / ((x0 - xm) * (xm - x1));
                *w03 = 0;
                *w10 = (x0 - x1) * (1 / (xm - x0) + 1 / (x0 - x2));
                *w11 = (x0 - x1) * (2 / (x0 - xm) + 1 / (x2 - x0));
                *w12 = (2 * x0 - x1 - xm) / (xm - x0);
                *w13 = 1;
                *w20 = (x1 - x0) * (1 / (xm - x1) + 1 / (x1 - x2));
                *w21 = (x1 - x0) * (2 / (x1 - xm) + 1 / (x2 - x1));
                *w22 = (xm - x0) / (xm - x1);
                *w23 = 0;
                *w30 = SQ(x1 - x0) / ((-x1 + x2) * (-x0 + x2));
                *w31 = SQ(x1 - x0) / ((x1 - x2) * (-x0 + x2));
                *w32 = 0;
                *w33 = 0;
            }
        }
    }
}

int ora_spline_load(ora_spline *s, int ndim, const int *n, const char *path, int regular, const int *islog)
{
    memset(s, 0, sizeof(*s));
    s->ndim = ndim;
    s->regular = regular;
    size_t nf = 1;
    for (int i = 0; i < ndim; ++i) {
        s->n[i] = n[i];
        s->x[i] = (double *)calloc((size_t)n[i], sizeof(double));
        nf *= (size_t)n[i];
    }
    for (int i = 0; i <= ndim; ++i) s->islog[i] = islog ? islog[i] : 0;
    s->f = (double *)malloc(nf * sizeof(double));
    FILE *fp = fopen(path, "rb");
    if (!fp) return -3;
    float rec[ORA_SPL_MAXDIM + 1];
    int idx[ORA_SPL_MAXDIM] = {0};
    for (size_t r = 0; r < nf; ++r) {
        if (fread(rec, sizeof(float), (size_t)ndim + 1, fp) != (size_t)ndim + 1) { fclose(fp); return -3; }
        /* decompose the record number, last index fastest */
        size_t q = r;
        for (int i = ndim - 1; i >= 0; --i) { idx[i] = (int)(q % (size_t)n[i]); q /= (size_t)n[i]; }
        for (int i = 0; i < ndim; ++i) s->x[i][idx[i]] = (double)rec[i];
        s->f[r] = (double)rec[ndim];
    }
    fclose(fp);
    for (int i = 0; i < ndim; ++i)
        if (s->islog[i])
            for (int j = 0; j < n[i]; ++j) s->x[i][j] = log(s->x[i][j]);
    if (s->islog[ndim])
        for (size_t j = 0; j < nf; ++j) s->f[j] = log(s->f[j]);
    compute_weights(s);
    return 0;
}

void ora_spline_free(ora_spline *s)
{
    for (int i = 0; i < s->ndim; ++i) {
        free(s->x[i]);
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b) free(s->w[i][a][b]);
    }
    free(s->f);
    memset(s, 0, sizeof(*s));
}

int ora_spline_eval(const ora_spline *s, const double *x0in, double *out)
{
    const int D = s->ndim;
    double x0[ORA_SPL_MAXDIM];
    for (int i = 0; i < D; ++i) x0[i] = s->islog[i] ? ora_log(x0in[i]) : x0in[i];   /* evaluated like the GPU */
    for (int i = 0; i < D; ++i)
        if (x0[i] <= s->x[i][0] || x0[i] >= s->x[i][s->n[i] - 1]) return -4;
    int k[ORA_SPL_MAXDIM];
    for (int i = 0; i < D; ++i) {
        const double *x = s->x[i];
        if (s->regular) {
            k[i] = (int)((x0[i] - x[0]) / (x[1] - x[0]));
            if (x0[i] < x[1]) k[i] = 0;
            else if (x0[i] > x[s->n[i] - 2]) k[i] = s->n[i] - 2;
        } else {
            int L = 0, R = s->n[i] - 1;
            while (L <= R) {
                const int m = (L + R) / 2;
                if (x0[i] < x[m]) R = m - 1;
                else { k[i] = m; L = m + 1; }
            }
        }
    }
    int lo[ORA_SPL_MAXDIM], cnt[ORA_SPL_MAXDIM];
    double t[ORA_SPL_MAXDIM];
    for (int i = 0; i < D; ++i) {
        if (k[i] == 0) { lo[i] = 0; cnt[i] = 3; }
        else if (k[i] == s->n[i] - 2) { lo[i] = k[i] - 1; cnt[i] = 3; }
        else { lo[i] = k[i] - 1; cnt[i] = 4; }
        t[i] = (x0[i] - s->x[i][k[i]]) / (s->x[i][k[i] + 1] - s->x[i][k[i]]);
    }
    /* iterate the stencil with dimension 0 fastest (interp.hpp:431-460) */
    int idx[ORA_SPL_MAXDIM] = {0};
    double res = 0;
    for (;;) {
        size_t off = 0;
        for (int i = 0; i < D; ++i) off = off * (size_t)s->n[i] + (size_t)(lo[i] + idx[i]);
        double v = s->f[off];
        for (int i = 0; i < D; ++i) {
            const int a = idx[i], kk = k[i];
            v *= (t[i] * t[i] * t[i] * s->w[i][a][0][kk] + SQ(t[i]) * s->w[i][a][1][kk]
                  + t[i] * s->w[i][a][2][kk] + s->w[i][a][3][kk]);
        }
        res += v;
        int p = 0;
        while (p < D && ++idx[p] == cnt[p]) { idx[p] = 0; ++p; }
        if (p == D) break;
    }
    *out = s->islog[D] ? exp(res) : res;
    return 0;
}
