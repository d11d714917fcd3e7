/*
 * nuSIprop oracle -- restatement of interp::spline_ND<N> (interp.hpp:13-638).
 * TEST INFRASTRUCTURE ONLY.
 */
#ifndef NUSI_ORA_SPLINE_H
#define NUSI_ORA_SPLINE_H

#define ORA_SPL_MAXDIM 4

typedef struct {
    int ndim;
    int n[ORA_SPL_MAXDIM];
    double *x[ORA_SPL_MAXDIM];      /* nodes (log'd where islog) */
    double *f;                      /* last index fastest */
    double *w[ORA_SPL_MAXDIM][4][4];/* interp.hpp:576-636 */
    int islog[ORA_SPL_MAXDIM + 1];
    int regular;
} ora_spline;

/* interp.hpp:173-320 (binary branch): float32 records {x0..x_{N-1}, f}, last index fastest.
 * returns 0, -3 if the file is missing/short */
int ora_spline_load(ora_spline *s, int ndim, const int *n, const char *path, int regular, const int *islog);
void ora_spline_free(ora_spline *s);
/* interp.hpp:345-467; returns 0 or -4 when x0 is outside the node range (reference exit(1)) */
int ora_spline_eval(const ora_spline *s, const double *x0, double *out);

#endif
