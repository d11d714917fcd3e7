/*
 * nuSIprop oracle -- fdlibm-algorithm elementary functions (see ora_libm.c).
 * TEST INFRASTRUCTURE ONLY.
 */
#ifndef NUSI_ORA_LIBM_H
#define NUSI_ORA_LIBM_H

double ora_log(double x);
double ora_log1p(double x);
double ora_exp(double x);
double ora_atan(double x);
double ora_atan2(double y, double x);
double ora_atanh(double x);
double ora_log10(double x);
double ora_pow(double x, double y);   /* x > 0: exp(y*log(x)) */

#endif
