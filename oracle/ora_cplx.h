/*
 * nuSIprop oracle -- explicit complex arithmetic.  TEST INFRASTRUCTURE ONLY.
 * Replaces the reference's GNU `double _Complex` (nuSIprop.hpp:846-869,
 * 1137-1182, 1432-1451; aux.hpp:77-96) with the operation sequence the GPU
 * uses (nusiprop_amd/csrc/nusi_math.hpp): (ac-bd, ad+bc) products, real
 * operands applied component-wise (as GNU C does), Smith's division (libgcc
 * __divdc3's algorithm for finite operands), clog = (log(x^2+y^2)/2, atan2).
 */
#ifndef NUSI_ORA_CPLX_H
#define NUSI_ORA_CPLX_H
#include <math.h>
#include "ora_libm.h"

typedef struct { double r, i; } zc;
static inline zc zmk(double r, double i) { zc z; z.r = r; z.i = i; return z; }
static inline zc zre(double r) { return zmk(r, 0.0); }
static inline zc zadd(zc a, zc b) { return zmk(a.r + b.r, a.i + b.i); }
static inline zc zsub(zc a, zc b) { return zmk(a.r - b.r, a.i - b.i); }
static inline zc zneg(zc a) { return zmk(-a.r, -a.i); }
static inline zc zaddr(zc a, double s) { return zmk(a.r + s, a.i); }        /* a + s */
static inline zc zrsub(double s, zc a) { return zmk(s - a.r, -a.i); }       /* s - a */
static inline zc zsubr(zc a, double s) { return zmk(a.r - s, a.i); }        /* a - s */
static inline zc zmul(zc a, zc b) { return zmk(a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r); }
static inline zc zscale(double s, zc a) { return zmk(s * a.r, s * a.i); }    /* s * a */
static inline zc zdivr(zc a, double s) { return zmk(a.r / s, a.i / s); }     /* a / s */
static inline zc zconj(zc a) { return zmk(a.r, -a.i); }
static inline zc zdiv(zc a, zc b)
{
    const double c = b.r, d = b.i;
    if (fabs(c) < fabs(d)) {
        const double ratio = c / d, den = (c * ratio) + d;
        return zmk(((a.r * ratio) + a.i) / den, ((a.i * ratio) - a.r) / den);
    }
    const double ratio = d / c, den = (d * ratio) + c;
    return zmk(((a.i * ratio) + a.r) / den, (a.i - (a.r * ratio)) / den);
}
static inline zc zrdiv(double s, zc b) { return zdiv(zre(s), b); }          /* s / b */
static inline double zarg(zc z) { return ora_atan2(z.i, z.r); }
static inline double zabs(zc z) { return sqrt(z.r * z.r + z.i * z.i); }
static inline zc zlog(zc z) { return zmk(0.5 * ora_log(z.r * z.r + z.i * z.i), ora_atan2(z.i, z.r)); }
static inline double zarg_real(double x) { return ora_atan2(0.0, x); }      /* carg of a promoted real */

#endif
