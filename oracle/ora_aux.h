/*
 * nuSIprop oracle -- restatement of aux.hpp (namespace nuSIaux).
 * TEST INFRASTRUCTURE ONLY: see ora_specfun.h.
 *
 *   ora_atandiff        aux.hpp:63-75    atan(x)-atan(y), Taylor when |x|,|y|>=1e2, same sign
 *   ora_dilogdiff_c     aux.hpp:77-96    Li2(x)-Li2(y) complex, asymptotic when |x|,|y|>1e2
 *   ora_dilogdiff       aux.hpp:98-113   Li2(-x)-Li2(-y)
 *   ora_dilog1mdiff     aux.hpp:115-130  Li2(-1-x)-Li2(-1-y)
 *   ora_dilog1pdiff     aux.hpp:132-148  Li2(1+x)-Li2(1+y), x,y<0
 *   ora_dilog1over1mdiff aux.hpp:150-166 Li2(1/(1-x))-Li2(1/(1-y)), x,y<0
 *   ora_getmL           aux.hpp:12-50    lightest neutrino mass (see the note there)
 *   GL3 nodes/weights   aux.hpp:53-54
 */
#ifndef NUSI_ORA_AUX_H
#define NUSI_ORA_AUX_H
#include "ora_cplx.h"

extern const double ora_gl_w[3];
extern const double ora_gl_x[3];

double ora_atandiff(double x, double y);
zc ora_dilogdiff_c(zc x, zc y);
double ora_dilogdiff(double x, double y);
double ora_dilog1mdiff(double x, double y);
double ora_dilog1pdiff(double x, double y);
double ora_dilog1over1mdiff(double x, double y);
int ora_getmL(double mSum, double dmqSL, double dmqAT, double *mL);

#endif
