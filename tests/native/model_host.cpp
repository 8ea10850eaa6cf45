// TEST HELPER: host (gcc) build of the device math in csrc/exo_model.h, so the
// algorithms of the HIP kernels can be unit-tested on the CPU against the
// oracle.  Never linked into the product.
#include <string.h>
#include "exo_model.h"

using namespace exo;

extern "C" {
int mh_rk45(const double *ii25, const double *dnz21, const double *snz21, const double *T, double *q) {
    OdeM M;
    memcpy(M.ii, ii25, sizeof M.ii);
    memcpy(M.dn, dnz21, sizeof M.dn);
    memcpy(M.sn, snz21, sizeof M.sn);
    return rk45_solve(M, T, q) ? 0 : -1;
}
void mh_link_coms(const double *q5, double *act42, double *ref6) {
    Urdf U;
    build_urdf(U);
    double act[14][3];
    link_coms(U, q5, act, ref6);
    memcpy(act42, act, sizeof act);
}
double mh_cos_atan2(double y, double x) { return cos_atan2(y, x); }
double mh_philox_u01(unsigned long long seed, unsigned env, unsigned episode, unsigned p) {
    return philox_u01(seed, env, episode, p);
}
}
