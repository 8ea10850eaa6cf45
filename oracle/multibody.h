/* ORACLE -- TEST INFRASTRUCTURE ONLY.  Multibody physics restatement (multibody.c). */
#ifndef EXO_ORACLE_MULTIBODY_H
#define EXO_ORACLE_MULTIBODY_H

typedef struct {
    double dt, gravity, kp, kd, motor_impulse, passive_impulse, limit_impulse, erp, lin_damp, ang_damp, max_vel;
    int iters;
} mb_params;

void oracle_mb_default_params(mb_params *p);
void oracle_mb_aba(const double *q, const double *qd, const double *tau, const mb_params *p, double *qdd);
void oracle_mb_rnea(const double *q, const double *qd, const double *qdd, const mb_params *p, double *tau);
void oracle_mb_mass(const double *q, double *M);
void oracle_mb_link_coms(const double *q, double *com);
int oracle_mb_step(double *q, double *qd, const double *tgt5, const mb_params *p, double *stats);

#endif
