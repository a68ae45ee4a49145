// symmetry.h -- Particle::symmetrise's per-particle step (device), shared by
// symmetry.hip (thx_pf_symmetrise) and the expectation driver's perturbation.
#pragma once

#include "common.h"

namespace thx {

constexpr int SYM_MAX = 64;   // the icosahedral groups have 59 non-identity elements

// quaternion_mul, src/Geometry/Euler.cpp:13-26
THX_DEV void sym_qmul(const double* a, const double* b, double* c)
{
    c[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    c[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    c[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    c[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
}

// symmetryCounterpart (src/Geometry/Symmetry.cpp:309-335), q in place: of q
// and every conj(s_i) q the one with the largest |<., a>|, the first on ties
THX_DEV void sym_counterpart(double* q, const double* a, const double* symQ, int nSym)
{
    double best[4] = {q[0], q[1], q[2], q[3]};
    double s = fabs(q[0] * a[0] + q[1] * a[1] + q[2] * a[2] + q[3] * a[3]);
    for (int e = 0; e < nSym; e++) {
        const double* sq = symQ + 4 * e;
        const double cq[4] = {sq[0], -sq[1], -sq[2], -sq[3]};
        double p[4];
        sym_qmul(cq, q, p);
        const double t = fabs(p[0] * a[0] + p[1] * a[1] + p[2] * a[2] + p[3] * a[3]);
        if (t > s) {
            s = t;
            for (int k = 0; k < 4; k++) best[k] = p[k];
        }
    }
    for (int k = 0; k < 4; k++) q[k] = best[k];
}

}  // namespace thx
