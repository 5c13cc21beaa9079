/*
 * wbc_ref.c — TEST INFRASTRUCTURE ONLY.  Plain-C fp64 restatement of the reference's per-cycle
 * whole-body-control path, written the way the reference computes it (dense Eigen-style
 * algebra), for two uses:
 *   1. the checker for the HIP engine at batch sizes where numpy is too slow (tests/), and
 *   2. the CPU baseline timed by bench.py (cpu_baseline.kind = "port").
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Restates (file:line in the reference, /root/reference):
 *   iDynTree KinDynComputations, MIXED representation: setRobotState (src/whole_body_controller.cpp:258),
 *     getCenterOfMassPosition/Velocity (:260-261), getFreeFloatingMassMatrix (:266),
 *     generalizedBiasForces - generalizedGravityForces (:544-551), getFrameFreeFloatingJacobian
 *     (:327-341), getWorldTransform (:349-359), getFrameVel (:369-379)  [un-vendored library,
 *     restated from Kane's equations with generalized speeds nu = (p_B_dot, omega_W, qdot)];
 *   WholeBodyController::updateState (:256-294) with computeTransformationMatrix (:296-320),
 *     computeJacobians (:322-342), computeDerivatives (:384-402);
 *   solveQP (:466-542) with computeNonSlidingConstraints (:404-424), computeDesiredWrench
 *     (:426-445), computeCommandedAccelerationSwingLegs (:447-464);
 *   computeJointTorques (:553-577);
 *   qpOASES::SQProblem init/hotstart (:517-535) — stands in as the dense Goldfarb-Idnani dual
 *     active-set method (H > 0: the optimum is unique; qpOASES is un-vendored).
 * Every 18x18 inverse is a dense partial-pivot LU inverse evaluated where the reference evaluates
 * transformationMatrix_.inverse() (:270 twice, :278, :282, :289, :293 twice) — deliberately not
 * optimised, so the timing reflects the reference's algorithm.
 *
 * Parity status: unpinned against the reference binary (not buildable: ROS/Eigen/iDynTree/qpOASES
 * absent); cross-checked against oracle/wbc_np.py and physics identities.
 */
#include "wbc_ref.h"

#include <math.h>
#include <string.h>

#define ND 18
#define NJ 12
#define NL 4
#define NV 42
#define NC 70
#define QP_INFTY 1.0e20

/* ------------------------------------------------------------------ dense helpers */
static void mat_mul(const double* A, const double* B, double* C, int n, int k, int m) {
    /* C (n x m) = A (n x k) B (k x m), row-major; C must not alias */
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j) {
            double s = 0.0;
            for (int t = 0; t < k; ++t) s += A[i * k + t] * B[t * m + j];
            C[i * m + j] = s;
        }
}
static void mat_T(const double* A, double* AT, int n, int m) {
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j) AT[j * n + i] = A[i * m + j];
}
/* dense inverse by LU with partial pivoting (Eigen's PartialPivLU::inverse) */
static int mat_inv(const double* A, double* Ai, int n) {
    double LU[ND * ND];
    int piv[ND];
    memcpy(LU, A, sizeof(double) * n * n);
    for (int i = 0; i < n; ++i) piv[i] = i;
    for (int k = 0; k < n; ++k) {
        int p = k;
        double best = fabs(LU[k * n + k]);
        for (int i = k + 1; i < n; ++i)
            if (fabs(LU[i * n + k]) > best) { best = fabs(LU[i * n + k]); p = i; }
        if (best == 0.0) return -1;
        if (p != k) {
            for (int j = 0; j < n; ++j) { double t = LU[k * n + j]; LU[k * n + j] = LU[p * n + j]; LU[p * n + j] = t; }
            int t = piv[k]; piv[k] = piv[p]; piv[p] = t;
        }
        for (int i = k + 1; i < n; ++i) {
            double f = LU[i * n + k] / LU[k * n + k];
            LU[i * n + k] = f;
            for (int j = k + 1; j < n; ++j) LU[i * n + j] -= f * LU[k * n + j];
        }
    }
    for (int c = 0; c < n; ++c) {
        double y[ND];
        for (int i = 0; i < n; ++i) {
            double s = (piv[i] == c) ? 1.0 : 0.0;
            for (int j = 0; j < i; ++j) s -= LU[i * n + j] * y[j];
            y[i] = s;
        }
        for (int i = n - 1; i >= 0; --i) {
            double s = y[i];
            for (int j = i + 1; j < n; ++j) s -= LU[i * n + j] * y[j];
            y[i] = s / LU[i * n + i];
        }
        for (int i = 0; i < n; ++i) Ai[i * n + c] = y[i];
    }
    return 0;
}
static void cross(const double* a, const double* b, double* o) {
    double x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z;
}
static void skew(const double* v, double* S) { /* skewOperator, cpp:3-10 */
    S[0] = 0.0;   S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2];  S[4] = 0.0;   S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0];  S[8] = 0.0;
}
static void mv3(const double* M, const double* v, double* o) {
    double x = M[0] * v[0] + M[1] * v[1] + M[2] * v[2], y = M[3] * v[0] + M[4] * v[1] + M[5] * v[2],
           z = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
    o[0] = x; o[1] = y; o[2] = z;
}
static void mm3(const double* A, const double* B, double* C) { mat_mul(A, B, C, 3, 3, 3); }
static void quat_R(const double* q, double* R) { /* Eigen toRotationMatrix, cpp:209-213; q = (x,y,z,w) */
    double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
static void axis_rot(const double* a, double q, double* R) {
    double n = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    double x = a[0] / n, y = a[1] / n, z = a[2] / n, s = sin(q), c = cos(q), v = 1 - c;
    R[0] = c + x * x * v;     R[1] = x * y * v - z * s; R[2] = x * z * v + y * s;
    R[3] = y * x * v + z * s; R[4] = c + y * y * v;     R[5] = y * z * v - x * s;
    R[6] = z * x * v - y * s; R[7] = z * y * v + x * s; R[8] = c + z * z * v;
}

/* ------------------------------------------------------------------ kinematics / dynamics */
typedef struct {
    double m, c[3], I[9], Jv[3 * ND], Jw[3 * ND], w[3], alpha[3], a[3];
} body_t;

void wbc_ref_kindyn(const wbc_model* md, const double* pose, const double* nu, const double* qj, wbc_ref_kindyn_t* out) {
    const double* pB = pose;
    double RB[9];
    quat_R(pose + 3, RB);
    const double *wB = nu + 3, *qd = nu + 6;
    body_t b[13];
    memset(b, 0, sizeof(b));
    /* base */
    {
        double c[3], r[3], S[9], t[3];
        mv3(RB, md->base_com, c);
        for (int i = 0; i < 3; ++i) c[i] += pB[i], r[i] = c[i] - pB[i];
        b[0].m = md->base_mass;
        memcpy(b[0].c, c, sizeof c);
        double tmp[9], RT[9];
        mm3(RB, md->base_inertia, tmp);
        mat_T(RB, RT, 3, 3);
        mm3(tmp, RT, b[0].I);
        skew(r, S);
        for (int i = 0; i < 3; ++i) {
            b[0].Jv[i * ND + i] = 1.0;
            for (int j = 0; j < 3; ++j) b[0].Jv[i * ND + 3 + j] = -S[i * 3 + j];
            b[0].Jw[i * ND + 3 + i] = 1.0;
        }
        memcpy(b[0].w, wB, 3 * sizeof(double));
        cross(wB, r, t);
        cross(wB, t, b[0].a);
    }
    memset(out, 0, sizeof(*out));
    for (int l = 0; l < NL; ++l) {
        double Rp[9], op[3], wp[3], alp[3] = {0, 0, 0}, aop[3] = {0, 0, 0};
        memcpy(Rp, RB, sizeof Rp);
        memcpy(op, pB, sizeof op);
        memcpy(wp, wB, sizeof wp);
        int cols[3];
        double ax[3][3], org[3][3];
        for (int k = 0; k < 3; ++k) {
            const wbc_link* lk = &md->link[l][k];
            const int col = 6 + 3 * l + k;
            double Rj[9], oj[3], aj[3], Rl[9], Rc[9], rel[3], t[3], u[3], ao[3], wc[3], alc[3];
            mm3(Rp, lk->R, Rj);
            mv3(Rp, lk->p, oj);
            for (int i = 0; i < 3; ++i) oj[i] += op[i];
            mv3(Rj, lk->axis, aj);
            axis_rot(lk->axis, qj[3 * l + k], Rl);
            mm3(Rj, Rl, Rc);
            cols[k] = col;
            memcpy(ax[k], aj, sizeof aj);
            memcpy(org[k], oj, sizeof oj);
            for (int i = 0; i < 3; ++i) rel[i] = oj[i] - op[i];
            cross(alp, rel, ao);
            cross(wp, rel, t);
            cross(wp, t, u);
            for (int i = 0; i < 3; ++i) ao[i] += aop[i] + u[i];
            cross(wp, aj, t);
            for (int i = 0; i < 3; ++i) {
                wc[i] = wp[i] + aj[i] * qd[3 * l + k];
                alc[i] = alp[i] + t[i] * qd[3 * l + k];
            }
            body_t* bb = &b[1 + 3 * l + k];
            double c[3], r[3], S[9], RcT[9], tmp[9];
            mv3(Rc, lk->com, c);
            for (int i = 0; i < 3; ++i) c[i] += oj[i], r[i] = c[i] - pB[i];
            bb->m = lk->mass;
            memcpy(bb->c, c, sizeof c);
            mm3(Rc, lk->inertia, tmp);
            mat_T(Rc, RcT, 3, 3);
            mm3(tmp, RcT, bb->I);
            skew(r, S);
            for (int i = 0; i < 3; ++i) {
                bb->Jv[i * ND + i] = 1.0;
                for (int j = 0; j < 3; ++j) bb->Jv[i * ND + 3 + j] = -S[i * 3 + j];
                bb->Jw[i * ND + 3 + i] = 1.0;
            }
            for (int kk = 0; kk <= k; ++kk) {
                double d[3], v[3];
                for (int i = 0; i < 3; ++i) d[i] = c[i] - org[kk][i];
                cross(ax[kk], d, v);
                for (int i = 0; i < 3; ++i) {
                    bb->Jv[i * ND + cols[kk]] = v[i];
                    bb->Jw[i * ND + cols[kk]] = ax[kk][i];
                }
            }
            double d[3], ac[3];
            for (int i = 0; i < 3; ++i) d[i] = c[i] - oj[i];
            cross(alc, d, ac);
            cross(wc, d, t);
            cross(wc, t, u);
            for (int i = 0; i < 3; ++i) ac[i] += ao[i] + u[i];
            memcpy(bb->w, wc, sizeof wc);
            memcpy(bb->alpha, alc, sizeof alc);
            memcpy(bb->a, ac, sizeof ac);
            memcpy(Rp, Rc, sizeof Rp);
            memcpy(op, oj, sizeof op);
            memcpy(wp, wc, sizeof wp);
            memcpy(alp, alc, sizeof alp);
            memcpy(aop, ao, sizeof aop);
        }
        double pf[3], rfB[3], S[9];
        mv3(Rp, md->foot[l], pf);
        for (int i = 0; i < 3; ++i) pf[i] += op[i], rfB[i] = pf[i] - pB[i];
        memcpy(out->foot_pos + 3 * l, pf, sizeof pf);
        skew(rfB, S);
        for (int i = 0; i < 3; ++i) {
            double* row = out->foot_J + (3 * l + i) * ND;
            row[i] = 1.0;
            for (int j = 0; j < 3; ++j) row[3 + j] = -S[i * 3 + j];
        }
        for (int kk = 0; kk < 3; ++kk) {
            double d[3], v[3];
            for (int i = 0; i < 3; ++i) d[i] = pf[i] - org[kk][i];
            cross(ax[kk], d, v);
            for (int i = 0; i < 3; ++i) out->foot_J[(3 * l + i) * ND + cols[kk]] = v[i];
        }
    }
    /* M = sum Jv' m Jv + Jw' I Jw ; h = sum Jv' m a + Jw' (I alpha + w x I w) */
    double msum = 0.0, mc[3] = {0, 0, 0}, mv[3] = {0, 0, 0};
    for (int k = 0; k < 13; ++k) {
        const body_t* bb = &b[k];
        double IJw[3 * ND];
        mat_mul(bb->I, bb->Jw, IJw, 3, 3, ND);
        for (int i = 0; i < ND; ++i)
            for (int j = 0; j < ND; ++j) {
                double s = 0.0;
                for (int t = 0; t < 3; ++t) s += bb->m * bb->Jv[t * ND + i] * bb->Jv[t * ND + j] + bb->Jw[t * ND + i] * IJw[t * ND + j];
                out->M[i * ND + j] += s;
            }
        double Ia[3], Iw[3], wIw[3], N[3];
        mv3(bb->I, bb->alpha, Ia);
        mv3(bb->I, bb->w, Iw);
        cross(bb->w, Iw, wIw);
        for (int i = 0; i < 3; ++i) N[i] = Ia[i] + wIw[i];
        for (int j = 0; j < ND; ++j) {
            double s = 0.0;
            for (int t = 0; t < 3; ++t) s += bb->Jv[t * ND + j] * bb->m * bb->a[t] + bb->Jw[t * ND + j] * N[t];
            out->Cnu[j] += s;
        }
        double v[3];
        mat_mul(bb->Jv, nu, v, 3, ND, 1);
        msum += bb->m;
        for (int i = 0; i < 3; ++i) mc[i] += bb->m * bb->c[i], mv[i] += bb->m * v[i];
    }
    for (int i = 0; i < ND; ++i)
        for (int j = i + 1; j < ND; ++j) {
            double s = 0.5 * (out->M[i * ND + j] + out->M[j * ND + i]);
            out->M[i * ND + j] = out->M[j * ND + i] = s;
        }
    for (int i = 0; i < 3; ++i) out->com[i] = mc[i] / msum, out->com_vel[i] = mv[i] / msum;
    mat_mul(out->foot_J, nu, out->foot_vel, 3 * NL, ND, 1);
    memcpy(out->RB, RB, sizeof RB);
}

/* ------------------------------------------------------------------ Goldfarb-Idnani (dense) */
/* min 1/2 x'Hx + g'x  s.t. CE x = ce (me rows), CI x >= ci (mi rows); n <= NV. */
/* Warm start (qpOASES SQProblem::hotstart from the previous working set, cpp:523-535): the nwarm
 * inequality ids in warm[] (the active set the previous solve ended with, same contact mask) are
 * added after the equalities without steps; the point where every active row holds with equality
 * then gives the multipliers in closed form (R'v = -s_A(x0), u = R^-1 v, x = x0 + J1 v).  A
 * dependent warm row or a multiplier below -1e-10 rejects the warm set and the solve continues
 * from the equality-constrained point, as a cold solve.  Re-adds are not counted in iters (only
 * working-set changes of the loop are).  On return act_out[0..*nact_out) holds the active
 * inequality ids (for the next hotstart). */
/* selnorm / tolv (may be NULL): the selection scale of each inequality (slack / selnorm; default
 * its row norm) and its violation tolerance (default 1e-10 max(1, |ci|)). */
/* Diagnostic trace of the loop's decisions (tools/split_diverge.py): when set, each pass of the
 * inequality loop appends TRACE_W doubles -- iteration, chosen row p, its scaled violation, the
 * closest competing violation outside the tie band, t1, t2, the second-smallest drop ratio, n_p'z,
 * the r[k] closest to the eps threshold, and the dropped row (-1 on an add) -- and the final pass
 * the largest inactive slack / tolerance ratio.  Never set by the tests' checking paths. */
#define TRACE_W 12
static __thread double* g_trace;
static __thread int g_trace_cap, g_trace_n;
void wbc_ref_set_trace(double* buf, int cap) {
    g_trace = buf;
    g_trace_cap = cap;
    g_trace_n = 0;
}
int wbc_ref_trace_len(void) { return g_trace_n; }
static void trace_put(const double* v) {
    if (g_trace && g_trace_n < g_trace_cap) {
        memcpy(g_trace + (size_t)g_trace_n * TRACE_W, v, sizeof(double) * TRACE_W);
        ++g_trace_n;
    }
}

static int gi_solve(int n, const double* H, const double* g, int me, const double* CE, const double* ce, int mi,
                    const double* CI, const double* ci, int max_iter, const int* warm, int nwarm, double* x,
                    int* iters_out, int* act_out, int* nact_out, const double* selnorm, const double* tolv, int rrel) {
    double L[NV * NV], J[NV * NV], R[NV * NV], u[NV], d[NV], z[NV], r[NV], ni[2 * NC], x0[NV];
    if (nact_out) *nact_out = 0;
    int act[NV]; /* >= 0: inequality id ; < 0: equality -(id+1) */
    int q = 0, iters = 0;
    const double eps = 1e-14;
    memset(L, 0, sizeof L);
    /* Cholesky H = L L' */
    for (int j = 0; j < n; ++j) {
        double s = H[j * n + j];
        for (int k = 0; k < j; ++k) s -= L[j * NV + k] * L[j * NV + k];
        if (!(s > 0.0)) return WBC_REF_NUMERIC;
        L[j * NV + j] = sqrt(s);
        for (int i = j + 1; i < n; ++i) {
            double t = H[i * n + j];
            for (int k = 0; k < j; ++k) t -= L[i * NV + k] * L[j * NV + k];
            L[i * NV + j] = t / L[j * NV + j];
        }
    }
    /* J = L^-T : column c of L^-T is row c of L^-1; solve L y = e_c */
    memset(J, 0, sizeof J);
    for (int c = 0; c < n; ++c) {
        double y[NV];
        for (int i = 0; i < n; ++i) {
            double s = (i == c) ? 1.0 : 0.0;
            for (int k = 0; k < i; ++k) s -= L[i * NV + k] * y[k];
            y[i] = s / L[i * NV + i];
        }
        for (int i = 0; i < n; ++i) J[c * NV + i] = y[i]; /* J[c][i] = (L^-1)[i][c] */
    }
    /* x = -H^-1 g = -J J' g */
    {
        double t[NV];
        for (int i = 0; i < n; ++i) {
            double s = 0.0;
            for (int k = 0; k < n; ++k) s += J[k * NV + i] * g[k];
            t[i] = s;
        }
        for (int i = 0; i < n; ++i) {
            double s = 0.0;
            for (int k = 0; k < n; ++k) s += J[i * NV + k] * t[k];
            x[i] = -s;
        }
    }
    memcpy(x0, x, sizeof(double) * n);
    memset(R, 0, sizeof R);
    for (int i = 0; i < mi; ++i) {
        double s = 0.0;
        for (int k = 0; k < n; ++k) s += CI[i * n + k] * CI[i * n + k];
        if (selnorm) s = selnorm[i] * selnorm[i];
        ni[i] = sqrt(s > 1e-300 ? s : 1e-300);
    }
#define COMPUTE_DZR(np_)                                                               \
    do {                                                                               \
        for (int i_ = 0; i_ < n; ++i_) {                                               \
            double s_ = 0.0;                                                           \
            for (int k_ = 0; k_ < n; ++k_) s_ += J[k_ * NV + i_] * (np_)[k_];          \
            d[i_] = s_;                                                                \
        }                                                                              \
        for (int i_ = 0; i_ < n; ++i_) {                                               \
            double s_ = 0.0;                                                           \
            for (int k_ = q; k_ < n; ++k_) s_ += J[i_ * NV + k_] * d[k_];              \
            z[i_] = s_;                                                                \
        }                                                                              \
        for (int i_ = q - 1; i_ >= 0; --i_) {                                          \
            double s_ = d[i_];                                                         \
            for (int k_ = i_ + 1; k_ < q; ++k_) s_ -= R[i_ * NV + k_] * r[k_];         \
            r[i_] = s_ / R[i_ * NV + i_];                                              \
        }                                                                              \
    } while (0)
    /* add: Householder on d[q:], J <- J P ; R column q = [d1; alpha] */
#define ADD_CONSTRAINT(ok_)                                                            \
    do {                                                                               \
        double nrm_ = 0.0, dn_ = 0.0;                                                  \
        for (int k_ = q; k_ < n; ++k_) nrm_ += d[k_] * d[k_];                          \
        for (int k_ = 0; k_ < n; ++k_) dn_ += d[k_] * d[k_];                           \
        nrm_ = sqrt(nrm_);                                                             \
        if (nrm_ <= 1e-14 * (sqrt(dn_) > 1.0 ? sqrt(dn_) : 1.0)) { ok_ = 0; break; }  \
        double alpha_ = d[q] >= 0 ? -nrm_ : nrm_;                                      \
        double v_[NV];                                                                 \
        for (int k_ = q; k_ < n; ++k_) v_[k_] = d[k_];                                 \
        v_[q] -= alpha_;                                                               \
        double vv_ = 0.0;                                                              \
        for (int k_ = q; k_ < n; ++k_) vv_ += v_[k_] * v_[k_];                         \
        for (int i_ = 0; i_ < n; ++i_) {                                               \
            double s_ = 0.0;                                                           \
            for (int k_ = q; k_ < n; ++k_) s_ += J[i_ * NV + k_] * v_[k_];             \
            s_ *= 2.0 / vv_;                                                           \
            for (int k_ = q; k_ < n; ++k_) J[i_ * NV + k_] -= s_ * v_[k_];             \
        }                                                                              \
        for (int i_ = 0; i_ < q; ++i_) R[i_ * NV + q] = d[i_];                         \
        R[q * NV + q] = alpha_;                                                        \
        ++q;                                                                           \
        ok_ = 1;                                                                       \
    } while (0)

    for (int e = 0; e < me; ++e) {
        const double* np_ = CE + e * n;
        COMPUTE_DZR(np_);
        double s = -ce[e], zn = 0.0, nn = 0.0;
        for (int k = 0; k < n; ++k) s += np_[k] * x[k], zn += z[k] * np_[k], nn += np_[k] * np_[k];
        if (fabs(zn) <= eps * (nn > 1.0 ? nn : 1.0)) {
            if (fabs(s) <= 1e-9 * (fabs(ce[e]) > 1.0 ? fabs(ce[e]) : 1.0)) continue;
            *iters_out = 0;
            return WBC_REF_INFEASIBLE;
        }
        double t = -s / zn;
        for (int k = 0; k < n; ++k) x[k] += t * z[k];
        for (int k = 0; k < q; ++k) u[k] -= t * r[k];
        u[q] = t;
        act[q] = -(e + 1);
        int ok = 0;
        ADD_CONSTRAINT(ok);
        if (!ok) return WBC_REF_NUMERIC;
    }
    const int n_eq = q;
    for (int w = 0; w < nwarm; ++w)
        if (warm[w] < 0 || warm[w] >= mi) nwarm = 0;
    if (nwarm > 0 && n_eq + nwarm <= n) {
        static __thread double Js[NV * NV], Rs[NV * NV];
        double xs[NV], us[NV];
        int acts[NV];
        memcpy(Js, J, sizeof J);
        memcpy(Rs, R, sizeof R);
        memcpy(xs, x, sizeof xs);
        memcpy(us, u, sizeof us);
        memcpy(acts, act, sizeof acts);
        int ok = 1;
        for (int w = 0; w < nwarm && ok; ++w) {
            const double* np_ = CI + warm[w] * n;
            for (int i = 0; i < n; ++i) {
                double s_ = 0.0;
                for (int k = 0; k < n; ++k) s_ += J[k * NV + i] * np_[k];
                d[i] = s_;
            }
            act[q] = warm[w];
            ADD_CONSTRAINT(ok);
        }
        if (ok) {
            /* R' v = -s_A(x0) (forward), u = R^-1 v (backward), x = x0 + J[:, 0:q] v */
            double v[NV], sa[NV];
            for (int k = 0; k < q; ++k) {
                const double* row = act[k] < 0 ? CE + (-act[k] - 1) * n : CI + act[k] * n;
                double s_ = act[k] < 0 ? -ce[-act[k] - 1] : -ci[act[k]];
                for (int i = 0; i < n; ++i) s_ += row[i] * x0[i];
                sa[k] = s_;
            }
            for (int k = 0; k < q; ++k) {
                double s_ = -sa[k];
                for (int i = 0; i < k; ++i) s_ -= R[i * NV + k] * v[i];
                v[k] = s_ / R[k * NV + k];
            }
            for (int k = q - 1; k >= 0; --k) {
                double s_ = v[k];
                for (int i = k + 1; i < q; ++i) s_ -= R[k * NV + i] * u[i];
                u[k] = s_ / R[k * NV + k];
            }
            for (int k = n_eq; k < q; ++k)
                if (u[k] < -1e-10) ok = 0;
            if (ok) {
                for (int i = 0; i < n; ++i) {
                    double s_ = x0[i];
                    for (int k = 0; k < q; ++k) s_ += J[i * NV + k] * v[k];
                    x[i] = s_;
                }
                for (int k = n_eq; k < q; ++k)
                    if (u[k] < 0.0) u[k] = 0.0;
            }
        }
        if (!ok) { /* reject: back to the equality-constrained point */
            memcpy(J, Js, sizeof J);
            memcpy(R, Rs, sizeof R);
            memcpy(x, xs, sizeof xs);
            memcpy(u, us, sizeof us);
            memcpy(act, acts, sizeof acts);
            q = n_eq;
        }
    }
#define GI_RETURN(st_)                                                                 \
    do {                                                                               \
        if (act_out && nact_out) {                                                     \
            for (int k_ = n_eq; k_ < q; ++k_) act_out[k_ - n_eq] = act[k_];           \
            *nact_out = q - n_eq;                                                      \
        }                                                                              \
        return (st_);                                                                  \
    } while (0)
    for (;;) {
        /* most violated inactive inequality (scaled).  Near-ties are ties: the lowest row id among
         * the rows within WBC_TIE_BAND (relative) of the most violated one, the rule the engine's
         * kernels apply (wbc_kernel.hip solve16 / solve_phase / solve_stance), so rounding cannot
         * send the two down different routes when two rows are violated alike in exact arithmetic
         * (the +-x faces of a foot with f_x = 0) */
        int p = -1;
        double best = 0.0, wv[2 * NC];
        for (int i = 0; i < mi; ++i) {
            wv[i] = 0.0;
            int isact = 0;
            for (int k = n_eq; k < q; ++k)
                if (act[k] == i) { isact = 1; break; }
            if (isact) continue;
            double s = -ci[i];
            for (int k = 0; k < n; ++k) s += CI[i * n + k] * x[k];
            double tol = tolv ? tolv[i] : 1e-10 * (fabs(ci[i]) > 1.0 ? fabs(ci[i]) : 1.0);
            if (s < -tol) {
                wv[i] = s / ni[i];
                if (wv[i] < best) best = wv[i];
            }
        }
        if (best < 0.0) {
            const double thr = best * (1.0 - WBC_TIE_BAND);
            for (int i = 0; i < mi && p < 0; ++i)
                if (wv[i] < 0.0 && wv[i] <= thr) p = i;
        }
        double tr[TRACE_W] = {0};
        if (g_trace) {
            /* closest competitor outside the band; closest inactive slack to its tolerance */
            double second = 0.0, near = 0.0;
            const double thr = best * (1.0 - WBC_TIE_BAND);
            for (int i = 0; i < mi; ++i) {
                if (wv[i] < 0.0 && wv[i] > thr && wv[i] < second) second = wv[i];
                int isact = 0;
                for (int k = n_eq; k < q; ++k)
                    if (act[k] == i) { isact = 1; break; }
                if (isact || wv[i] < 0.0) continue;
                double sl = -ci[i];
                for (int k = 0; k < n; ++k) sl += CI[i * n + k] * x[k];
                const double tol = tolv ? tolv[i] : 1e-10 * (fabs(ci[i]) > 1.0 ? fabs(ci[i]) : 1.0);
                if (-sl / tol > near) near = -sl / tol;
            }
            tr[0] = iters; tr[1] = p; tr[2] = best; tr[3] = second; tr[10] = near;
        }
        if (p < 0) { if (g_trace) { tr[1] = -2; trace_put(tr); } *iters_out = iters; GI_RETURN(WBC_REF_OK); }
        const double* np_ = CI + p * n;
        double sp = -ci[p];
        for (int k = 0; k < n; ++k) sp += np_[k] * x[k];
        double up = 0.0;
        for (;;) {
            if (++iters > max_iter) { *iters_out = max_iter; return WBC_REF_MAX_ITER; }
            COMPUTE_DZR(np_);
            double t1 = INFINITY;
            int l = -1;
            /* rrel (the literal / 24-variable form, WBC_R_REL): an r[k] that is rounding noise next to
             * the largest |r| (a pending row dependent on the active set, z = 0: the infeasibility
             * test) is not a drop candidate, so the two forms' different rounding cannot take
             * different numbers of noise drops before INFEASIBLE */
            double rthr = eps;
            if (rrel) {
                double rmax = 0.0;
                for (int k = 0; k < q; ++k) rmax = fabs(r[k]) > rmax ? fabs(r[k]) : rmax;
                if (WBC_R_REL * rmax > rthr) rthr = WBC_R_REL * rmax;
            }
            for (int k = n_eq; k < q; ++k)
                if (r[k] > rthr && u[k] / r[k] < t1) { t1 = u[k] / r[k]; l = k; }
            double zz = 0.0, zn = 0.0;
            for (int k = 0; k < n; ++k) zz += z[k] * z[k], zn += z[k] * np_[k];
            double t2 = (zz > eps * eps && zn > eps) ? -sp / zn : INFINITY;
            double t = t1 < t2 ? t1 : t2;
            if (g_trace) {
                double t1b = INFINITY, rnear = INFINITY, rmax = 0.0;
                for (int k = 0; k < q; ++k) rmax = fabs(r[k]) > rmax ? fabs(r[k]) : rmax;
                tr[11] = rmax;
                for (int k = n_eq; k < q; ++k) {
                    if (r[k] > eps && k != l && u[k] / r[k] < t1b) t1b = u[k] / r[k];
                    const double ar = fabs(r[k]);
                    if (ar > 1e-17 && fabs(log10(ar / eps)) < fabs(log10(rnear / eps))) rnear = ar;
                }
                tr[0] = iters; tr[4] = t1; tr[5] = t2; tr[6] = t1b; tr[7] = zn; tr[8] = rnear;
                tr[9] = (isfinite(t2) && t == t2) ? -1 : (l >= 0 ? act[l] : -3);
                trace_put(tr);
                tr[1] = -1; tr[2] = tr[3] = 0.0;  /* a drop's next pass: same p, no new selection */
            }
            if (!isfinite(t)) { *iters_out = iters; return WBC_REF_INFEASIBLE; }
            if (isfinite(t2)) {
                for (int k = 0; k < n; ++k) x[k] += t * z[k];
                sp += t * zn;
            }
            for (int k = 0; k < q; ++k) u[k] -= t * r[k];
            up += t;
            if (isfinite(t2) && t == t2) {
                u[q] = up;
                act[q] = p;
                int ok = 0;
                ADD_CONSTRAINT(ok);
                if (!ok) return WBC_REF_NUMERIC;
                break;
            }
            /* drop slot l: delete column, Givens on rows of R, mirror on J columns */
            for (int k = l; k < q - 1; ++k) {
                for (int i = 0; i < n; ++i) R[i * NV + k] = R[i * NV + k + 1];
                u[k] = u[k + 1];
                act[k] = act[k + 1];
            }
            for (int i = 0; i < n; ++i) R[i * NV + q - 1] = 0.0;
            for (int j = l; j < q - 1; ++j) {
                double a = R[j * NV + j], bb = R[(j + 1) * NV + j], h = hypot(a, bb), c = 1.0, s = 0.0;
                if (h > 0) { c = a / h; s = bb / h; }
                for (int k = j; k < q - 1; ++k) {
                    double r1 = R[j * NV + k], r2 = R[(j + 1) * NV + k];
                    R[j * NV + k] = c * r1 + s * r2;
                    R[(j + 1) * NV + k] = -s * r1 + c * r2;
                }
                for (int i = 0; i < n; ++i) {
                    double j1 = J[i * NV + j], j2 = J[i * NV + j + 1];
                    J[i * NV + j] = c * j1 + s * j2;
                    J[i * NV + j + 1] = -s * j1 + c * j2;
                }
            }
            --q;
        }
    }
#undef COMPUTE_DZR
#undef ADD_CONSTRAINT
#undef GI_RETURN
}

/* qpOASES general constraints lbA <= A x <= ubA -> (CE, CI); identically-zero rows (quirk A.12) are
 * dropped when feasible for x, flagged infeasible otherwise; two-sided rows are split. */
static int solve_qp(const double* H, const double* g, const double* A, const double* lb, const double* ub, int max_iter,
                    const int* warm, int nwarm, double* x, int* iters, int* act_out, int* nact_out) {
    static const int n = NV;
    double CE[NC * NV], ce[NC], CI[2 * NC * NV], ci[2 * NC];
    int me = 0, mi = 0;
    for (int i = 0; i < NC; ++i) {
        const double* row = A + i * n;
        int nz = 0;
        for (int k = 0; k < n; ++k)
            if (row[k] != 0.0) { nz = 1; break; }
        const int lo_inf = lb[i] <= -QP_INFTY, hi_inf = ub[i] >= QP_INFTY;
        if (!nz) {
            if ((!lo_inf && lb[i] > 1e-9 * (fabs(lb[i]) > 1 ? fabs(lb[i]) : 1)) ||
                (!hi_inf && ub[i] < -1e-9 * (fabs(ub[i]) > 1 ? fabs(ub[i]) : 1))) {
                memset(x, 0, sizeof(double) * n);
                *iters = 0;
                return WBC_REF_INFEASIBLE;
            }
            continue;
        }
        if (!lo_inf && !hi_inf && lb[i] == ub[i]) {
            memcpy(CE + me * n, row, sizeof(double) * n);
            ce[me++] = lb[i];
            continue;
        }
        if (!lo_inf) {
            memcpy(CI + mi * n, row, sizeof(double) * n);
            ci[mi++] = lb[i];
        }
        if (!hi_inf) {
            for (int k = 0; k < n; ++k) CI[mi * n + k] = -row[k];
            ci[mi++] = -ub[i];
        }
    }
    return gi_solve(n, H, g, me, CE, ce, mi, CI, ci, max_iter, warm, nwarm, x, iters, act_out, nact_out, NULL, NULL, 1);
}

/* The dense Goldfarb-Idnani above for other callers (oracle/wbc_fast.c), cold (no warm set). */
int wbc_ref_gi(int n, const double* H, const double* g, int me, const double* CE, const double* ce, int mi, const double* CI,
               const double* ci, int max_iter, double* x, int* iters) {
    return gi_solve(n, H, g, me, CE, ce, mi, CI, ci, max_iter, NULL, 0, x, iters, NULL, NULL, NULL, NULL, 0);
}

/* ------------------------------------------------------------------ the engine's 12-variable form */
/* The same QP reduced exactly to 12 variables for every contact mask (the numpy
 * restatement oracle/wbc_reduced.py documents the derivation): z = one 3-slot per leg (a swing
 * leg's joint accelerations, a stance leg's force); a and the swing slacks eliminated (s_i = |r_i|,
 * the pair of slack rows becomes the penalty 1/2 w r_i^2), the stance equalities solved for the
 * stance joints by Woodbury (qdd_S = q0 + Y phi, phi = B z).  Inequality rows in the engine's
 * numbering: friction face 4 l + rr of stance leg l, torque row 16 + 2 j (+ side) / 16 + 2 j + 1
 * (- side).  Selected by slack / |reference row| with the reference row's tolerance, as the
 * kernel (wbc_kernel.hip solve16) does, so both count the same working-set changes; hotstart from
 * the previous solve's set in this numbering (friction rows of legs no longer in contact dropped).
 * Returns the QP status, or -1 when the elimination is not usable (a near-singular stance leg or
 * S6): the engine then solves the literal form, and so does the caller. */
static int reduced_solve(const wbc_params* pr, wbc_ref_state* st, const wbc_ref_kindyn_t* kd, const double* T,
                         const double* Tinv, const double* Mbar_b, const double* Mbar_j, const double* bbar,
                         const double* W, const double* r1, const double* rsw, const int* kap, double* x, double* tau,
                         int* iters) {
    double Jbar[12 * ND], E[12 * 6], Jbj[144], K[6 * 12], Jl[4][9];
    mat_mul(kd->foot_J, Tinv, Jbar, 12, ND, ND);
    for (int i = 0; i < 12; ++i) {
        for (int c = 0; c < 6; ++c) E[i * 6 + c] = Jbar[i * ND + c];
        for (int j = 0; j < 12; ++j) Jbj[i * 12 + j] = Jbar[i * ND + 6 + j];
    }
    for (int a = 0; a < 6; ++a)
        for (int j = 0; j < 12; ++j) K[a * 12 + j] = T[a * ND + 6 + j]; /* Jbj = Jblk - E K */
    for (int l = 0; l < 4; ++l)
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) Jl[l][3 * r + c] = kd->foot_J[(3 * l + r) * ND + 6 + 3 * l + c];
    double Mbi[36];
    if (mat_inv(Mbar_b, Mbi, 6)) return -1;
    const double g0 = pr->gravity, wsw = pr->slack_weight;
    int stj[12];
    for (int i = 0; i < 12; ++i) stj[i] = kap[i / 3];
    /* stance rows: W = J_S^-1 E_S, w = J_S^-1 e_S */
    double Wr[72] = {0}, w[12] = {0};
    for (int l = 0; l < 4; ++l) {
        if (!kap[l]) continue;
        double Ji[9], det, amx = 0.0;
        for (int t = 0; t < 9; ++t) amx = fmax(amx, fabs(Jl[l][t]));
        double c00 = Jl[l][4] * Jl[l][8] - Jl[l][5] * Jl[l][7], c01 = Jl[l][5] * Jl[l][6] - Jl[l][3] * Jl[l][8],
               c02 = Jl[l][3] * Jl[l][7] - Jl[l][4] * Jl[l][6];
        det = Jl[l][0] * c00 + Jl[l][1] * c01 + Jl[l][2] * c02;
        if (!(fabs(det) > 1e-9 * amx * amx * amx)) return -1;
        if (mat_inv(Jl[l], Ji, 3)) return -1;
        for (int k = 0; k < 3; ++k) {
            const int i = 3 * l + k;
            for (int c = 0; c < 6; ++c) {
                double t = 0.0;
                for (int kk = 0; kk < 3; ++kk) t += Ji[k * 3 + kk] * E[(3 * l + kk) * 6 + c];
                Wr[i * 6 + c] = t;
            }
            double t = 0.0;
            for (int kk = 0; kk < 3; ++kk) t += Ji[k * 3 + kk] * (r1[3 * l + kk] + (kk == 2 ? g0 : 0.0));
            w[i] = t;
        }
    }
    double S6[36], S6i[36], z6[6];
    for (int a = 0; a < 6; ++a) {
        for (int b = 0; b < 6; ++b) {
            double t = (a == b) ? 1.0 : 0.0;
            for (int j = 0; j < 12; ++j) t -= K[a * 12 + j] * Wr[j * 6 + b];
            S6[a * 6 + b] = t;
        }
        double t = 0.0;
        for (int j = 0; j < 12; ++j) t += K[a * 12 + j] * w[j];
        z6[a] = t;
    }
    {
        double smx = 0.0, pmin = 1e300, LU[36];
        for (int t = 0; t < 36; ++t) smx = fmax(smx, fabs(S6[t]));
        memcpy(LU, S6, sizeof LU); /* pivots of Gauss-Jordan without pivoting, as the kernel */
        for (int k = 0; k < 6; ++k) {
            pmin = fmin(pmin, fabs(LU[k * 6 + k]));
            for (int i = k + 1; i < 6; ++i) {
                const double f = LU[i * 6 + k] / LU[k * 6 + k];
                for (int j = k; j < 6; ++j) LU[i * 6 + j] -= f * LU[k * 6 + j];
            }
        }
        if (!(pmin > 1e-6 * smx)) return -1;
        if (mat_inv(S6, S6i, 6)) return -1;
    }
    double Y[72], q0[12];
    for (int i = 0; i < 12; ++i) {
        double q = w[i];
        for (int c = 0; c < 6; ++c) {
            double t = 0.0;
            for (int b = 0; b < 6; ++b) t += Wr[i * 6 + b] * S6i[b * 6 + c];
            Y[i * 6 + c] = t;
            q += t * z6[c];
        }
        q0[i] = q;
    }
    /* B (phi = B z), P (E_S^T f), the leg rows Rho = own + v^T B with rho0 and weights */
    double B[6 * 12] = {0}, P[6 * 12] = {0}, cpsi[6] = {0, 0, -g0, 0, 0, 0};
    for (int j = 0; j < 12; ++j) {
        for (int a = 0; a < 6; ++a) {
            if (stj[j]) {
                double t = 0.0;
                for (int b = 0; b < 6; ++b) t += Mbi[a * 6 + b] * E[j * 6 + b];
                B[a * 12 + j] = -t;
                P[a * 12 + j] = E[j * 6 + a];
            } else {
                B[a * 12 + j] = K[a * 12 + j];
            }
            if (stj[j]) cpsi[a] -= K[a * 12 + j] * q0[j];
        }
    }
    double Rho[144] = {0}, rho0[12], wt[12], V6[72];
    for (int i = 0; i < 12; ++i) {
        const int l = i / 3, k = i % 3;
        double v[6];
        if (stj[i]) {
            for (int c = 0; c < 6; ++c) v[c] = Y[i * 6 + c];
            rho0[i] = q0[i];
            wt[i] = 1.0;
        } else {
            for (int c = 0; c < 6; ++c) {
                double t = 0.0;
                for (int b = 0; b < 6; ++b) t += S6i[b * 6 + c] * E[i * 6 + b];
                v[c] = -t;
            }
            double ec = 0.0;
            for (int c = 0; c < 6; ++c) ec += E[i * 6 + c] * cpsi[c];
            rho0[i] = ec - rsw[i];
            wt[i] = wsw;
            for (int c = 0; c < 3; ++c) Rho[i * 12 + 3 * l + c] = Jl[l][3 * k + c];
        }
        for (int c = 0; c < 6; ++c) V6[i * 6 + c] = v[c];
        for (int j = 0; j < 12; ++j) {
            double t = 0.0;
            for (int c = 0; c < 6; ++c) t += v[c] * B[c * 12 + j];
            Rho[i * 12 + j] += t;
        }
    }
    double H[144], g[12];
    {
        double CP[36];
        for (int a = 0; a < 6; ++a)
            for (int b = 0; b < 6; ++b) {
                double t = (a == b) ? 1.0 : 0.0;
                for (int c = 0; c < 6; ++c) t += Mbi[a * 6 + c] * Mbi[c * 6 + b];
                CP[a * 6 + b] = t;
            }
        for (int a = 0; a < 12; ++a)
            for (int j = 0; j < 12; ++j) {
                double t = (a == j) ? 1.0 : 0.0;
                for (int c = 0; c < 6; ++c)
                    for (int d = 0; d < 6; ++d) t += P[c * 12 + a] * CP[c * 6 + d] * P[d * 12 + j];
                for (int i = 0; i < 12; ++i) t += wt[i] * Rho[i * 12 + a] * Rho[i * 12 + j];
                H[a * 12 + j] = t;
            }
        const double wv[6] = {W[0], W[1], W[2] + g0 / (Mbar_b[0]), W[3], W[4], W[5]};
        for (int a = 0; a < 12; ++a) {
            double t = 0.0;
            for (int c = 0; c < 6; ++c) t -= P[c * 12 + a] * wv[c];
            for (int i = 0; i < 12; ++i) t += wt[i] * Rho[i * 12 + a] * rho0[i];
            g[a] = t;
        }
    }
    /* torque map and the inequality rows */
    double t0[12], Nt[144], nselr[12];
    for (int r = 0; r < 12; ++r) {
        double my[6] = {0}, t = bbar[6 + r], s2 = 0.0;
        for (int s_ = 0; s_ < 12; ++s_) {
            const double mk = Mbar_j[r * 12 + s_];
            s2 += mk * mk;
            if (stj[s_]) {
                s2 += Jbj[s_ * 12 + r] * Jbj[s_ * 12 + r];
                t += mk * q0[s_];
                for (int c = 0; c < 6; ++c) my[c] += mk * Y[s_ * 6 + c];
            }
        }
        t0[r] = t;
        nselr[r] = s2;
        for (int j = 0; j < 12; ++j) {
            double v = stj[j] ? Jbj[j * 12 + r] : -Mbar_j[r * 12 + j];
            for (int c = 0; c < 6; ++c) v -= my[c] * B[c * 12 + j];
            Nt[r * 12 + j] = v;
        }
    }
    const double mu = pr->friction, tm = pr->max_torque;
    const double D[12] = {1, 0, -mu, -1, 0, -mu, 0, 1, -mu, 0, -1, -mu};
    double CI[40 * 12], ci[40], seln[40], tolv[40];
    int ids[40], mi = 0, idpos[40];
    for (int t = 0; t < 40; ++t) idpos[t] = -1;
    for (int l = 0; l < 4; ++l) {
        if (!kap[l]) continue;
        for (int rr = 0; rr < 4; ++rr) {
            for (int j = 0; j < 12; ++j) CI[mi * 12 + j] = 0.0;
            for (int c = 0; c < 3; ++c) CI[mi * 12 + 3 * l + c] = -D[rr * 3 + c];
            ci[mi] = 0.0;
            seln[mi] = sqrt(1.0 + mu * mu);
            tolv[mi] = 1e-10;
            ids[mi] = 4 * l + rr;
            idpos[4 * l + rr] = mi;
            ++mi;
        }
    }
    for (int j = 0; j < 12; ++j)
        for (int side = 0; side < 2; ++side) {
            const double sg = side ? -1.0 : 1.0;
            for (int c = 0; c < 12; ++c) CI[mi * 12 + c] = -sg * Nt[j * 12 + c];
            ci[mi] = -tm - sg * t0[j];
            seln[mi] = sqrt(nselr[j] > 1e-300 ? nselr[j] : 1e-300);
            const double bref = -tm - sg * bbar[6 + j];
            tolv[mi] = 1e-10 * (fabs(bref) > 1.0 ? fabs(bref) : 1.0);
            ids[mi] = 16 + 2 * j + side;
            idpos[16 + 2 * j + side] = mi;
            ++mi;
        }
    /* vacuous rows (quirk A.12): a swing leg's R1 row reads 0 = r1 */
    for (int i = 0; i < 12; ++i)
        if (!stj[i] && fabs(r1[i]) > 1e-9 * (fabs(r1[i]) > 1.0 ? fabs(r1[i]) : 1.0)) {
            *iters = 0;
            st->ws12 = 0;
            st->ws12_valid = 1;
            return WBC_REF_INFEASIBLE;
        }
    int warm[12], nwarm = 0;
    if (st->first && !st->cold_qp && st->ws12_valid) {
        for (int id = 0; id < 40; ++id)
            if (((st->ws12 >> id) & 1ull) && idpos[id] >= 0) {
                if (nwarm < 12) warm[nwarm] = idpos[id];
                ++nwarm;
            }
        if (nwarm > 12) nwarm = 0;
    }
    double z[NV]; /* gi_solve saves and restores NV entries (warm start) */
    int act[NV], nact = 0;
    const int status = gi_solve(12, H, g, 0, NULL, NULL, mi, CI, ci, pr->max_wsr, nwarm ? warm : NULL, nwarm, z, iters, act,
                                &nact, seln, tolv, 0);
    st->ws12 = 0;
    st->ws12_valid = 1;
    if (status == WBC_REF_OK)
        for (int k = 0; k < nact; ++k) st->ws12 |= 1ull << ids[act[k]];
    if (status != WBC_REF_OK) return status;
    /* back to the 42 variables */
    double phi[6];
    for (int c = 0; c < 6; ++c) {
        double t = 0.0;
        for (int j = 0; j < 12; ++j) t += B[c * 12 + j] * z[j];
        phi[c] = t;
    }
    double ef[6];
    for (int c = 0; c < 6; ++c) {
        double t = 0.0;
        for (int j = 0; j < 12; ++j) t += P[c * 12 + j] * z[j];
        ef[c] = t;
    }
    for (int a = 0; a < 6; ++a) {
        double t = (a == 2) ? -g0 : 0.0;
        for (int b = 0; b < 6; ++b) t += Mbi[a * 6 + b] * ef[b];
        x[a] = t;
    }
    for (int i = 0; i < 12; ++i) {
        double qv = z[i];
        if (stj[i]) {
            qv = q0[i];
            for (int c = 0; c < 6; ++c) qv += Y[i * 6 + c] * phi[c];
        }
        x[6 + i] = qv;
        x[18 + i] = stj[i] ? z[i] : 0.0;
        double r = rho0[i];
        for (int j = 0; j < 12; ++j) r += Rho[i * 12 + j] * z[j];
        x[30 + i] = stj[i] ? fabs(rsw[i]) : fabs(r);
    }
    for (int r = 0; r < 12; ++r) {
        double t = t0[r];
        for (int j = 0; j < 12; ++j) t -= Nt[r * 12 + j] * z[j];
        tau[r] = t;
    }
    (void)V6;
    return status;
}

/* ------------------------------------------------------------------ controller */
void wbc_ref_state_init(wbc_ref_state* s) { /* setInitialState, cpp:65-120 (history part) */
    memset(s, 0, sizeof(*s));
    for (int i = 0; i < ND; ++i) s->old_T[i * ND + i] = 1.0;
    s->contacts = 15;
}

int wbc_ref_step(const wbc_model* md, const wbc_params* pr, wbc_ref_state* st, const double* pose, const double* nu,
                 const double* qj, const double* ref, int contacts, int switching, double* tau, double* grf, double* x,
                 int* iters, wbc_ref_debug_t* dbg) {
    wbc_ref_kindyn_t kd;
    wbc_ref_kindyn(md, pose, nu, qj, &kd);
    const double* pB = pose;
    const double mtot = md->total_mass;
    int kap[NL];
    for (int l = 0; l < NL; ++l) kap[l] = (contacts >> l) & 1;
    /* updateState (cpp:256-294) */
    double vc[6] = {kd.com_vel[0], kd.com_vel[1], kd.com_vel[2], nu[3], nu[4], nu[5]};
    const double* R = kd.RB;
    double cur_pose[6] = {kd.com[0], kd.com[1], kd.com[2], atan2(R[7], R[8]),
                          atan2(-R[6], sqrt(R[7] * R[7] + R[8] * R[8])), atan2(R[3], R[0])};
    const double* M = kd.M;
    double Mbb[36], Mbbinv[36];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) Mbb[i * 6 + j] = M[i * ND + j];
    /* computeTransformationMatrix (cpp:296-320) */
    double T[ND * ND];
    {
        double Adinv[36], S[9], rr[3], tmp1[36], sel_M[6 * ND], full[6 * ND];
        for (int i = 0; i < 3; ++i) rr[i] = kd.com[i] - pB[i];
        skew(rr, S);
        memset(Adinv, 0, sizeof Adinv);
        for (int i = 0; i < 6; ++i) Adinv[i * 6 + i] = 1.0;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Adinv[i * 6 + 3 + j] = -S[i * 3 + j];
        if (mat_inv(Mbb, Mbbinv, 6)) return WBC_REF_NUMERIC;
        mat_mul(Adinv, Mbbinv, tmp1, 6, 6, 6);
        for (int i = 0; i < 6; ++i) memcpy(sel_M + i * ND, M + i * ND, sizeof(double) * ND); /* [I 0] M */
        mat_mul(tmp1, sel_M, full, 6, 6, ND);
        memset(T, 0, sizeof T);
        memcpy(T, full, sizeof full);
        for (int i = 6; i < ND; ++i) T[i * ND + i] = 1.0;
    }
    double Tinv[ND * ND], TinvT[ND * ND], Mbar[ND * ND], tmpA[ND * ND];
    if (mat_inv(T, Tinv, ND)) return WBC_REF_NUMERIC; /* cpp:270 */
    mat_T(Tinv, TinvT, ND, ND);
    mat_mul(TinvT, M, tmpA, ND, ND, ND);
    if (mat_inv(T, Tinv, ND)) return WBC_REF_NUMERIC; /* cpp:270 (second evaluation) */
    mat_mul(tmpA, Tinv, Mbar, ND, ND, ND);
    double Mbar_b[36], Mbar_j[NJ * NJ];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) Mbar_b[i * 6 + j] = Mbar[i * ND + j];
    for (int i = 0; i < NJ; ++i)
        for (int j = 0; j < NJ; ++j) Mbar_j[i * NJ + j] = Mbar[(6 + i) * ND + 6 + j];
    /* computeJacobians (cpp:322-342) */
    double Jst[3 * NL * ND], Jsw[3 * NL * ND], Jc[3 * NL * ND], Js[3 * NL * ND];
    for (int i = 0; i < 3 * NL; ++i)
        for (int j = 0; j < ND; ++j) {
            const double v = kd.foot_J[i * ND + j];
            Jst[i * ND + j] = v * kap[i / 3];
            Jsw[i * ND + j] = v * (!kap[i / 3]);
        }
    if (mat_inv(T, Tinv, ND)) return WBC_REF_NUMERIC; /* cpp:278 */
    mat_mul(Jst, Tinv, Jc, 3 * NL, ND, ND);
    if (mat_inv(T, Tinv, ND)) return WBC_REF_NUMERIC; /* cpp:282 */
    mat_mul(Jsw, Tinv, Js, 3 * NL, ND, ND);
    /* centroidGeneralizedBias_ = T^-T (C nu + M Tdot_inv nu) (cpp:289) */
    double bbar[ND];
    {
        double t1[ND], h[ND];
        mat_mul(st->Tdot_inv, nu, t1, ND, ND, 1);
        mat_mul(M, t1, h, ND, ND, 1);
        for (int i = 0; i < ND; ++i) h[i] += kd.Cnu[i];
        if (mat_inv(T, Tinv, ND)) return WBC_REF_NUMERIC;
        mat_T(Tinv, TinvT, ND, ND);
        mat_mul(TinvT, h, bbar, ND, ND, 1);
    }
    /* computeDerivatives (cpp:384-402) */
    double Tdot[ND * ND], Jc_dot[3 * NL * ND], Js_dot[3 * NL * ND];
    if (switching) {
        memset(Tdot, 0, sizeof Tdot);
        memset(Jc_dot, 0, sizeof Jc_dot);
        memset(Js_dot, 0, sizeof Js_dot);
    } else {
        const double dt = 1.0 / pr->loop_rate;
        for (int i = 0; i < ND * ND; ++i) Tdot[i] = (T[i] - st->old_T[i]) / dt;
        for (int i = 0; i < 3 * NL * ND; ++i) {
            Jc_dot[i] = (Jc[i] - st->old_Jc[i]) / dt;
            Js_dot[i] = (Js[i] - st->old_Js[i]) / dt;
        }
    }
    memcpy(st->old_T, T, sizeof T);
    memcpy(st->old_Jc, Jc, sizeof Jc);
    memcpy(st->old_Js, Js, sizeof Js);
    /* Tdot_inv = -T^-1 Tdot T^-1 (cpp:293) */
    {
        double t1[ND * ND];
        if (mat_inv(T, Tinv, ND)) return WBC_REF_NUMERIC;
        mat_mul(Tinv, Tdot, t1, ND, ND, ND);
        if (mat_inv(T, Tinv, ND)) return WBC_REF_NUMERIC;
        mat_mul(t1, Tinv, st->Tdot_inv, ND, ND, ND);
        for (int i = 0; i < ND * ND; ++i) st->Tdot_inv[i] = -st->Tdot_inv[i];
    }
    /* solveQP (cpp:466-542) */
    static _Thread_local double H[NV * NV], A[NC * NV];  /* per thread: the CPU baseline runs robots in parallel */
    double g[NV], lb[NC], ub[NC], W[6];
    {
        const int sl = 6 + NJ + 3 * NL;
        memset(H, 0, sizeof H);
        /* S' Jc_com Q Jc_com' S + R,  Q = I6, R = I42 with slack block slackWeight I */
        for (int i = 0; i < 3 * NL; ++i)
            for (int j = 0; j < 3 * NL; ++j) {
                double s = 0.0;
                for (int k = 0; k < 6; ++k) s += Jc[i * ND + k] * Jc[j * ND + k];
                H[(18 + i) * NV + 18 + j] = s;
            }
        for (int i = 0; i < NV; ++i) H[i * NV + i] += (i >= sl) ? pr->slack_weight : 1.0;
        /* computeDesiredWrench (cpp:426-445) */
        const double gw[6] = {0, 0, mtot * pr->gravity, 0, 0, 0};
        for (int k = 0; k < 6; ++k) {
            double mba = 0.0;
            for (int j = 0; j < 6; ++j) mba += Mbar_b[k * 6 + j] * ref[12 + j];
            const double kp = (k == 2) ? pr->kp_z : pr->kp;
            W[k] = -kp * (cur_pose[k] - ref[k]) - pr->kd * (vc[k] - ref[6 + k]) - pr->ki * st->e_int[k] + gw[k] + mba;
        }
        for (int k = 0; k < 6; ++k) st->e_int[k] += (cur_pose[k] - ref[k]) / pr->loop_rate;
        memset(g, 0, sizeof g);
        for (int i = 0; i < 3 * NL; ++i) {
            double s = 0.0;
            for (int k = 0; k < 6; ++k) s += Jc[i * ND + k] * W[k];
            g[18 + i] = -s;
        }
        /* computeNonSlidingConstraints (cpp:404-424) */
        const double mu = pr->friction;
        const double D[12] = {1, 0, -mu, -1, 0, -mu, 0, 1, -mu, 0, -1, -mu};
        memset(A, 0, sizeof A);
        for (int i = 0; i < 6; ++i) { /* R0 */
            for (int j = 0; j < 6; ++j) A[i * NV + j] = Mbar_b[i * 6 + j];
            for (int j = 0; j < 3 * NL; ++j) A[i * NV + 18 + j] = -Jc[j * ND + i];
        }
        for (int i = 0; i < 3 * NL; ++i) { /* R1 */
            for (int j = 0; j < ND; ++j) A[(6 + i) * NV + j] = Jc[i * ND + j];
        }
        for (int l = 0; l < NL; ++l) /* R2 */
            for (int rr = 0; rr < 4; ++rr)
                for (int c = 0; c < 3; ++c) A[(18 + 4 * l + rr) * NV + 18 + 3 * l + c] = D[rr * 3 + c] * kap[l];
        for (int i = 0; i < NJ; ++i) { /* R3 */
            for (int j = 0; j < NJ; ++j) A[(34 + i) * NV + 6 + j] = Mbar_j[i * NJ + j];
            for (int j = 0; j < 3 * NL; ++j) A[(34 + i) * NV + 18 + j] = -Jc[j * ND + 6 + i];
        }
        for (int i = 0; i < 3 * NL; ++i) { /* R4, R5 */
            for (int j = 0; j < ND; ++j) A[(46 + i) * NV + j] = A[(58 + i) * NV + j] = Js[i * ND + j];
            A[(46 + i) * NV + 30 + i] = -1.0;
            A[(58 + i) * NV + 30 + i] = 1.0;
        }
        /* bounds (cpp:503-515); computeCommandedAccelerationSwingLegs (cpp:447-464) */
        double cmd[3 * NL];
        for (int i = 0; i < 3 * NL; ++i)
            cmd[i] = (ref[42 + i] + pr->kd_swing * (ref[30 + i] - kd.foot_vel[i]) + pr->kp_swing * (ref[18 + i] - kd.foot_pos[i])) *
                     (!kap[i / 3]);
        for (int i = 0; i < 6; ++i) lb[i] = ub[i] = -gw[i];
        for (int i = 0; i < 3 * NL; ++i) {
            double s1 = 0.0, s2 = 0.0;
            for (int k = 0; k < 6; ++k) s1 += Jc_dot[i * ND + k] * vc[k], s2 += Js_dot[i * ND + k] * vc[k];
            for (int k = 0; k < NJ; ++k) s1 += Jc_dot[i * ND + 6 + k] * nu[6 + k], s2 += Js_dot[i * ND + 6 + k] * nu[6 + k];
            lb[6 + i] = ub[6 + i] = -s1;
            ub[46 + i] = cmd[i] - s2;
            lb[46 + i] = -QP_INFTY;
            lb[58 + i] = cmd[i] - s2;
            ub[58 + i] = QP_INFTY;
            if (dbg) { dbg->r1[i] = -s1; dbg->rsw[i] = cmd[i] - s2; }
        }
        for (int i = 0; i < 4 * NL; ++i) { lb[18 + i] = -QP_INFTY; ub[18 + i] = 0.0; }
        for (int i = 0; i < NJ; ++i) {
            lb[34 + i] = -pr->max_torque - bbar[6 + i];
            ub[34 + i] = pr->max_torque - bbar[6 + i];
        }
    }
    int it = 0, nact = 0, act[NV];
    int status = -1;
    if (st->method == 1) {
        /* the engine's 12-variable form; -1: not usable here, the literal form below */
        double Tinv_r[ND * ND], rsw[12];
        for (int i = 0; i < 12; ++i) rsw[i] = ub[46 + i];
        if (mat_inv(T, Tinv_r, ND) == 0)
            status = reduced_solve(pr, st, &kd, T, Tinv_r, Mbar_b, Mbar_j, bbar, W, lb + 6, rsw, kap, x, tau, &it);
        if (status < 0) st->ws12_valid = 0;
        else {
            *iters = it;
            st->contacts = contacts;
            st->first = 1;
            st->ws_n = 0;
            if (status != WBC_REF_OK) {
                memset(x, 0, sizeof(double) * NV);
                memset(tau, 0, sizeof(double) * NJ);
                memset(grf, 0, sizeof(double) * NJ);
            } else {
                for (int i = 0; i < NJ; ++i) grf[i] = x[18 + i];
            }
            goto debug_out;
        }
    }
    /* init on the first cycle, hotstart from the previous working set afterwards (cpp:523-531);
     * the working set only carries over under the same contact mask (the constraint rows differ
     * otherwise) */
    {
    const int warm = st->first && !st->cold_qp && st->ws_n > 0 && st->ws_kap == contacts;
    status = solve_qp(H, g, A, lb, ub, pr->max_wsr, warm ? st->ws : NULL, warm ? st->ws_n : 0, x, &it, act, &nact);
    }
    *iters = it;
    st->contacts = contacts;
    st->first = 1;
    st->ws_kap = contacts;
    st->ws_n = (status == WBC_REF_OK) ? nact : 0;
    for (int k = 0; k < st->ws_n; ++k) st->ws[k] = act[k];
    if (status != WBC_REF_OK) {
        memset(x, 0, sizeof(double) * NV);
        memset(tau, 0, sizeof(double) * NJ);
        memset(grf, 0, sizeof(double) * NJ);
    } else {
        /* computeJointTorques (cpp:553-577) */
        for (int i = 0; i < NJ; ++i) {
            double s = bbar[6 + i];
            for (int j = 0; j < NJ; ++j) s += Mbar_j[i * NJ + j] * x[6 + j];
            for (int j = 0; j < 3 * NL; ++j) s -= Jc[j * ND + 6 + i] * x[18 + j];
            tau[i] = s;
            grf[i] = x[18 + i];
        }
    }
debug_out:
    if (dbg) {
        memcpy(dbg->com, kd.com, sizeof kd.com);
        memcpy(dbg->comvel, kd.com_vel, sizeof kd.com_vel);
        memcpy(dbg->pose, cur_pose, sizeof cur_pose);
        memcpy(dbg->vc, vc, sizeof vc);
        memcpy(dbg->M, M, sizeof kd.M);
        memcpy(dbg->Cnu, kd.Cnu, sizeof kd.Cnu);
        memcpy(dbg->Mbar_b, Mbar_b, sizeof Mbar_b);
        memcpy(dbg->Mbar_j, Mbar_j, sizeof Mbar_j);
        memcpy(dbg->bbar, bbar, sizeof bbar);
        memcpy(dbg->W, W, sizeof W);
        if (mat_inv(T, Tinv, ND) == 0) mat_mul(kd.foot_J, Tinv, dbg->Jbar, 3 * NL, ND, ND);
    }
    return status;
}

void wbc_ref_run_batch(const wbc_model* md, const wbc_params* pr, int B, const double* pose, const double* nu,
                       const double* qj, const double* ref, const uint8_t* contacts, const uint8_t* switching, double* tau,
                       double* grf, double* x, int32_t* status, int32_t* iters) {
    wbc_ref_run_batch_method(md, pr, B, pose, nu, qj, ref, contacts, switching, tau, grf, x, status, iters, 0);
}

void wbc_ref_run_batch_method(const wbc_model* md, const wbc_params* pr, int B, const double* pose, const double* nu,
                              const double* qj, const double* ref, const uint8_t* contacts, const uint8_t* switching,
                              double* tau, double* grf, double* x, int32_t* status, int32_t* iters, int method) {
    for (int b = 0; b < B; ++b) {
        wbc_ref_state st;
        wbc_ref_state_init(&st);
        st.method = method;
        int it = 0;
        status[b] = wbc_ref_step(md, pr, &st, pose + 7 * b, nu + 18 * b, qj + 12 * b, ref + 54 * b, contacts[b],
                                 switching[b], tau + 12 * b, grf + 12 * b, x + NV * b, &it, NULL);
        iters[b] = it;
    }
}

/* n stateful robots stepped together (the per-robot `Robot` of oracle/wbc_ref.py, one call per
 * cycle): robot i reads row idx[i] of the batch input arrays and writes row i of the outputs.
 * The tests use it to follow a sample of a large batch through a whole trajectory. */
void wbc_ref_step_states(const wbc_model* md, const wbc_params* pr, int n, wbc_ref_state* st, const int32_t* idx,
                         const double* pose, const double* nu, const double* qj, const double* ref,
                         const uint8_t* contacts, const uint8_t* switching, double* tau, double* grf, double* x,
                         int32_t* status, int32_t* iters, int threads) {
#pragma omp parallel for schedule(dynamic, 4) num_threads(threads > 0 ? threads : 1)
    for (int i = 0; i < n; ++i) {
        const int b = idx[i];
        int it = 0;
        status[i] = wbc_ref_step(md, pr, st + i, pose + 7 * b, nu + 18 * b, qj + 12 * b, ref + 54 * b, contacts[b],
                                 switching[b], tau + 12 * i, grf + 12 * i, x + NV * i, &it, NULL);
        iters[i] = it;
    }
}
