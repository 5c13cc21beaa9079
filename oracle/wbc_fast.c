/* wbc_fast.c — CPU BASELINE ONLY (CPU baseline variant (ii) "structure-exploiting").
 *
 * bench.py's cpu_baseline leg times this next to oracle/wbc_ref.c (variant (i), the dense
 * reference-faithful restatement).  Tests use it only as a checked CPU restatement; the product
 * path never touches it.
 *
 * The same algorithm as the GPU engine, written for one robot per CPU thread, cold solves only
 * (the stateless configurations the baseline is timed on: derivative terms and the integral error
 * are zero, quirk A.7 "switching" cycle):
 *   - dynamics: the 13-body Kane form of wbc_ref.c, but each body's Jacobians touch only the 6
 *     base columns and its own leg's joints, so M and C nu accumulate over those 9 columns;
 *   - centroidal transform in closed form (no 18x18 inverse): A_j from M_bj, I_c from M_bb,
 *     Mbar_j = M_jj - A_lin'A_lin/m - A_ang'I_c^-1 A_ang, Jbar_f = [I, -S(d) | J_fj - A_lin/m +
 *     S(d) I_c^-1 A_ang], bbar_j = h_j - A_j' Mbar_b^-1 Ad' h_b (src/whole_body_controller.cpp:256-294);
 *   - the QP (cpp:466-535) reduced exactly: four-contact stance eliminates its 12 equalities
 *     (qdd = q0 - P f, Woodbury over the per-leg 3x3 blocks) and solves 12 force variables with
 *     40 inequality rows; other masks solve the 24-variable form y = [qdd; one 3-slot per leg]
 *     (a eliminated, swing forces 0, stance slacks |rsw|), both with the dense Goldfarb-Idnani of
 *     wbc_ref.c (wbc_ref_gi);
 *   - torques tau = Mbar_j qdd + bbar_j - Jbar_c,j' f (cpp:553-577).
 */
#include <math.h>
#include <string.h>

#include "wbc_ref.h"

#define ND 18
#define NJ 12
#define NL 4

static void cross3(const double* a, const double* b, double* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
static void skew3(const double* v, double* S) {
    S[0] = 0; S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2]; S[4] = 0; S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}
static void mv3(const double* M, const double* v, double* o) {
    for (int i = 0; i < 3; ++i) o[i] = M[3 * i] * v[0] + M[3 * i + 1] * v[1] + M[3 * i + 2] * v[2];
}
static void mm3(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}
static int inv3(const double* A, double* o, double* det_out) {
    const double c00 = A[4] * A[8] - A[5] * A[7], c01 = A[5] * A[6] - A[3] * A[8], c02 = A[3] * A[7] - A[4] * A[6];
    const double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
    if (det_out) *det_out = det;
    if (det == 0.0) return 1;
    const double id = 1.0 / det;
    o[0] = c00 * id; o[1] = (A[2] * A[7] - A[1] * A[8]) * id; o[2] = (A[1] * A[5] - A[2] * A[4]) * id;
    o[3] = c01 * id; o[4] = (A[0] * A[8] - A[2] * A[6]) * id; o[5] = (A[2] * A[3] - A[0] * A[5]) * id;
    o[6] = c02 * id; o[7] = (A[1] * A[6] - A[0] * A[7]) * id; o[8] = (A[0] * A[4] - A[1] * A[3]) * id;
    return 0;
}
static void quat_R(const double* q, double* R) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w); R[2] = 2 * (x * z + y * w);
    R[3] = 2 * (x * y + z * w); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
    R[6] = 2 * (x * z - y * w); R[7] = 2 * (y * z + x * w); R[8] = 1 - 2 * (x * x + y * y);
}
static void axis_rot(const double* a, double q, double* R) {
    const double c = cos(q), s = sin(q), v = 1 - c, x = a[0], y = a[1], z = a[2];
    R[0] = c + x * x * v;     R[1] = x * y * v - z * s; R[2] = x * z * v + y * s;
    R[3] = y * x * v + z * s; R[4] = c + y * y * v;     R[5] = y * z * v - x * s;
    R[6] = z * x * v - y * s; R[7] = z * y * v + x * s; R[8] = c + z * z * v;
}

/* Kane form over the lumped 13-body tree, accumulated on the 9 columns each body touches. */
typedef struct {
    double M[ND * ND], Cnu[ND], foot_J[12 * ND], foot_pos[12], foot_vel[12], com[3], com_vel[3], RB[9];
} kd_t;

static void body_accumulate(kd_t* out, const int* cols, int nc, double m, const double* I, const double (*Jv)[9],
                            const double (*Jw)[9], const double* w, const double* alpha, const double* acc) {
    double IJw[3][9];
    for (int t = 0; t < 3; ++t)
        for (int c = 0; c < nc; ++c) IJw[t][c] = I[3 * t] * Jw[0][c] + I[3 * t + 1] * Jw[1][c] + I[3 * t + 2] * Jw[2][c];
    for (int a = 0; a < nc; ++a)
        for (int b = a; b < nc; ++b) {
            double s = 0.0;
            for (int t = 0; t < 3; ++t) s += m * Jv[t][a] * Jv[t][b] + Jw[t][a] * IJw[t][b];
            out->M[cols[a] * ND + cols[b]] += s;
            if (b != a) out->M[cols[b] * ND + cols[a]] += s;
        }
    double Ia[3], Iw[3], wIw[3], N[3];
    mv3(I, alpha, Ia);
    mv3(I, w, Iw);
    cross3(w, Iw, wIw);
    for (int i = 0; i < 3; ++i) N[i] = Ia[i] + wIw[i];
    for (int c = 0; c < nc; ++c) {
        double s = 0.0;
        for (int t = 0; t < 3; ++t) s += Jv[t][c] * m * acc[t] + Jw[t][c] * N[t];
        out->Cnu[cols[c]] += s;
    }
}

static void kindyn(const wbc_model* md, const double* pose, const double* nu, const double* qj, kd_t* out) {
    memset(out, 0, sizeof(*out));
    const double* pB = pose;
    double RB[9];
    quat_R(pose + 3, RB);
    const double *wB = nu + 3, *qd = nu + 6;
    double msum = 0.0, mc[3] = {0, 0, 0}, mv[3] = {0, 0, 0};
    int cols[9];
    double Jv[3][9], Jw[3][9];
    for (int c = 0; c < 6; ++c) cols[c] = c;
    /* base body */
    {
        double c[3], r[3], S[9], t[3], tmp[9], RT[9], I[9], a[3];
        mv3(RB, md->base_com, c);
        for (int i = 0; i < 3; ++i) c[i] += pB[i], r[i] = c[i] - pB[i];
        mm3(RB, md->base_inertia, tmp);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) RT[3 * i + j] = RB[3 * j + i];
        mm3(tmp, RT, I);
        skew3(r, S);
        memset(Jv, 0, sizeof Jv);
        memset(Jw, 0, sizeof Jw);
        for (int i = 0; i < 3; ++i) {
            Jv[i][i] = 1.0;
            for (int j = 0; j < 3; ++j) Jv[i][3 + j] = -S[3 * i + j];
            Jw[i][3 + i] = 1.0;
        }
        cross3(wB, r, t);
        cross3(wB, t, a);
        body_accumulate(out, cols, 6, md->base_mass, I, Jv, Jw, wB, (const double[3]){0, 0, 0}, a);
        double v[3] = {nu[0], nu[1], nu[2]}, wr[3];
        cross3(wB, r, wr);
        for (int i = 0; i < 3; ++i) v[i] += wr[i];
        msum += md->base_mass;
        for (int i = 0; i < 3; ++i) mc[i] += md->base_mass * c[i], mv[i] += md->base_mass * v[i];
    }
    for (int l = 0; l < NL; ++l) {
        double Rp[9], op[3], wp[3], alp[3] = {0, 0, 0}, aop[3] = {0, 0, 0}, ax[3][3], org[3][3];
        memcpy(Rp, RB, sizeof Rp);
        memcpy(op, pB, sizeof op);
        memcpy(wp, wB, sizeof wp);
        for (int k = 0; k < 3; ++k) {
            const wbc_link* lk = &md->link[l][k];
            double Rj[9], oj[3], aj[3], Rl[9], Rc[9], rel[3], t[3], u[3], ao[3], wc[3], alc[3];
            mm3(Rp, lk->R, Rj);
            mv3(Rp, lk->p, oj);
            for (int i = 0; i < 3; ++i) oj[i] += op[i];
            mv3(Rj, lk->axis, aj);
            axis_rot(lk->axis, qj[3 * l + k], Rl);
            mm3(Rj, Rl, Rc);
            memcpy(ax[k], aj, sizeof aj);
            memcpy(org[k], oj, sizeof oj);
            for (int i = 0; i < 3; ++i) rel[i] = oj[i] - op[i];
            cross3(alp, rel, ao);
            cross3(wp, rel, t);
            cross3(wp, t, u);
            for (int i = 0; i < 3; ++i) ao[i] += aop[i] + u[i];
            cross3(wp, aj, t);
            for (int i = 0; i < 3; ++i) {
                wc[i] = wp[i] + aj[i] * qd[3 * l + k];
                alc[i] = alp[i] + t[i] * qd[3 * l + k];
            }
            double c[3], r[3], S[9], RcT[9], tmp[9], I[9];
            mv3(Rc, lk->com, c);
            for (int i = 0; i < 3; ++i) c[i] += oj[i], r[i] = c[i] - pB[i];
            mm3(Rc, lk->inertia, tmp);
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) RcT[3 * i + j] = Rc[3 * j + i];
            mm3(tmp, RcT, I);
            skew3(r, S);
            memset(Jv, 0, sizeof Jv);
            memset(Jw, 0, sizeof Jw);
            for (int i = 0; i < 3; ++i) {
                Jv[i][i] = 1.0;
                for (int j = 0; j < 3; ++j) Jv[i][3 + j] = -S[3 * i + j];
                Jw[i][3 + i] = 1.0;
            }
            for (int kk = 0; kk <= k; ++kk) {
                double d[3], v[3];
                for (int i = 0; i < 3; ++i) d[i] = c[i] - org[kk][i];
                cross3(ax[kk], d, v);
                cols[6 + kk] = 6 + 3 * l + kk;
                for (int i = 0; i < 3; ++i) {
                    Jv[i][6 + kk] = v[i];
                    Jw[i][6 + kk] = ax[kk][i];
                }
            }
            double d[3], ac[3];
            for (int i = 0; i < 3; ++i) d[i] = c[i] - oj[i];
            cross3(alc, d, ac);
            cross3(wc, d, t);
            cross3(wc, t, u);
            for (int i = 0; i < 3; ++i) ac[i] += ao[i] + u[i];
            body_accumulate(out, cols, 7 + k, lk->mass, I, Jv, Jw, wc, alc, ac);
            double v[3] = {0, 0, 0};
            for (int i = 0; i < 3; ++i) {
                for (int cc = 0; cc < 6; ++cc) v[i] += Jv[i][cc] * nu[cc];
                for (int kk = 0; kk <= k; ++kk) v[i] += Jv[i][6 + kk] * qd[3 * l + kk];
            }
            msum += lk->mass;
            for (int i = 0; i < 3; ++i) mc[i] += lk->mass * c[i], mv[i] += lk->mass * v[i];
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
        skew3(rfB, S);
        for (int i = 0; i < 3; ++i) {
            double* row = out->foot_J + (3 * l + i) * ND;
            row[i] = 1.0;
            for (int j = 0; j < 3; ++j) row[3 + j] = -S[3 * i + j];
        }
        for (int kk = 0; kk < 3; ++kk) {
            double d[3], v[3];
            for (int i = 0; i < 3; ++i) d[i] = pf[i] - org[kk][i];
            cross3(ax[kk], d, v);
            for (int i = 0; i < 3; ++i) out->foot_J[(3 * l + i) * ND + 6 + 3 * l + kk] = v[i];
        }
        for (int i = 0; i < 3; ++i) {  /* foot velocity: 6 base + 3 leg columns */
            const double* row = out->foot_J + (3 * l + i) * ND;
            double s = 0.0;
            for (int cc = 0; cc < 6; ++cc) s += row[cc] * nu[cc];
            for (int kk = 0; kk < 3; ++kk) s += row[6 + 3 * l + kk] * qd[3 * l + kk];
            out->foot_vel[3 * l + i] = s;
        }
    }
    for (int i = 0; i < 3; ++i) out->com[i] = mc[i] / msum, out->com_vel[i] = mv[i] / msum;
    memcpy(out->RB, RB, sizeof RB);
}

/* One cold step (stateless: switching cycle, fresh history).  Returns the QP status. */
int wbc_fast_step(const wbc_model* md, const wbc_params* pr, const double* pose, const double* nu, const double* qj,
                  const double* ref, int contacts, double* tau, double* grf, int* iters_out) {
    kd_t kd;
    kindyn(md, pose, nu, qj, &kd);
    const double m = md->total_mass, im = 1.0 / m, g0 = pr->gravity;
    int kap[NL], ns = 0;
    for (int l = 0; l < NL; ++l) kap[l] = (contacts >> l) & 1, ns += kap[l];
    const double* M = kd.M;
    double r[3], Sr[9];
    for (int i = 0; i < 3; ++i) r[i] = kd.com[i] - pose[i];
    skew3(r, Sr);
    /* A_j (about the CoM) from M_bj = [A_lin; S(r) A_lin + A_ang]; I_c = I_B + m S(r) S(r) */
    double Al[3][NJ], Aa[3][NJ], Ic[9], Icinv[9], KA[3][NJ];
    for (int j = 0; j < NJ; ++j) {
        for (int i = 0; i < 3; ++i) Al[i][j] = M[i * ND + 6 + j];
        for (int i = 0; i < 3; ++i) Aa[i][j] = M[(3 + i) * ND + 6 + j] - (Sr[3 * i] * Al[0][j] + Sr[3 * i + 1] * Al[1][j] + Sr[3 * i + 2] * Al[2][j]);
    }
    {
        double SS[9];
        mm3(Sr, Sr, SS);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Ic[3 * i + j] = M[(3 + i) * ND + 3 + j] + m * SS[3 * i + j];
        if (inv3(Ic, Icinv, NULL)) return WBC_REF_NUMERIC;
    }
    for (int j = 0; j < NJ; ++j)
        for (int i = 0; i < 3; ++i) KA[i][j] = Icinv[3 * i] * Aa[0][j] + Icinv[3 * i + 1] * Aa[1][j] + Icinv[3 * i + 2] * Aa[2][j];
    double Mbj[NJ * NJ], Jbj[NJ * NJ], d[NL][3], bbj[NJ];
    for (int i = 0; i < NJ; ++i)
        for (int j = 0; j < NJ; ++j) {
            double s = M[(6 + i) * ND + 6 + j];
            for (int t = 0; t < 3; ++t) s -= Al[t][i] * Al[t][j] * im + Aa[t][i] * KA[t][j];
            Mbj[i * NJ + j] = s;
        }
    for (int l = 0; l < NL; ++l) {
        for (int i = 0; i < 3; ++i) d[l][i] = kd.foot_pos[3 * l + i] - kd.com[i];
        for (int j = 0; j < NJ; ++j) {
            double ka[3] = {KA[0][j], KA[1][j], KA[2][j]}, dk[3];
            cross3(d[l], ka, dk);  /* S(d) I_c^-1 A_ang column j */
            for (int i = 0; i < 3; ++i) Jbj[(3 * l + i) * NJ + j] = kd.foot_J[(3 * l + i) * ND + 6 + j] - Al[i][j] * im + dk[i];
        }
    }
    { /* bbar_j = h_j - A_j' Mbar_b^-1 [h_lin; h_ang - r x h_lin]  (h = C nu: cold, Tdot_inv = 0) */
        const double* h = kd.Cnu;
        double ha[3], rh[3], u[6];
        cross3(r, h, rh);
        for (int i = 0; i < 3; ++i) ha[i] = h[3 + i] - rh[i];
        for (int i = 0; i < 3; ++i) u[i] = h[i] * im;
        mv3(Icinv, ha, u + 3);
        for (int j = 0; j < NJ; ++j) {
            double s = h[6 + j];
            for (int t = 0; t < 3; ++t) s -= Al[t][j] * u[t] + Aa[t][j] * u[3 + t];
            bbj[j] = s;
        }
    }
    /* desired wrench (cpp:426-445), cold: integral error 0 */
    double W[6];
    {
        const double* R = kd.RB;
        const double cur[6] = {kd.com[0], kd.com[1], kd.com[2], atan2(R[7], R[8]), atan2(-R[6], sqrt(R[7] * R[7] + R[8] * R[8])),
                               atan2(R[3], R[0])};
        const double vc[6] = {kd.com_vel[0], kd.com_vel[1], kd.com_vel[2], nu[3], nu[4], nu[5]};
        double Ia[3];
        mv3(Ic, ref + 15, Ia);
        for (int k = 0; k < 6; ++k) {
            const double kp = (k == 2) ? pr->kp_z : pr->kp;
            const double mba = (k < 3) ? m * ref[12 + k] : Ia[k - 3];
            W[k] = -kp * (cur[k] - ref[k]) - pr->kd * (vc[k] - ref[6 + k]) + (k == 2 ? m * g0 : 0.0) + mba;
        }
    }
    /* G = E Mbar_b^-1 E' (E rows [e_k, -S(d_l) row k]); slot Hessian H_s = I + E (I + Mbar_b^-2) E';
     * slot gradient g_s = -E (W + [0, 0, g/m, 0, 0, 0]); R1 right-hand side (cold) e = g e_z */
    double E[NJ][6];
    for (int l = 0; l < NL; ++l)
        for (int k = 0; k < 3; ++k) {
            double* e = E[3 * l + k];
            double ek[3] = {k == 0, k == 1, k == 2}, c[3];
            cross3(d[l], ek, c);  /* (-S(d) row k)' = d x e_k */
            e[0] = ek[0]; e[1] = ek[1]; e[2] = ek[2];
            e[3] = c[0]; e[4] = c[1]; e[5] = c[2];
        }
    double Mi6[36] = {0};
    for (int i = 0; i < 3; ++i) Mi6[i * 6 + i] = im;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Mi6[(3 + i) * 6 + 3 + j] = Icinv[3 * i + j];
    double G[NJ * NJ], Hs[NJ * NJ], gs[NJ];
    {
        double Mi2[36] = {0}, EMi[NJ][6], EH[NJ][6];
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double s = (i == j) ? 1.0 : 0.0;
                for (int t = 0; t < 6; ++t) s += Mi6[i * 6 + t] * Mi6[t * 6 + j];
                Mi2[i * 6 + j] = s;
            }
        for (int i = 0; i < NJ; ++i)
            for (int j = 0; j < 6; ++j) {
                double s1 = 0.0, s2 = 0.0;
                for (int t = 0; t < 6; ++t) s1 += E[i][t] * Mi6[t * 6 + j], s2 += E[i][t] * Mi2[t * 6 + j];
                EMi[i][j] = s1;
                EH[i][j] = s2;
            }
        for (int i = 0; i < NJ; ++i)
            for (int j = 0; j < NJ; ++j) {
                double s1 = 0.0, s2 = (i == j) ? 1.0 : 0.0;
                for (int t = 0; t < 6; ++t) s1 += EMi[i][t] * E[j][t], s2 += EH[i][t] * E[j][t];
                G[i * NJ + j] = s1;
                Hs[i * NJ + j] = s2;
            }
        double wg[6];
        for (int t = 0; t < 6; ++t) wg[t] = W[t] + (t == 2 ? g0 * im : 0.0);
        for (int i = 0; i < NJ; ++i) {
            double s = 0.0;
            for (int t = 0; t < 6; ++t) s += E[i][t] * wg[t];
            gs[i] = -s;
        }
    }
    const double mu = pr->friction, tmax = pr->max_torque;
    double qdd[NJ], f[NJ];
    int st, it = 0;
    if (ns == NL) {
        /* Four-contact stance: qdd = q0 - P f, P = Jbj^-1 G = W S^-1 Mbar_b^-1 E', W = Jblk^-1 E,
         * S = I6 - K W, q0 = w + Y K w (w = Jblk^-1 e, Y = W S^-1), K = Mbar_b^-1 A_j. */
        double Wm[NJ][6], w[NJ], K[6][NJ];
        for (int j = 0; j < NJ; ++j)
            for (int t = 0; t < 3; ++t) K[t][j] = Al[t][j] * im, K[3 + t][j] = KA[t][j];
        for (int l = 0; l < NL; ++l) {
            double Jl[9], Jli[9], det;
            for (int i = 0; i < 3; ++i)
                for (int k = 0; k < 3; ++k) Jl[3 * i + k] = kd.foot_J[(3 * l + i) * ND + 6 + 3 * l + k];
            double amx = 0.0;
            for (int t = 0; t < 9; ++t) amx = fmax(amx, fabs(Jl[t]));
            if (inv3(Jl, Jli, &det) || !(fabs(det) > 1e-9 * amx * amx * amx)) goto general; /* near-singular leg */
            for (int k = 0; k < 3; ++k) {
                const int i = 3 * l + k;
                w[i] = Jli[3 * k + 2] * g0;  /* e = (0, 0, g) per leg (cold: r1 = 0) */
                for (int t = 0; t < 6; ++t) Wm[i][t] = Jli[3 * k] * E[3 * l][t] + Jli[3 * k + 1] * E[3 * l + 1][t] + Jli[3 * k + 2] * E[3 * l + 2][t];
            }
        }
        double S[6][13], z[6];
        for (int a = 0; a < 6; ++a) {
            double zz = 0.0;
            for (int b = 0; b < 6; ++b) {
                double s = 0.0;
                for (int j = 0; j < NJ; ++j) s += K[a][j] * Wm[j][b];
                S[a][b] = (a == b) - s;
                S[a][6 + b] = (a == b);
            }
            for (int j = 0; j < NJ; ++j) zz += K[a][j] * w[j];
            z[a] = zz;
        }
        for (int k = 0; k < 6; ++k) { /* Gauss-Jordan with partial pivoting: S^-1 in columns 6..11 */
            int p = k;
            for (int a = k + 1; a < 6; ++a)
                if (fabs(S[a][k]) > fabs(S[p][k])) p = a;
            if (!(fabs(S[p][k]) > 1e-12)) goto general;
            if (p != k)
                for (int c = 0; c < 12; ++c) { double t = S[k][c]; S[k][c] = S[p][c]; S[p][c] = t; }
            const double ip = 1.0 / S[k][k];
            for (int c = 0; c < 12; ++c) S[k][c] *= ip;
            for (int a = 0; a < 6; ++a)
                if (a != k) {
                    const double fa = S[a][k];
                    for (int c = 0; c < 12; ++c) S[a][c] -= fa * S[k][c];
                }
        }
        double Y[NJ][6], q0[NJ];
        for (int i = 0; i < NJ; ++i) {
            double q = w[i];
            for (int c = 0; c < 6; ++c) {
                double s = 0.0;
                for (int t = 0; t < 6; ++t) s += Wm[i][t] * S[t][6 + c];
                Y[i][c] = s;
                q += s * z[c];
            }
            q0[i] = q;
        }
        /* P = Y Mbar_b^-1 E' ; H_f = H_s + P'P ; g_f = g_s - P'q0 ; Nt = Mbj P + Jbj' ; t0 = bbj + Mbj q0 */
        double YM[NJ][6], P[NJ * NJ], Hf[NJ * NJ], gf[NJ], Nt[NJ * NJ], t0[NJ];
        for (int i = 0; i < NJ; ++i)
            for (int c = 0; c < 6; ++c) {
                double s = 0.0;
                for (int t = 0; t < 6; ++t) s += Y[i][t] * Mi6[t * 6 + c];
                YM[i][c] = s;
            }
        for (int i = 0; i < NJ; ++i)
            for (int j = 0; j < NJ; ++j) {
                double s = 0.0;
                for (int t = 0; t < 6; ++t) s += YM[i][t] * E[j][t];
                P[i * NJ + j] = s;
            }
        for (int i = 0; i < NJ; ++i) {
            double s = gs[i];
            for (int k = 0; k < NJ; ++k) s -= P[k * NJ + i] * q0[k];
            gf[i] = s;
            for (int j = i; j < NJ; ++j) {
                double h = Hs[i * NJ + j];
                for (int k = 0; k < NJ; ++k) h += P[k * NJ + i] * P[k * NJ + j];
                Hf[i * NJ + j] = Hf[j * NJ + i] = h;
            }
        }
        for (int j = 0; j < NJ; ++j) {
            double tt = bbj[j];
            for (int k = 0; k < NJ; ++k) tt += Mbj[j * NJ + k] * q0[k];
            t0[j] = tt;
            for (int c = 0; c < NJ; ++c) {
                double s = Jbj[c * NJ + j];
                for (int k = 0; k < NJ; ++k) s += Mbj[j * NJ + k] * P[k * NJ + c];
                Nt[j * NJ + c] = s;
            }
        }
        /* rows: friction faces -D_rr f_l >= 0, torque rows +-(t0 - Nt f) >= -tau_max */
        double CI[40 * NJ], ci[40];
        memset(CI, 0, sizeof CI);
        const double D[4][3] = {{-1, 0, mu}, {1, 0, mu}, {0, -1, mu}, {0, 1, mu}};
        for (int l = 0; l < NL; ++l)
            for (int rr = 0; rr < 4; ++rr) {
                for (int c = 0; c < 3; ++c) CI[(4 * l + rr) * NJ + 3 * l + c] = D[rr][c];
                ci[4 * l + rr] = 0.0;
            }
        for (int j = 0; j < NJ; ++j)
            for (int sgi = 0; sgi < 2; ++sgi) {
                const double sg = sgi ? -1.0 : 1.0;
                const int row = 16 + 2 * j + sgi;
                for (int c = 0; c < NJ; ++c) CI[row * NJ + c] = -sg * Nt[j * NJ + c];
                ci[row] = -tmax - sg * t0[j];
            }
        st = wbc_ref_gi(NJ, Hf, gf, 0, NULL, NULL, 40, CI, ci, pr->max_wsr, f, &it);
        if (st == WBC_REF_OK) {
            for (int j = 0; j < NJ; ++j) {
                double s = t0[j], q = q0[j];
                for (int c = 0; c < NJ; ++c) s -= Nt[j * NJ + c] * f[c], q -= P[j * NJ + c] * f[c];
                tau[j] = s;
                qdd[j] = q;
                grf[j] = f[j];
            }
        }
        *iters_out = it;
        if (st != WBC_REF_OK) {
            memset(tau, 0, sizeof(double) * NJ);
            memset(grf, 0, sizeof(double) * NJ);
        }
        return st;
    }
general:;
    /* 24-variable form y = [qdd; slot l = f_l (stance) or s_l (swing)]: H = blkdiag(I, H_s | w I),
     * R1 stance equalities Jbj_i qdd + G_i f = e_i, friction faces, torque rows, swing rows. */
    {
        enum { N = 24 };
        double H[N * N], g[N], CE[12 * N], ce[12], CI[52 * N], ci[52], y[N];
        memset(H, 0, sizeof H);
        memset(g, 0, sizeof g);
        for (int i = 0; i < NJ; ++i) H[i * N + i] = 1.0;
        for (int i = 0; i < NJ; ++i) {
            const int li = i / 3;
            for (int j = 0; j < NJ; ++j) {
                const int lj = j / 3;
                double v = 0.0;
                if (kap[li] && kap[lj]) v = Hs[i * NJ + j];
                else if (!kap[li] && i == j) v = pr->slack_weight;
                H[(12 + i) * N + 12 + j] = v;
            }
            if (kap[li]) g[12 + i] = gs[i];
        }
        int me = 0, mi = 0;
        /* cold swing commands and R4/R5 bounds: rsw = cmd (Js_dot = 0) */
        double rsw[NJ];
        for (int i = 0; i < NJ; ++i)
            rsw[i] = kap[i / 3] ? 0.0
                                : ref[42 + i] + pr->kd_swing * (ref[30 + i] - kd.foot_vel[i]) + pr->kp_swing * (ref[18 + i] - kd.foot_pos[i]);
        for (int i = 0; i < NJ; ++i) {
            if (!kap[i / 3]) continue;
            double* row = CE + me * N;
            memset(row, 0, sizeof(double) * N);
            for (int j = 0; j < NJ; ++j) row[j] = Jbj[i * NJ + j];
            for (int j = 0; j < NJ; ++j)
                if (kap[j / 3]) row[12 + j] = G[i * NJ + j];
            ce[me++] = ((i % 3) == 2) ? g0 : 0.0;
        }
        const double D[4][3] = {{-1, 0, mu}, {1, 0, mu}, {0, -1, mu}, {0, 1, mu}};
        for (int l = 0; l < NL; ++l) {
            if (!kap[l]) continue;
            for (int rr = 0; rr < 4; ++rr) {
                double* row = CI + mi * N;
                memset(row, 0, sizeof(double) * N);
                for (int c = 0; c < 3; ++c) row[12 + 3 * l + c] = D[rr][c];
                ci[mi++] = 0.0;
            }
        }
        for (int j = 0; j < NJ; ++j)
            for (int sgi = 0; sgi < 2; ++sgi) {
                const double sg = sgi ? -1.0 : 1.0;
                double* row = CI + mi * N;
                memset(row, 0, sizeof(double) * N);
                for (int k = 0; k < NJ; ++k) row[k] = sg * Mbj[j * NJ + k];
                for (int c = 0; c < NJ; ++c)
                    if (kap[c / 3]) row[12 + c] = -sg * Jbj[c * NJ + j];
                ci[mi++] = sgi ? -tmax + bbj[j] : -tmax - bbj[j];
            }
        for (int i = 0; i < NJ; ++i) { /* swing rows +-(Js_j qdd + Js_com a) + s >= +-(rsw + g e_z) */
            const int l = i / 3;
            if (kap[l]) continue;
            double wrow[N];
            memset(wrow, 0, sizeof wrow);
            for (int j = 0; j < NJ; ++j) wrow[j] = Jbj[i * NJ + j];
            for (int j = 0; j < NJ; ++j)
                if (kap[j / 3]) wrow[12 + j] = G[i * NJ + j];
            const double cp = rsw[i] + (((i % 3) == 2) ? g0 : 0.0);
            for (int sgi = 0; sgi < 2; ++sgi) {
                const double sg = sgi ? 1.0 : -1.0;
                double* row = CI + mi * N;
                for (int k = 0; k < N; ++k) row[k] = sg * wrow[k];
                row[12 + i] += 1.0;
                ci[mi++] = sg * cp;
            }
        }
        st = wbc_ref_gi(N, H, g, me, CE, ce, mi, CI, ci, pr->max_wsr, y, &it);
        *iters_out = it;
        if (st != WBC_REF_OK) {
            memset(tau, 0, sizeof(double) * NJ);
            memset(grf, 0, sizeof(double) * NJ);
            return st;
        }
        for (int i = 0; i < NJ; ++i) {
            qdd[i] = y[i];
            f[i] = kap[i / 3] ? y[12 + i] : 0.0;
        }
        for (int j = 0; j < NJ; ++j) {
            double s = bbj[j];
            for (int k = 0; k < NJ; ++k) s += Mbj[j * NJ + k] * qdd[k] - Jbj[k * NJ + j] * f[k];
            tau[j] = s;
            grf[j] = f[j];
        }
        return st;
    }
}

/* B cold robots on `threads` OpenMP threads (static schedule, one robot per iteration). */
void wbc_fast_run_batch(const wbc_model* md, const wbc_params* pr, int B, const double* pose, const double* nu,
                        const double* qj, const double* ref, const uint8_t* contacts, double* tau, double* grf,
                        int32_t* status, int32_t* iters, int threads) {
#pragma omp parallel for schedule(static) num_threads(threads)
    for (int b = 0; b < B; ++b) {
        int it = 0;
        status[b] = wbc_fast_step(md, pr, pose + 7 * b, nu + 18 * b, qj + 12 * b, ref + 54 * b, contacts[b], tau + 12 * b,
                                  grf + 12 * b, &it);
        iters[b] = it;
    }
}

/* The dense reference-faithful restatement (wbc_ref.c) on the same OpenMP schedule. */
void wbc_ref_run_batch_omp(const wbc_model* md, const wbc_params* pr, int B, const double* pose, const double* nu,
                           const double* qj, const double* ref, const uint8_t* contacts, const uint8_t* switching,
                           double* tau, double* grf, int32_t* status, int32_t* iters, int threads) {
#pragma omp parallel for schedule(static) num_threads(threads)
    for (int b = 0; b < B; ++b) {
        wbc_ref_state st;
        wbc_ref_state_init(&st);
        double x[42];
        int it = 0;
        status[b] = wbc_ref_step(md, pr, &st, pose + 7 * b, nu + 18 * b, qj + 12 * b, ref + 54 * b, contacts[b], switching[b],
                                 tau + 12 * b, grf + 12 * b, x, &it, NULL);
        iters[b] = it;
    }
}
