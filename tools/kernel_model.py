"""Design model of the HIP kernel's algorithm, in numpy (development tool, not the oracle).

The HIP kernel (quadrupedwholebodycontroller_amd/csrc/wbc_kernel.hip) does not translate the
reference's dense Eigen code.  It uses closed forms of the same quantities and a reduced QP.
This file is that algorithm written sequentially, so the derivation can be checked against
the reference restatement (oracle/wbc_np.py) on the CPU (tests/test_kernel_model.py).

Closed forms (r = c - p_B, Ad = [[I, S(r)], [0, I]], A_j = centroidal momentum matrix, joint
columns, about the CoM):
  Mbar_b = Ad' M_bb Ad              = diag(m I3, I_c)                         (cpp:270-271)
  T^-1   = [[Ad, -K], [0, I]],  K = M_bb^-1 M_bj = Ad Mbar_b^-1 A_j         (cpp:296-320)
  Mbar_j = M_jj - A_lin'A_lin/m - A_ang' I_c^-1 A_ang                        (cpp:272)
  Jbar_f = [I, -S(p_f - c) | J_f,j - A_lin/m + S(p_f - c) I_c^-1 A_ang]      (cpp:278-284)
  T_top  = [Ad^-1, Mbar_b^-1 A_j]                                            (cpp:317)
  bbar_j = h_j - A_j' Mbar_b^-1 Ad' h_b,  h = C nu + M Tdot_inv nu           (cpp:289)

Reduced QP.  With H > 0 the optimum of the reference QP (42 vars, 70 rows) is unique.  Three
eliminations keep it exact:
  * a = Mbar_b^-1 (Jc' f - gw) from the 6 dynamics equalities (R0);
  * forces of legs with contact flag 0 appear in no constraint: f = 0;
  * slacks of legs with contact flag 1 have zero rows in R4/R5: s = |rhs|.
What is left is a strictly convex QP in n = 24 variables y = [qdd (12), one 3-slot per leg:
f_l if the leg is in stance, s_l if it swings], with 3*ns equalities and at most 48+ns
inequality rows.  It is solved with the Goldfarb-Idnani dual active-set method: Householder
reflection on add, Givens on drop, and the products C = J' N of every constraint normal kept
up to date (one constraint per lane on the GPU).
"""
from __future__ import annotations

import numpy as np

import os, sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import wbc_np as W  # noqa: E402

NL, NJ = 4, 12


def skew(v):
    return W.skew(v)


class Hist:
    """Compact per-robot history (what the stateful kernel keeps in HBM)."""

    def __init__(self):
        self.T_top = np.hstack([np.eye(6), np.zeros((6, 12))])  # old T top rows (T_old = I)
        self.Jbar = np.zeros((12, 18))  # old unmasked Jbar_feet
        self.kappa = np.ones(4, int)     # contacts of the old Jbar (irrelevant while Jbar = 0)
        self.Tdinv_top = np.zeros((6, 18))
        self.e_int = np.zeros(6)


def structured_update(model, params, base_pose, nu, qj, ref, kappa, switching, hist: Hist):
    kd = W.KinDyn(model, base_pose, nu, qj)
    p = params
    m = kd.total_mass
    pB = kd.pB
    c = kd.com
    r = c - pB
    bodies = kd.bodies
    Ic = np.zeros((3, 3))
    for b in bodies:
        d = b["c"] - c
        Ic += b["I"] + b["m"] * (d @ d * np.eye(3) - np.outer(d, d))
    Ic_inv = np.linalg.inv(Ic)
    # centroidal momentum matrix, joint columns (about c)
    A_lin = np.zeros((3, 12)); A_ang = np.zeros((3, 12))
    M_jj = np.zeros((12, 12))
    for bi, b in enumerate(bodies[1:]):
        Jv, Jw = b["Jv"][:, 6:], b["Jw"][:, 6:]
        A_lin += b["m"] * Jv
        A_ang += b["m"] * skew(b["c"] - c) @ Jv + b["I"] @ Jw
        M_jj += b["m"] * Jv.T @ Jv + Jw.T @ b["I"] @ Jw
    Mbar_j = M_jj - A_lin.T @ A_lin / m - A_ang.T @ Ic_inv @ A_ang
    Mbinv = np.zeros((6, 6)); Mbinv[:3, :3] = np.eye(3) / m; Mbinv[3:, 3:] = Ic_inv
    Mbar_b = np.zeros((6, 6)); Mbar_b[:3, :3] = m * np.eye(3); Mbar_b[3:, 3:] = Ic
    A_j = np.vstack([A_lin, A_ang])
    # centroidal foot Jacobians (unmasked)
    Jbar = np.zeros((12, 18))
    for l in range(4):
        d = kd.foot_pos[l] - c
        Jbar[3 * l:3 * l + 3, :3] = np.eye(3)
        Jbar[3 * l:3 * l + 3, 3:6] = -skew(d)
        Jbar[3 * l:3 * l + 3, 6:] = kd.foot_J[3 * l:3 * l + 3, 6:] - A_lin / m + skew(d) @ Ic_inv @ A_ang
    Ad = np.eye(6); Ad[:3, 3:] = skew(r)
    Adinv = np.eye(6); Adinv[:3, 3:] = -skew(r)
    T_top = np.hstack([Adinv, Mbinv @ A_j])
    # bias: h = C nu + M[:, :6] y, y = Tdinv_top nu (previous cycle)
    h = kd.Cnu.copy()
    y = hist.Tdinv_top @ nu
    M_bj = np.vstack([A_lin, skew(r) @ A_lin + A_ang])
    I_B = Ic - m * skew(r) @ skew(r)
    M_bb = np.block([[m * np.eye(3), -m * skew(r)], [m * skew(r), I_B]])
    h[:6] += M_bb @ y
    h[6:] += M_bj.T @ y
    hb_c = np.concatenate([h[:3], h[3:6] - np.cross(r, h[:3])])
    bbar_j = h[6:] - A_j.T @ (Mbinv @ hb_c)
    # finite differences (cpp:384-402), compact history
    dt = 1.0 / p["loop_rate"]
    kmask = np.repeat(kappa, 3)[:, None].astype(float)
    kmask_old = np.repeat(hist.kappa, 3)[:, None].astype(float)
    Jc = Jbar * kmask; Js = Jbar * (1 - kmask)
    if switching:
        Tdot_top = np.zeros((6, 18)); Jc_dot = np.zeros((12, 18)); Js_dot = np.zeros((12, 18))
    else:
        Tdot_top = (T_top - hist.T_top) / dt
        Jc_dot = (Jc - hist.Jbar * kmask_old) / dt
        Js_dot = (Js - hist.Jbar * (1 - kmask_old)) / dt
    K = Ad @ Mbinv @ A_j
    Tdinv_new = -Ad @ np.hstack([Tdot_top[:, :6] @ Ad, -Tdot_top[:, :6] @ K + Tdot_top[:, 6:]])
    # task quantities
    vc = np.concatenate([kd.com_vel, nu[3:6]])
    pose = np.concatenate([c, W.eul_angles_rpy(kd.RB)])
    qd = nu[6:]
    r1 = -Jc_dot[:, :6] @ vc - Jc_dot[:, 6:] @ qd
    cmd = (ref[42:54] + p["kd_swing"] * (ref[30:42] - kd.foot_vel.ravel())
           + p["kp_swing"] * (ref[18:30] - kd.foot_pos.ravel())) * (1 - kmask[:, 0])
    rsw = cmd - Js_dot[:, :6] @ vc - Js_dot[:, 6:] @ qd
    Kp = p["kp"] * np.ones(6); Kp[2] = p["kp_z"]
    gw = np.array([0, 0, m * p["gravity"], 0, 0, 0])
    Wr = -Kp * (pose - ref[0:6]) - p["kd"] * (vc - ref[6:12]) - p["ki"] * hist.e_int + gw + Mbar_b @ ref[12:18]
    new_hist = Hist()
    new_hist.T_top = T_top; new_hist.Jbar = Jbar; new_hist.kappa = np.array(kappa)
    new_hist.Tdinv_top = Tdinv_new; new_hist.e_int = hist.e_int + (pose - ref[0:6]) / p["loop_rate"]
    prob = dict(m=m, Ic=Ic, Ic_inv=Ic_inv, Mbinv=Mbinv, Mbar_b=Mbar_b, Mbar_j=Mbar_j, Jbar=Jbar, Jc=Jc, Js=Js,
                bbar_j=bbar_j, r1=r1, rsw=rsw, W=Wr, kappa=np.array(kappa), vc=vc, pose=pose, kd=kd)
    return prob, new_hist


def reduced_qp(prob, params):
    """Build the n = 24 reduced problem: H (24x24), g, equalities (E, e), inequalities (G >= h)."""
    p = params
    kap = prob["kappa"]
    m, g0 = prob["m"], p["gravity"]
    Jc_com = prob["Jc"][:, :6]; Jc_j = prob["Jc"][:, 6:]
    Js_com = prob["Js"][:, :6]; Js_j = prob["Js"][:, 6:]
    Mbinv = prob["Mbinv"]
    n = 24
    H = np.zeros((n, n)); g = np.zeros(n)
    H[:12, :12] = np.eye(12)
    G6 = np.eye(6) + Mbinv @ Mbinv
    Hff = np.eye(12) + Jc_com @ G6 @ Jc_com.T  # zero coupling for swing rows
    gf = -Jc_com @ (prob["W"] + np.array([0, 0, g0 / m, 0, 0, 0]))
    for l in range(4):
        sl = slice(12 + 3 * l, 15 + 3 * l)
        if kap[l]:
            for mm in range(4):
                if kap[mm]:
                    H[sl, 12 + 3 * mm:15 + 3 * mm] = Hff[3 * l:3 * l + 3, 3 * mm:3 * mm + 3]
            g[sl] = gf[3 * l:3 * l + 3]
        else:
            H[sl, sl] = p["slack_weight"] * np.eye(3)
    # P = Mbinv Jc' (6x12): a = P f + a0
    Pm = Mbinv @ Jc_com.T
    E, e, Gi, hi = [], [], [], []
    infeasible = False
    mu = p["friction"]
    D = np.array([[1, 0, -mu], [-1, 0, -mu], [0, 1, -mu], [0, -1, -mu]], float)
    for l in range(4):
        for k in range(3):
            i = 3 * l + k
            if kap[l]:
                row = np.zeros(n)
                row[:12] = Jc_j[i]
                cf = Jc_com[i] @ Pm  # over all 12 force components
                for mm in range(4):
                    if kap[mm]:
                        row[12 + 3 * mm:15 + 3 * mm] = cf[3 * mm:3 * mm + 3]
                E.append(row); e.append(prob["r1"][i] + (g0 if k == 2 else 0.0))
            else:
                if abs(prob["r1"][i]) > 1e-9 * max(1.0, abs(prob["r1"][i])) and prob["r1"][i] != 0.0:
                    infeasible = True
    for l in range(4):
        if kap[l]:
            for rr in range(4):
                row = np.zeros(n); row[12 + 3 * l:15 + 3 * l] = -D[rr]
                Gi.append(row); hi.append(0.0)
    tmax = p["max_torque"]
    for i in range(12):
        row = np.zeros(n)
        row[:12] = prob["Mbar_j"][i]
        for mm in range(4):
            if kap[mm]:
                row[12 + 3 * mm:15 + 3 * mm] = -Jc_j[3 * mm:3 * mm + 3, i]
        Gi.append(row.copy()); hi.append(-tmax - prob["bbar_j"][i])
        Gi.append(-row); hi.append(-(tmax - prob["bbar_j"][i]))
    for l in range(4):
        if kap[l]:
            continue
        for k in range(3):
            i = 3 * l + k
            w = np.zeros(n)
            w[:12] = Js_j[i]
            cf = Js_com[i] @ Pm
            for mm in range(4):
                if kap[mm]:
                    w[12 + 3 * mm:15 + 3 * mm] = cf[3 * mm:3 * mm + 3]
            cprime = prob["rsw"][i] + (g0 if k == 2 else 0.0)
            s = np.zeros(n); s[12 + i] = 1.0
            Gi.append(-w + s); hi.append(-cprime)
            Gi.append(w + s); hi.append(cprime)
    mk = lambda L: np.array(L).reshape(-1, n)
    return H, g, mk(E), np.array(e), mk(Gi), np.array(hi), infeasible


def expand(prob, params, y):
    """Reduced solution y -> reference x (42) and torques."""
    kap = prob["kappa"]
    x = np.zeros(42)
    f = np.zeros(12)
    for l in range(4):
        if kap[l]:
            f[3 * l:3 * l + 3] = y[12 + 3 * l:15 + 3 * l]
            x[30 + 3 * l:33 + 3 * l] = np.abs(prob["rsw"][3 * l:3 * l + 3])
        else:
            x[30 + 3 * l:33 + 3 * l] = y[12 + 3 * l:15 + 3 * l]
    gw = np.array([0, 0, prob["m"] * params["gravity"], 0, 0, 0])
    x[:6] = prob["Mbinv"] @ (prob["Jc"][:, :6].T @ f - gw)
    x[6:18] = y[:12]
    x[18:30] = f
    tau = prob["Mbar_j"] @ y[:12] + prob["bbar_j"] - prob["Jc"][:, 6:].T @ f
    return x, tau


def gi_kernel_style(H, g, E, e, G, h, max_iter=100):
    """Goldfarb-Idnani exactly as the kernel organises it: C = J'N kept for all rows,
    constraint slacks updated incrementally, Householder add, Givens drop."""
    n = g.size
    N = np.vstack([E, G]).T  # n x m  (columns = normals)
    b = np.concatenate([e, h])
    me, m = E.shape[0], N.shape[1]
    L = np.linalg.cholesky(H)
    J = np.linalg.inv(L).T
    x = -J @ (J.T @ g)
    C = J.T @ N
    s = N.T @ x - b
    R = np.zeros((n, n)); q = 0
    act = []; u = []
    eps = 1e-14

    def rsolve(d1):
        return np.linalg.solve(R[:q, :q], d1) if q else np.zeros(0)

    def add(d):
        nonlocal q
        v = d[q:].copy(); nrm = np.linalg.norm(v)
        if nrm <= 1e-13 * max(1.0, np.linalg.norm(d)):
            return False
        alpha = -nrm if v[0] >= 0 else nrm
        v[0] -= alpha
        beta = 1.0 / (nrm * (nrm + abs(d[q])))  # 2/(v'v)
        J[:, q:] -= beta * np.outer(J[:, q:] @ v, v)
        C[q:, :] -= beta * np.outer(v, v @ C[q:, :])
        R[:q, q] = d[:q]; R[q, q] = alpha
        q += 1
        return True

    def drop(k):
        nonlocal q
        R[:, k:q - 1] = R[:, k + 1:q]; R[:, q - 1] = 0.0
        for j in range(k, q - 1):
            a_, b_ = R[j, j], R[j + 1, j]
            rr = np.hypot(a_, b_); cg, sg = (a_ / rr, b_ / rr) if rr > 0 else (1.0, 0.0)
            t1, t2 = R[j, j:q - 1].copy(), R[j + 1, j:q - 1].copy()
            R[j, j:q - 1] = cg * t1 + sg * t2; R[j + 1, j:q - 1] = -sg * t1 + cg * t2
            c1, c2 = J[:, j].copy(), J[:, j + 1].copy()
            J[:, j] = cg * c1 + sg * c2; J[:, j + 1] = -sg * c1 + cg * c2
            r1_, r2_ = C[j].copy(), C[j + 1].copy()
            C[j] = cg * r1_ + sg * r2_; C[j + 1] = -sg * r1_ + cg * r2_
        q -= 1
        del act[k]; del u[k]

    for i in range(me):
        d = C[:, i].copy()
        r = rsolve(d[:q])
        zn = d[q:] @ d[q:]
        if zn <= 1e-26 * max(1.0, N[:, i] @ N[:, i]):
            if abs(s[i]) <= 1e-9 * max(1.0, abs(b[i])):
                continue
            return x, W.QP_INFEASIBLE, 0
        t = -s[i] / zn
        z = J[:, q:] @ d[q:]
        x += t * z
        s += t * (C[q:, :].T @ d[q:])
        u = [uk - t * rk for uk, rk in zip(u, r)] + [t]
        act.append(i)
        if not add(d):
            return x, W.QP_NUMERIC, 0
    neq = q
    nrm = np.linalg.norm(N, axis=0)
    iters = 0
    while True:
        inact = np.ones(m, bool); inact[act] = False; inact[:me] = False
        viol = np.where(inact, s / nrm, np.inf)
        tol = 1e-10 * np.maximum(1.0, np.abs(b)) / nrm
        p = int(np.argmin(np.where(viol < -tol, viol, np.inf)))
        if not (viol[p] < -tol[p]):
            return x, W.QP_OK, iters
        up = 0.0
        while True:
            iters += 1
            if iters > max_iter:
                return x, W.QP_MAX_ITER, iters - 1
            d = C[:, p].copy()
            r = rsolve(d[:q])
            t1, l = np.inf, -1
            for k in range(neq, q):
                if r[k] > eps and u[k] / r[k] < t1:
                    t1, l = u[k] / r[k], k
            zn = d[q:] @ d[q:]
            t2 = -s[p] / zn if zn > 1e-26 else np.inf
            t = min(t1, t2)
            if not np.isfinite(t):
                return x, W.QP_INFEASIBLE, iters
            if np.isfinite(t2):
                z = J[:, q:] @ d[q:]
                x += t * z
                s += t * (C[q:, :].T @ d[q:])
            u = [uk - t * rk for uk, rk in zip(u, r)]
            up += t
            if np.isfinite(t2) and t == t2:
                u.append(up); act.append(p)
                if not add(d):
                    return x, W.QP_NUMERIC, iters
                break
            drop(l)


def kernel_step(model, params, base_pose, nu, qj, ref, kappa, switching, hist=None):
    hist = hist or Hist()
    prob, nh = structured_update(model, params, base_pose, nu, qj, ref, kappa, switching, hist)
    H, g, E, e, G, h, infeasible = reduced_qp(prob, params)
    if infeasible:
        return None, None, W.QP_INFEASIBLE, 0, prob, nh
    y, st, it = gi_kernel_style(H, g, E, e, G, h, params["max_wsr"])
    x, tau = expand(prob, params, y)
    return x, tau, st, it, prob, nh
