"""Exact reduction of the reference QP to 12 variables for every contact mask (test infrastructure).

This is the engine's QP method restated densely in numpy, so that tests can check
on CPU that the reduction is exact: its optimum, mapped back to the reference's 42 variables,
equals the optimum of the literal 42 x 70 QP of src/whole_body_controller.cpp:466-515 (which
`wbc_np.ReferenceWBC.assemble_qp` restates), and its status (OK / INFEASIBLE) is the reference
QP's.  Only `tests/` import it.

The reference QP (variables x = [a (6); qdd (12); f (12); s (12)], H positive definite) has a
unique optimum, so exact eliminations do not change it:

  * a = Mb^-1 (E_S^T f - w_g) (R0, the six centroidal dynamics equalities; E = J̄c,com rows
    [I, -S(d_l)]; only stance legs carry force);
  * the swing slacks: R4 / R5 read s_i >= +-(Js_i [a; qdd] - rsw_i), and s_i enters the objective
    only as 1/2 w s_i^2 (w = slack_weight), so s_i = |r_i| with r_i = Js_i [a; qdd] - rsw_i and the
    pair of rows becomes the penalty 1/2 w r_i^2; for stance legs the rows are vacuous
    (s_i = |rsw_i|);
  * the stance equalities R1 (3 per stance leg): J̄_S qdd + G_S f = e_S solved for the stance
    legs' joint accelerations.  With J̄_S qdd = J_S qdd_S - E_S K qdd (J_S the legs' own 3x3 foot
    Jacobian blocks, K = Mb^-1 A_j) and Woodbury (W = J_S^-1 E_S, S6 = I - K_S W, Y = W S6^-1):
    qdd_S = q0 + Y phi, phi = K_W qdd_W - Mb^-1 E_S^T f, q0 = w + Y K_S w, w = J_S^-1 e_S.

What is left is z = one 3-slot per leg: the swing legs' joint accelerations and the stance legs'
forces (12 variables for every mask), with only inequality rows: the stance legs' friction faces
and the 24 torque rows, tau = t0 - Nt z.  Its Hessian is
H = I + P^T (I + Mb^-2) P + sum_i w_i Rho_i^T Rho_i, where P z = E_S^T f and the 12 "leg rows" Rho
are the stance joints' accelerations (w_i = 1) and the swing feet's task residuals
(w_i = slack_weight).
"""
from __future__ import annotations

import numpy as np

import wbc_np as W

NL, NJ, NV = 4, 12, 42


def reduced_problem(c: "W.ReferenceWBC"):
    """The 12-variable problem of a controller after update_state() and assemble_qp().

    Returns a dict (H, g, CI, ci, nsel, plus the maps back to the 42 variables), or None when the
    elimination is not usable (a near-singular stance leg or S6)."""
    p = c.params
    m = c.model.total_mass
    kap = np.asarray(c.foot_contacts, int)
    Tinv = np.linalg.inv(c.T)
    Jbar = c.kd.foot_J @ Tinv  # unmasked
    E, Jbj = Jbar[:, :6], Jbar[:, 6:]
    Jblk = np.zeros((12, 12))
    for l in range(NL):
        Jblk[3 * l:3 * l + 3, 3 * l:3 * l + 3] = c.kd.foot_J[3 * l:3 * l + 3, 6 + 3 * l:9 + 3 * l]
    K = np.linalg.lstsq(E, Jblk - Jbj, rcond=None)[0]  # E K = Jblk - Jbj, E has full column rank
    Mb = c.Mbar_b
    Mbi = np.linalg.inv(Mb)
    g0 = p["gravity"]
    st = np.repeat(kap, 3).astype(bool)  # per row / joint / slot
    # stance equalities: e = r1 + g e_z
    e = c.r1 + np.tile([0.0, 0.0, g0], NL)
    Wr, w = np.zeros((12, 6)), np.zeros(12)
    for l in range(NL):
        if kap[l]:
            Jl = c.kd.foot_J[3 * l:3 * l + 3, 6 + 3 * l:9 + 3 * l]
            if abs(np.linalg.det(Jl)) <= 1e-9 * np.abs(Jl).max() ** 3:
                return None
            Ji = np.linalg.inv(Jl)
            Wr[3 * l:3 * l + 3] = Ji @ E[3 * l:3 * l + 3]
            w[3 * l:3 * l + 3] = Ji @ e[3 * l:3 * l + 3]
    S6 = np.eye(6) - K @ Wr  # rows of W for swing legs are zero
    z6 = K @ w
    S6i = np.linalg.inv(S6)
    Y = Wr @ S6i
    q0 = w + Y @ z6
    # phi = B z
    B = np.zeros((6, 12))
    P = np.zeros((6, 12))
    for j in range(12):
        if st[j]:
            B[:, j] = -Mbi @ E[j]
            P[:, j] = E[j]
        else:
            B[:, j] = K[:, j]
    # leg rows: stance -> qdd_S = q0 + Y B z ; swing -> r = c_i + J_l[k] z_l - (E_i S6^-1) B z
    cpsi = np.array([0.0, 0.0, -g0, 0.0, 0.0, 0.0]) - K[:, st] @ q0[st]
    Rho, rho0, wt = np.zeros((12, 12)), np.zeros(12), np.zeros(12)
    for i in range(12):
        l, k = divmod(i, 3)
        if st[i]:
            Rho[i] = Y[i] @ B
            rho0[i] = q0[i]
            wt[i] = 1.0
        else:
            own = np.zeros(12)
            own[3 * l:3 * l + 3] = Jblk[i, 3 * l:3 * l + 3]
            vt = -S6i.T @ E[i]
            Rho[i] = own + vt @ B
            rho0[i] = E[i] @ cpsi - c.rsw[i]
            wt[i] = p["slack_weight"]
    CP = np.eye(6) + Mbi @ Mbi
    H = np.eye(12) + P.T @ CP @ P + Rho.T @ (wt[:, None] * Rho)
    gw_m = np.array([0.0, 0.0, g0 / m, 0.0, 0.0, 0.0])
    g = -P.T @ (c.W + gw_m) + Rho.T @ (wt * rho0)
    # torque rows: tau = bbar_j + Mbar_j qdd - Jbj^T f ; qdd = [z_W ; q0 + Y B z]
    Mj = c.Mbar_j
    t0 = c.bbar[6:] + Mj[:, st] @ q0[st]
    MY = Mj[:, st] @ Y[st]
    Nt = np.zeros((12, 12))
    for j in range(12):
        Nt[:, j] = -MY @ B[:, j] + (Jbj[j, :] if st[j] else -Mj[:, j])
    # inequality rows in the unified numbering: friction face 4 l + rr (stance legs only), then the
    # torque rows 16 + 2 j (+ upper side, t0 - Nt z >= -tau_max) and 16 + 2 j + 1 (lower side)
    mu, tm = p["friction"], p["max_torque"]
    D = np.array([[1.0, 0, -mu], [-1.0, 0, -mu], [0, 1.0, -mu], [0, -1.0, -mu]])
    CI, ci, nsel, ids = [], [], [], []
    for l in range(NL):
        if kap[l]:
            for rr in range(4):
                n = np.zeros(12)
                n[3 * l:3 * l + 3] = -D[rr]
                CI.append(n); ci.append(0.0); nsel.append(1.0 + mu * mu); ids.append(4 * l + rr)
    for j in range(12):
        s2 = Mj[j] @ Mj[j] + sum(Jbj[r, j] ** 2 for r in range(12) if st[r])
        for sg in (1.0, -1.0):
            CI.append(-sg * Nt[j]); ci.append(-tm - sg * t0[j]); nsel.append(s2)
            ids.append(16 + 2 * j + (0 if sg > 0 else 1))
    # vacuous rows: the swing legs' R1 rows read 0 = r1 (quirk A.12)
    vac_ok = all(abs(c.r1[i]) <= 1e-9 * max(1.0, abs(c.r1[i])) for i in range(12) if not st[i])
    return dict(H=H, g=g, CI=np.array(CI), ci=np.array(ci), nsel=np.array(nsel), ids=ids, st=st, B=B, Y=Y, q0=q0,
                P=P, Mbi=Mbi, Rho=Rho, rho0=rho0, wt=wt, Nt=Nt, t0=t0, vac_ok=vac_ok, S6=S6)


def to_x42(c, rp, z):
    """The reference's 42 variables and the torques from the reduced optimum z."""
    st = rp["st"]
    phi = rp["B"] @ z
    qdd = np.where(st, rp["q0"] + rp["Y"] @ phi, z)
    f = np.where(st, z, 0.0)
    a = rp["Mbi"] @ (rp["P"] @ z) - np.array([0.0, 0.0, c.params["gravity"], 0.0, 0.0, 0.0])
    r = rp["rho0"] + rp["Rho"] @ z
    s = np.where(st, np.abs(c.rsw), np.abs(r))
    tau = rp["t0"] - rp["Nt"] @ z
    return np.concatenate([a, qdd, f, s]), tau


def reduced_step(c: "W.ReferenceWBC"):
    """One cycle of a controller through the reduction.  Returns (tau, x42, status, iters) or None
    when the elimination is not usable (the engine then takes the general path)."""
    c.update_state()
    c.assemble_qp()
    rp = reduced_problem(c)
    if rp is None:
        return None
    if not rp["vac_ok"]:
        return np.zeros(NJ), np.zeros(NV), W.QP_INFEASIBLE, 0
    z, stt, it, _ = W.gi_solve(rp["H"], rp["g"], np.zeros((0, 12)), np.zeros(0), rp["CI"], rp["ci"],
                               c.params["max_wsr"])
    if stt != W.QP_OK:
        return np.zeros(NJ), np.zeros(NV), stt, it
    x, tau = to_x42(c, rp, z)
    return tau, x, stt, it
