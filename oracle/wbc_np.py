"""wbc_np — numpy fp64 restatement of the reference WBC hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker.  The product path (quadrupedwholebodycontroller_amd) never does.

What it restates (all citations into the reference, /root/reference):
  * iDynTree KinDynComputations in MIXED representation (the default; the reference never
    changes it): setRobotState (src/whole_body_controller.cpp:258), CoM position/velocity
    (:260-261), getFreeFloatingMassMatrix (:266), generalizedBiasForces -
    generalizedGravityForces (:544-551), getFrameFreeFloatingJacobian (:327-341),
    getWorldTransform (:349-359), getFrameVel (:369-379).  The library is an un-vendored
    submodule (.gitmodules:4-6, no pinned commit); its published algorithms are restated
    from first principles (Kane's equations with generalized speeds nu = [p_B_dot; omega_W; qdot]).
  * WholeBodyController::updateState / solveQP / computeJointTorques (:256-577) literally:
    dense 18x18 inverses, dense products, finite differences, QP assembly in the reference's
    row/column order, including the quirks listed in SURVEY.md Appendix A.
  * qpOASES::SQProblem init/hotstart (:517-535; un-vendored, .gitmodules:1-3).  H is positive
    definite, so the QP optimum is unique; any exact method returns it.  This module uses the
    Goldfarb-Idnani dual active-set method (dense, 42 variables) and certifies the result
    with KKT residuals (`kkt_residuals`).

Parity status: the reference cannot be built or run here (ROS/Eigen/iDynTree/qpOASES absent,
SURVEY.md 8c) and its repository holds no tests or golden vectors, so this oracle is
"parity unpinned" against the reference binary.  It is pinned instead by physics identities
(tests/test_oracle_physics.py) and by a second, independent C restatement (oracle/wbc_ref.c).
"""
from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
MODEL_JSON = os.path.join(os.path.dirname(HERE), "quadrupedwholebodycontroller_amd", "model", "anymal.json")

NJ, NL, ND = 12, 4, 18
NV = 6 + NJ + 3 * NL + 3 * NL  # hpp:31
NC = 6 + 3 * NL + 4 * NL + NJ + 6 * NL  # hpp:32
INFTY = 1.0e20  # qpOASES::INFTY (used at cpp:508,512,514)

QP_OK, QP_MAX_ITER, QP_INFEASIBLE, QP_NUMERIC = 0, 1, 2, 3
TIE_BAND = 1e-9  # include/wbc.h WBC_TIE_BAND: near-ties in the row selection are ties (lowest id)


# --------------------------------------------------------------------------------------
# model / params
# --------------------------------------------------------------------------------------
class Model:
    def __init__(self, path=MODEL_JSON):
        with open(path) as f:
            d = json.load(f)
        self.base_mass = d["base"]["mass"]
        self.base_com = np.array(d["base"]["com"])
        self.base_I = np.array(d["base"]["inertia"])
        self.R = np.array([[lk["R"] for lk in leg] for leg in d["legs"]])  # 4x3x3x3
        self.p = np.array([[lk["p"] for lk in leg] for leg in d["legs"]])
        self.axis = np.array([[lk["axis"] for lk in leg] for leg in d["legs"]])
        self.mass = np.array([[lk["mass"] for lk in leg] for leg in d["legs"]])
        self.com = np.array([[lk["com"] for lk in leg] for leg in d["legs"]])
        self.I = np.array([[lk["inertia"] for lk in leg] for leg in d["legs"]])
        self.foot = np.array(d["foot"])
        self.total_mass = d["total_mass"]  # model_.getTotalMass(), cpp:72
        self.joint_names = d["joint_names"]


def default_params():
    """config/params_controller.yaml:1-12 (+ gravityAcceleration hpp:30, nWSR cpp:517)."""
    return dict(friction=1.0, loop_rate=400.0, max_torque=80.0, kp=6000.0, kp_z=10000.0, kd=1800.0,
                ki=0.0, kp_swing=250.0, kd_swing=20.0, slack_weight=1000.0,
                initial_reference_pose=np.array([0.0, 0.0, 0.50, 0.0, 0.0, 0.0]), gravity=9.81,
                max_wsr=100)


# --------------------------------------------------------------------------------------
# small helpers (cpp:3-20)
# --------------------------------------------------------------------------------------
def skew(v):
    """skewOperator, cpp:3-10."""
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def eul_angles_rpy(R):
    """eulAnglesRPY, cpp:12-20 (no angle wrapping)."""
    roll = np.arctan2(R[2, 1], R[2, 2])
    pitch = np.arctan2(-R[2, 0], np.sqrt(R[2, 1] * R[2, 1] + R[2, 2] * R[2, 2]))
    yaw = np.arctan2(R[1, 0], R[0, 0])
    return np.array([roll, pitch, yaw])


def quat_to_R(qx, qy, qz, qw):
    """Eigen::Quaterniond(w,x,y,z).toRotationMatrix() as used at cpp:209-213 (no normalisation)."""
    tx, ty, tz = 2 * qx, 2 * qy, 2 * qz
    twx, twy, twz = tx * qw, ty * qw, tz * qw
    txx, txy, txz = tx * qx, ty * qx, tz * qx
    tyy, tyz, tzz = ty * qy, tz * qy, tz * qz
    return np.array([[1 - (tyy + tzz), txy - twz, txz + twy],
                     [txy + twz, 1 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1 - (txx + tyy)]])


def axis_angle(a, q):
    a = a / np.linalg.norm(a)
    K = skew(a)
    return np.eye(3) + np.sin(q) * K + (1 - np.cos(q)) * (K @ K)


# --------------------------------------------------------------------------------------
# iDynTree KinDynComputations restatement (MIXED representation)
# --------------------------------------------------------------------------------------
class KinDyn:
    """State after kinDynComp_.setRobotState(T_wb, q, baseVel, qdot, g) (cpp:258).

    Generalized speeds nu = [p_B_dot (world); omega (world); qdot] (MIXED).  For every rigid
    body b: com velocity v_b = Jv_b nu, angular velocity w_b = Jw_b nu; M = sum Jv'm Jv + Jw'I Jw
    (kinetic energy 1/2 nu'M nu).  Bias (Kane): h = sum Jv' m a_b + Jw'(I alpha_b + w x I w) with
    the accelerations evaluated at nu_dot = 0.  Gravity cancels in the reference's use
    (cpp:544-551), so `Cnu` is that h.
    """

    def __init__(self, model: Model, base_pose, nu, qj):
        base_pose = np.asarray(base_pose, float)
        nu = np.asarray(nu, float)
        qj = np.asarray(qj, float)
        pB = base_pose[:3]
        RB = quat_to_R(*base_pose[3:7])
        self.pB, self.RB, self.nu, self.qj = pB, RB, nu, qj
        vB, wB, qd = nu[:3], nu[3:6], nu[6:]
        bodies = []  # dicts: m, c, I (world), Jv, Jw, v, w, a (com accel), alpha
        # floating base (cpp: T_world_base_)
        cb = pB + RB @ model.base_com
        Jv = np.zeros((3, ND)); Jw = np.zeros((3, ND))
        Jv[:, 0:3] = np.eye(3); Jv[:, 3:6] = -skew(cb - pB); Jw[:, 3:6] = np.eye(3)
        bodies.append(dict(m=model.base_mass, c=cb, I=RB @ model.base_I @ RB.T, Jv=Jv, Jw=Jw,
                           w=wB.copy(), alpha=np.zeros(3),
                           a=np.cross(wB, np.cross(wB, cb - pB))))
        self.foot_pos = np.zeros((NL, 3))
        self.foot_J = np.zeros((3 * NL, ND))
        for l in range(NL):
            Rpar, opar = RB, pB
            wpar, alpar, aopar = wB.copy(), np.zeros(3), np.zeros(3)
            chain = []  # (col, axis world, origin world)
            for k in range(3):
                col = 6 + 3 * l + k
                Rj = Rpar @ model.R[l, k]
                oj = opar + Rpar @ model.p[l, k]
                aj = Rj @ model.axis[l, k]
                Rc = Rj @ axis_angle(model.axis[l, k], qj[3 * l + k])
                chain.append((col, aj, oj))
                # velocity / bias-acceleration recursion (joint origin is a point of the parent)
                ao = aopar + np.cross(alpar, oj - opar) + np.cross(wpar, np.cross(wpar, oj - opar))
                wc = wpar + aj * qd[3 * l + k]
                alc = alpar + np.cross(wpar, aj) * qd[3 * l + k]
                c = oj + Rc @ model.com[l, k]
                Jv = np.zeros((3, ND)); Jw = np.zeros((3, ND))
                Jv[:, 0:3] = np.eye(3); Jv[:, 3:6] = -skew(c - pB); Jw[:, 3:6] = np.eye(3)
                for (cc, a, o) in chain:
                    Jv[:, cc] = np.cross(a, c - o)
                    Jw[:, cc] = a
                ac = ao + np.cross(alc, c - oj) + np.cross(wc, np.cross(wc, c - oj))
                bodies.append(dict(m=model.mass[l, k], c=c, I=Rc @ model.I[l, k] @ Rc.T, Jv=Jv, Jw=Jw,
                                   w=wc, alpha=alc, a=ac))
                Rpar, opar, wpar, alpar, aopar = Rc, oj, wc, alc, ao
            pf = opar + Rpar @ model.foot[l]
            self.foot_pos[l] = pf
            J = np.zeros((3, ND))
            J[:, 0:3] = np.eye(3); J[:, 3:6] = -skew(pf - pB)
            for (cc, a, o) in chain:
                J[:, cc] = np.cross(a, pf - o)
            self.foot_J[3 * l:3 * l + 3] = J
        self.bodies = bodies
        M = np.zeros((ND, ND)); h = np.zeros(ND)
        msum, mc, mv = 0.0, np.zeros(3), np.zeros(3)
        for b in bodies:
            M += b["m"] * b["Jv"].T @ b["Jv"] + b["Jw"].T @ b["I"] @ b["Jw"]
            h += b["Jv"].T @ (b["m"] * b["a"]) + b["Jw"].T @ (b["I"] @ b["alpha"] + np.cross(b["w"], b["I"] @ b["w"]))
            msum += b["m"]; mc += b["m"] * b["c"]; mv += b["m"] * (b["Jv"] @ nu)
        self.M = 0.5 * (M + M.T)
        self.Cnu = h
        self.total_mass = msum
        self.com = mc / msum
        self.com_vel = mv / msum
        self.foot_vel = (self.foot_J @ nu).reshape(NL, 3)

    def kinetic_energy(self):
        return 0.5 * self.nu @ self.M @ self.nu


# --------------------------------------------------------------------------------------
# Goldfarb-Idnani dual active-set QP (stands in for qpOASES::SQProblem; unique optimum)
# --------------------------------------------------------------------------------------
def _givens(a, b):
    if b == 0.0:
        return 1.0, 0.0
    r = np.hypot(a, b)
    return a / r, b / r


def gi_solve(H, g, CE, ce, CI, ci, max_iter=100):
    """min 1/2 x'Hx + g'x  s.t. CE x = ce, CI x >= ci.  H symmetric positive definite.

    Returns (x, status, iters, active) with `iters` = inequality working-set changes (the
    quantity qpOASES bounds by nWSR, cpp:517)."""
    n = g.size
    me, mi = CE.shape[0], CI.shape[0]
    try:
        L = np.linalg.cholesky(H)
    except np.linalg.LinAlgError:
        return np.zeros(n), QP_NUMERIC, 0, []
    J = np.linalg.inv(L).T
    x = -np.linalg.solve(H, g)
    R = np.zeros((n, n))
    q = 0
    active = []  # constraint ids: ('e', i) or ('i', i)
    u = np.zeros(0)
    ni = np.linalg.norm(CI, axis=1) if mi else np.zeros(0)
    eps = 1e-14

    def add(d):
        nonlocal q, J, R
        # Householder on d[q:] -> (delta, 0, ..., 0); J <- J P
        v = d[q:].copy()
        nrm = np.linalg.norm(v)
        if nrm <= eps * max(1.0, np.linalg.norm(d)):
            return False
        alpha = -nrm if v[0] >= 0 else nrm
        v[0] -= alpha
        vv = v @ v
        if vv > 0:
            J[:, q:] -= np.outer(J[:, q:] @ v, v) * (2.0 / vv)
        R[:q, q] = d[:q]
        R[q, q] = alpha
        q += 1
        return True

    def drop(k):
        nonlocal q, J, R, u
        # remove column k of R; re-triangularise with Givens rotations on rows; mirror on J
        R[:, k:q - 1] = R[:, k + 1:q]
        R[:, q - 1] = 0.0
        for j in range(k, q - 1):
            c, s = _givens(R[j, j], R[j + 1, j])
            rj, rj1 = R[j, j:q - 1].copy(), R[j + 1, j:q - 1].copy()
            R[j, j:q - 1] = c * rj + s * rj1
            R[j + 1, j:q - 1] = -s * rj + c * rj1
            Jj, Jj1 = J[:, j].copy(), J[:, j + 1].copy()
            J[:, j] = c * Jj + s * Jj1
            J[:, j + 1] = -s * Jj + c * Jj1
        q -= 1
        del active[k]
        u = np.delete(u, k)

    # equality constraints first (always full steps)
    for i in range(me):
        npv = CE[i]
        d = J.T @ npv
        z = J[:, q:] @ d[q:]
        r = np.linalg.solve(R[:q, :q], d[:q]) if q else np.zeros(0)
        s = npv @ x - ce[i]
        zn = z @ npv
        if abs(zn) <= eps * max(1.0, npv @ npv):
            if abs(s) <= 1e-9 * max(1.0, abs(ce[i])):
                continue  # redundant, consistent
            return x, QP_INFEASIBLE, 0, active
        t = -s / zn
        x = x + t * z
        u = np.append(u - t * r, t)
        if not add(d):
            return x, QP_NUMERIC, 0, active
        active.append(("e", i))
    n_eq = q
    iters = 0
    while True:
        inact = np.ones(mi, bool)
        for (kind, i) in active:
            if kind == "i":
                inact[i] = False
        s_all = CI @ x - ci
        viol = np.where(inact, s_all / np.maximum(ni, 1e-300), np.inf)
        tol = 1e-10 * np.maximum(1.0, np.abs(ci)) / np.maximum(ni, 1e-300)
        cand = np.where(viol < -tol)[0]
        if cand.size == 0:
            return x, QP_OK, iters, active
        # near-ties are ties: the lowest id within TIE_BAND of the most violated (include/wbc.h
        # WBC_TIE_BAND, the engine's and the C oracle's rule)
        vm = viol[cand].min()
        p = cand[viol[cand] <= vm * (1.0 - TIE_BAND)][0]
        npv = CI[p]
        sp = s_all[p]
        up = 0.0
        while True:
            iters += 1
            if iters > max_iter:
                return x, QP_MAX_ITER, iters - 1, active
            d = J.T @ npv
            z = J[:, q:] @ d[q:]
            r = np.linalg.solve(R[:q, :q], d[:q]) if q else np.zeros(0)
            # partial step: largest dual step keeping active inequality multipliers >= 0
            t1, l = np.inf, -1
            for k in range(n_eq, q):
                if r[k] > eps:
                    tk = u[k] / r[k]
                    if tk < t1:
                        t1, l = tk, k
            zn = z @ npv
            t2 = -sp / zn if (z @ z) > eps * eps and zn > eps else np.inf
            t = min(t1, t2)
            if not np.isfinite(t):
                return x, QP_INFEASIBLE, iters, active
            if not np.isfinite(t2):
                u = u - t * r
                up += t
                drop(l)
                continue
            x = x + t * z
            u = u - t * r
            up += t
            sp += t * zn
            if t == t2:
                u = np.append(u, up)
                if not add(d):
                    return x, QP_NUMERIC, iters, active
                active.append(("i", p))
                break
            drop(l)


def split_constraints(A, lbA, ubA):
    """qpOASES general constraints lbA <= A x <= ubA -> (CE, ce, CI, ci, rowmap).

    Identically-zero rows (mode-masked stance/friction rows, quirk A.12) are dropped when their
    bounds admit 0 and flagged infeasible otherwise; two-sided rows are split."""
    CE, ce, CI, ci = [], [], [], []
    feasible = True
    for i in range(A.shape[0]):
        row = A[i]
        lo, hi = lbA[i], ubA[i]
        lo_inf, hi_inf = lo <= -INFTY, hi >= INFTY
        if not np.any(row != 0.0):
            if (not lo_inf and lo > 1e-9 * max(1, abs(lo))) or (not hi_inf and hi < -1e-9 * max(1, abs(hi))):
                feasible = False
            continue
        if not lo_inf and not hi_inf and lo == hi:
            CE.append(row); ce.append(lo)
            continue
        if not lo_inf:
            CI.append(row); ci.append(lo)
        if not hi_inf:
            CI.append(-row); ci.append(-hi)
    n = A.shape[1]
    mk = lambda rows: np.array(rows).reshape(-1, n)
    return mk(CE), np.array(ce), mk(CI), np.array(ci), feasible


def solve_qp(H, g, A, lbA, ubA, max_iter=100):
    CE, ce, CI, ci, feasible = split_constraints(A, lbA, ubA)
    if not feasible:
        return np.zeros(g.size), QP_INFEASIBLE, 0
    x, st, it, _ = gi_solve(H, g, CE, ce, CI, ci, max_iter)
    return x, st, it


def kkt_residuals(H, g, A, lbA, ubA, x):
    """Return (primal violation, stationarity residual, complementarity) with the multipliers
    recovered on the set of (numerically) active rows by least squares."""
    Ax = A @ x
    lo = np.where(lbA <= -INFTY, -np.inf, lbA)
    hi = np.where(ubA >= INFTY, np.inf, ubA)
    viol = np.maximum(np.maximum(lo - Ax, Ax - hi), 0.0)
    scale = 1.0 + np.abs(Ax)
    act = (np.abs(Ax - lo) <= 1e-7 * scale) | (np.abs(Ax - hi) <= 1e-7 * scale)
    grad = H @ x + g
    Aa = A[act]
    if Aa.shape[0]:
        lam, *_ = np.linalg.lstsq(Aa.T, -grad, rcond=None)
        stat = grad + Aa.T @ lam
    else:
        lam = np.zeros(0)
        stat = grad
    return float(viol.max(initial=0.0)), float(np.abs(stat).max()), act, lam


# --------------------------------------------------------------------------------------
# WholeBodyController restatement
# --------------------------------------------------------------------------------------
class ReferenceWBC:
    """Per-robot restatement of `class WholeBodyController` (hpp:35-171) hot-path methods."""

    def __init__(self, model: Model | None = None, params: dict | None = None):
        self.model = model or Model()
        self.params = dict(default_params(), **(params or {}))
        self.set_initial_state()
        self.qp_solution = np.zeros(NV)  # cpp:58

    # cpp:65-120
    def set_initial_state(self):
        p = self.params
        self.foot_contacts = np.ones(NL, dtype=int)
        self.total_mass = self.model.total_mass
        self.base_pose = np.array([0, 0, 0.60, 0, 0, 0, 1.0])
        self.joint_pos = np.array([0.0, -0.4, 0.8, 0.0, 0.4, -0.8, 0.0, 0.4, -0.8, 0.0, -0.4, 0.8])
        self.base_vel = np.zeros(6)
        self.joint_vel = np.zeros(NJ)
        self.old_T = np.eye(ND)
        self.old_Jc = np.zeros((3 * NL, ND))
        self.old_Js = np.zeros((3 * NL, ND))
        self.Tdot = np.zeros((ND, ND))
        self.Jc_dot = np.zeros((3 * NL, ND))
        self.Js_dot = np.zeros((3 * NL, ND))
        self.Tdot_inv = np.zeros((ND, ND))  # quirk A.1: read before first write; defined 0
        self.desired_pose = np.array(p["initial_reference_pose"], float)
        self.desired_com_vel = np.zeros(6)
        self.desired_com_acc = np.zeros(6)
        self.desired_sw_acc = np.zeros(3 * NL)
        self.desired_sw_vel = np.zeros(3 * NL)
        self.desired_sw_pos = np.zeros(3 * NL)
        self.integral_error = np.zeros(6)
        self.is_switching = False
        self.first_iteration = True

    # floatingBaseStateCallback / jointStateCallback (cpp:187-254), model joint order
    def set_state(self, base_pose, nu, qj):
        self.base_pose = np.asarray(base_pose, float).copy()
        self.base_vel = np.asarray(nu[:6], float).copy()
        self.joint_vel = np.asarray(nu[6:], float).copy()
        self.joint_pos = np.asarray(qj, float).copy()

    # referenceCallback (cpp:150-185)
    def reference_callback(self, ref, contacts):
        self.set_reference(ref, contacts, None)

    def set_reference(self, ref, contacts, switching=None):
        ref = np.asarray(ref, float)
        self.desired_pose = ref[0:6].copy()
        self.desired_com_vel = ref[6:12].copy()
        self.desired_com_acc = ref[12:18].copy()
        self.desired_sw_pos = ref[18:30].copy()
        self.desired_sw_vel = ref[30:42].copy()
        self.desired_sw_acc = ref[42:54].copy()
        contacts = np.asarray(contacts, int)
        if switching is None:
            switching = bool(np.any(contacts != self.foot_contacts))
        self.is_switching = bool(switching)
        self.foot_contacts = contacts.copy()

    # cpp:256-294
    def update_state(self):
        kd = KinDyn(self.model, self.base_pose, np.concatenate([self.base_vel, self.joint_vel]), self.joint_pos)
        self.kd = kd
        self.com = kd.com
        self.com_vel6 = np.concatenate([kd.com_vel, self.base_vel[3:6]])  # quirk A.4
        R = kd.RB
        self.current_pose = np.concatenate([self.com, eul_angles_rpy(R)])
        M = kd.M
        self.M = M
        self.M_bb = M[:6, :6].copy()
        T = self.compute_transformation_matrix()
        self.T = T
        Tinv = np.linalg.inv(T)  # transformationMatrix_.inverse() (dense LU), cpp:270-293
        Mbar = Tinv.T @ M @ Tinv
        self.Mbar = Mbar
        self.Mbar_b = Mbar[:6, :6].copy()
        self.Mbar_j = Mbar[6:, 6:].copy()
        Jst, Jsw = self.compute_jacobians(kd)
        self.Jc = Jst @ Tinv
        self.Js = Jsw @ Tinv
        nu = np.concatenate([self.base_vel, self.joint_vel])
        self.Cnu = kd.Cnu
        self.bbar = Tinv.T @ (self.Cnu + M @ self.Tdot_inv @ nu)  # quirk A.3
        self.compute_derivatives()
        self.Tdot_inv = -Tinv @ self.Tdot @ Tinv  # used next cycle

    # cpp:296-320
    def compute_transformation_matrix(self):
        pB = self.base_pose[:3]
        Ad = np.eye(6)
        Ad[0:3, 3:6] = skew(self.com - pB)
        Adinv = Ad.copy()
        Adinv[0:3, 3:6] = -Adinv[0:3, 3:6]
        sel = np.hstack([np.eye(6), np.zeros((6, NJ))])
        com_full = Adinv @ np.linalg.inv(self.M_bb) @ sel @ self.M
        T = np.zeros((ND, ND))
        T[:6, :] = com_full
        T[6:, 6:] = np.eye(NJ)
        return T

    # cpp:322-342
    def compute_jacobians(self, kd):
        Jst = np.zeros((3 * NL, ND)); Jsw = np.zeros((3 * NL, ND))
        for l in range(NL):
            Jf = kd.foot_J[3 * l:3 * l + 3]
            Jst[3 * l:3 * l + 3] = Jf * self.foot_contacts[l]
            Jsw[3 * l:3 * l + 3] = Jf * (0 if self.foot_contacts[l] else 1)
        return Jst, Jsw

    # cpp:384-402
    def compute_derivatives(self):
        if self.is_switching:
            self.Tdot = np.zeros((ND, ND))
            self.Jc_dot = np.zeros((3 * NL, ND))
            self.Js_dot = np.zeros((3 * NL, ND))
        else:
            dt = 1.0 / self.params["loop_rate"]
            self.Tdot = (self.T - self.old_T) / dt
            self.Jc_dot = (self.Jc - self.old_Jc) / dt
            self.Js_dot = (self.Js - self.old_Js) / dt
        self.old_T = self.T.copy()
        self.old_Jc = self.Jc.copy()
        self.old_Js = self.Js.copy()

    # cpp:404-424
    def compute_non_sliding_constraints(self):
        mu = self.params["friction"]
        t1 = np.array([1.0, 0, 0]); t2 = np.array([0, 1.0, 0]); n = np.array([0, 0, 1.0])
        D = np.vstack([t1 - mu * n, -(t1 + mu * n), t2 - mu * n, -(t2 + mu * n)])
        Dfr = np.zeros((4 * NL, 3 * NL))
        for l in range(NL):
            Dfr[4 * l:4 * l + 4, 3 * l:3 * l + 3] = D * self.foot_contacts[l]
        return Dfr

    # cpp:426-445
    def compute_desired_wrench(self):
        p = self.params
        Kp = p["kp"] * np.eye(6); Kp[2, 2] = p["kp_z"]
        Kd = p["kd"] * np.eye(6)
        Ki = p["ki"] * np.eye(6)
        gw = np.array([0, 0, self.total_mass * p["gravity"], 0, 0, 0])
        W = (-Kp @ (self.current_pose - self.desired_pose) - Kd @ (self.com_vel6 - self.desired_com_vel)
             - Ki @ self.integral_error + gw + self.Mbar_b @ self.desired_com_acc)
        self.integral_error = self.integral_error + (self.current_pose - self.desired_pose) / p["loop_rate"]
        return W

    # cpp:447-464 (feet from cpp:344-382)
    def compute_commanded_acceleration_swing_legs(self):
        p = self.params
        kd = self.kd
        cmd = (self.desired_sw_acc + p["kd_swing"] * (self.desired_sw_vel - kd.foot_vel.ravel())
               + p["kp_swing"] * (self.desired_sw_pos - kd.foot_pos.ravel()))
        for l in range(NL):
            cmd[3 * l:3 * l + 3] *= (0 if self.foot_contacts[l] else 1)
        return cmd

    # cpp:466-542
    def assemble_qp(self):
        p = self.params
        sl = 6 + NJ + 3 * NL
        S = np.hstack([np.zeros((3 * NL, 6 + NJ)), np.eye(3 * NL), np.zeros((3 * NL, 3 * NL))])
        Q = np.eye(6)
        Rm = np.eye(NV)
        Rm[sl:, sl:] = p["slack_weight"] * np.eye(3 * NL)
        Jc_com, Jc_j = self.Jc[:, :6], self.Jc[:, 6:]
        Js_com, Js_j = self.Js[:, :6], self.Js[:, 6:]
        H = S.T @ Jc_com @ Q @ Jc_com.T @ S + Rm
        W = self.compute_desired_wrench()
        self.W = W
        g = -S.T @ Jc_com @ Q @ W
        Dfr = self.compute_non_sliding_constraints()
        Z = np.zeros
        A = np.block([
            [self.Mbar_b, Z((6, NJ)), -Jc_com.T, Z((6, 3 * NL))],
            [Jc_com, Jc_j, Z((3 * NL, 3 * NL)), Z((3 * NL, 3 * NL))],
            [Z((4 * NL, 6)), Z((4 * NL, NJ)), Dfr, Z((4 * NL, 3 * NL))],
            [Z((NJ, 6)), self.Mbar_j, -Jc_j.T, Z((NJ, 3 * NL))],
            [Js_com, Js_j, Z((3 * NL, 3 * NL)), -np.eye(3 * NL)],
            [Js_com, Js_j, Z((3 * NL, 3 * NL)), np.eye(3 * NL)],
        ])
        qd = self.joint_vel.copy()
        gw = np.array([0, 0, self.total_mass * p["gravity"], 0, 0, 0])
        r1 = -self.Jc_dot[:, :6] @ self.com_vel6 - self.Jc_dot[:, 6:] @ qd
        cmd = self.compute_commanded_acceleration_swing_legs()
        rsw = cmd - self.Js_dot[:, :6] @ self.com_vel6 - self.Js_dot[:, 6:] @ qd
        self.r1, self.rsw, self.cmd = r1, rsw, cmd
        ub = np.concatenate([-gw, r1, np.zeros(4 * NL), p["max_torque"] * np.ones(NJ) - self.bbar[6:],
                             rsw, INFTY * np.ones(3 * NL)])
        lb = np.concatenate([-gw, r1, -INFTY * np.ones(4 * NL), -p["max_torque"] * np.ones(NJ) - self.bbar[6:],
                             -INFTY * np.ones(3 * NL), rsw])
        return H, g, A, lb, ub

    def solve_qp(self):
        H, g, A, lb, ub = self.assemble_qp()
        self.qp = (H, g, A, lb, ub)
        x, st, it = solve_qp(H, g, A, lb, ub, self.params["max_wsr"])
        self.first_iteration = False  # init on the first call, hotstart afterwards (cpp:523-533)
        self.qp_status, self.qp_iters = st, it
        self.qp_solution = x if st == QP_OK else np.zeros(NV)
        return st

    # cpp:553-577
    def compute_joint_torques(self):
        x = self.qp_solution
        qdd = x[6:18]
        f = x[18:30]
        tau = self.Mbar_j @ qdd + self.bbar[6:] - self.Jc[:, 6:].T @ f
        self.tau, self.grf = tau, f.copy()
        return tau

    def step(self):
        """One controlLoop() iteration (cpp:650-652)."""
        self.update_state()
        st = self.solve_qp()
        tau = self.compute_joint_torques()
        return tau, self.grf, self.qp_solution, st, self.qp_iters

    def debug_record(self):
        """Intermediates in include/wbc.h WBC_DBG_* layout (unmasked foot Jacobians)."""
        kd = self.kd
        Tinv = np.linalg.inv(self.T)
        return dict(com=self.com, comvel=kd.com_vel, pose=self.current_pose, vc=self.com_vel6, M=self.M,
                    Cnu=self.Cnu, Jfeet=kd.foot_J, pfeet=kd.foot_pos.ravel(), vfeet=kd.foot_vel.ravel(),
                    Mbar_b=self.Mbar_b, Mbar_j=self.Mbar_j, Jbar=kd.foot_J @ Tinv, bbar=self.bbar,
                    W=self.W, r1=self.r1, rsw=self.rsw)


def run_batch(base_pose, nu, qj, ref, contacts, switching, model=None, params=None):
    """Cold (stateless) batch: every robot from setInitialState() with explicit switching flags."""
    model = model or Model()
    B = base_pose.shape[0]
    out = dict(tau=np.zeros((B, NJ)), grf=np.zeros((B, NJ)), x=np.zeros((B, NV)),
               status=np.zeros(B, int), iters=np.zeros(B, int), ctrl=[])
    for b in range(B):
        c = ReferenceWBC(model, params)
        c.set_state(base_pose[b], nu[b], qj[b])
        c.set_reference(ref[b], [(contacts[b] >> i) & 1 for i in range(NL)], bool(switching[b]))
        tau, grf, x, st, it = c.step()
        out["tau"][b], out["grf"][b], out["x"][b], out["status"][b], out["iters"][b] = tau, grf, x, st, it
        out["ctrl"].append(c)
    return out
