"""qp_ipm — a second, independent QP method for the oracle.  TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module, and only as a checker.  The product path never does.

The reference solves its whole-body QP (src/whole_body_controller.cpp:466-535: H, g, the 70
general constraints lbA <= A x <= ubA, qpOASES SQProblem) with an active-set method.  The
oracle's own solver (oracle/wbc_np.py `gi_solve`, oracle/wbc_ref.c) is the Goldfarb-Idnani dual
active-set method, and so is the HIP kernel.  A mistake specific to that method (a wrong
degenerate-row rule, a wrong infeasibility verdict) would be shared by all three.  This module
answers the same two questions by different means:

  * feasible?  A phase-1 linear program over the raw constraint rows (scipy HiGHS): minimise
    the total bound violation v >= 0 of lbA - v <= A x <= ubA + v.  The QP is infeasible iff
    the minimum is positive (above a tolerance scaled by the bounds).  Zero rows (the
    reference's mode-masked rows) are kept: their bounds alone decide.
  * optimum?   A dense primal-dual interior-point method (Mehrotra predictor-corrector) on the
    same rows, then a polish: the rows the interior point leaves active are solved as
    equalities (one KKT solve) and the polished point is accepted only if it is primal
    feasible with non-negative multipliers.

Neither step uses a working set, Householder or Givens updates, or the dual path of GI.
"""
from __future__ import annotations

import numpy as np

INFTY = 1.0e20  # qpOASES::INFTY (cpp:508,512,514)
QP_OK, QP_INFEASIBLE, QP_NUMERIC = 0, 2, 3


def _rows(A, lbA, ubA):
    """lbA <= A x <= ubA -> equalities (E, e) and inequalities C x >= c; zero rows dropped
    (their feasibility is the phase-1 program's business)."""
    E, e, C, c = [], [], [], []
    for i in range(A.shape[0]):
        row, lo, hi = A[i], lbA[i], ubA[i]
        if not np.any(row != 0.0):
            continue
        lo_inf, hi_inf = lo <= -INFTY, hi >= INFTY
        if not lo_inf and not hi_inf and lo == hi:
            E.append(row); e.append(lo)
            continue
        if not lo_inf:
            C.append(row); c.append(lo)
        if not hi_inf:
            C.append(-row); c.append(-hi)
    n = A.shape[1]
    mk = lambda r: np.array(r, float).reshape(-1, n)
    return mk(E), np.array(e, float), mk(C), np.array(c, float)


def feasible(A, lbA, ubA, tol=1e-7):
    """Phase-1 LP: is there x with lbA <= A x <= ubA?  Returns (feasible, min total violation)."""
    from scipy.optimize import linprog

    m, n = A.shape
    lo = np.where(lbA <= -INFTY, -np.inf, lbA)
    hi = np.where(ubA >= INFTY, np.inf, ubA)
    # variables [x (free), v (>= 0, one per row)]: A x - v <= hi,  -A x - v <= -lo
    rows, rhs = [], []
    for i in range(m):
        ev = np.zeros(m); ev[i] = -1.0
        if np.isfinite(hi[i]):
            rows.append(np.concatenate([A[i], ev])); rhs.append(hi[i])
        if np.isfinite(lo[i]):
            rows.append(np.concatenate([-A[i], ev])); rhs.append(-lo[i])
    cost = np.concatenate([np.zeros(n), np.ones(m)])
    bounds = [(None, None)] * n + [(0, None)] * m
    res = linprog(cost, A_ub=np.array(rows), b_ub=np.array(rhs), bounds=bounds, method="highs",
                  options=dict(primal_feasibility_tolerance=1e-10, dual_feasibility_tolerance=1e-10))
    if res.status != 0:
        raise RuntimeError(f"phase-1 LP failed: {res.message}")
    scale = 1.0 + np.max(np.abs(np.concatenate([lo[np.isfinite(lo)], hi[np.isfinite(hi)]])), initial=0.0)
    return bool(res.fun <= tol * scale), float(res.fun)


def ipm(H, g, E, e, C, c, tol=1e-11, max_iter=200):
    """Mehrotra predictor-corrector on min 1/2 x'Hx + g'x, E x = e, C x >= c (slacks s = C x - c),
    Newton steps from the full augmented system [[H, -E', -C'], [E, 0, 0], [C, 0, S/Z]] (no
    C' (Z/S) C product, whose entries blow up as slacks vanish).  Stops when the residuals and
    the complementarity gap are below tol relative to the problem data; the polish supplies the
    last digits.  Returns (x, y, z, s, converged)."""
    n, me, mi = g.size, E.shape[0], C.shape[0]
    x = np.zeros(n)
    y = np.zeros(me)
    s = np.maximum(C @ x - c, 1.0) if mi else np.zeros(0)
    z = np.ones(mi)
    data = 1.0 + max(np.abs(e).max(initial=0.0), np.abs(c).max(initial=0.0), np.abs(g).max(initial=0.0),
                     np.abs(H).max(initial=0.0))
    N = n + me + mi
    K = np.zeros((N, N))
    K[:n, :n] = H
    K[:n, n:n + me] = -E.T
    K[:n, n + me:] = -C.T
    K[n:n + me, :n] = E
    K[n + me:, :n] = C
    di = np.arange(n + me, N)
    converged = False
    for _ in range(max_iter):
        rd = H @ x + g - E.T @ y - C.T @ z
        re = E @ x - e
        ri = C @ x - c - s
        mu = (s @ z) / mi if mi else 0.0
        xs = 1.0 + np.abs(x).max()
        if (max(np.abs(rd).max(initial=0.0), np.abs(re).max(initial=0.0), np.abs(ri).max(initial=0.0))
                <= tol * data * xs and mu <= tol * data * xs):
            converged = True
            break
        K[di, di] = s / z

        def solve(rc):
            sol = np.linalg.solve(K, np.concatenate([-rd, -re, -ri + rc / z]))
            dx, dy, dz = sol[:n], sol[n:n + me], sol[n + me:]
            ds = (rc - s * dz) / z
            return dx, dy, dz, ds

        def step(v, dv):
            neg = dv < 0
            return min(1.0, np.min(-v[neg] / dv[neg])) if np.any(neg) else 1.0

        # predictor (affine scaling)
        dxa, dya, dza, dsa = solve(-s * z)
        aa = min(step(s, dsa), step(z, dza))
        mu_aff = ((s + aa * dsa) @ (z + aa * dza)) / mi if mi else 0.0
        sigma = (mu_aff / mu) ** 3 if mu > 0 else 0.0
        # corrector
        dx, dy, dz, ds = solve(-s * z + sigma * mu - dsa * dza)
        a = min(1.0, 0.995 * min(step(s, ds), step(z, dz)))
        x, y, z, s = x + a * dx, y + a * dy, z + a * dz, s + a * ds
        if a < 1e-12:
            break  # stalled
    return x, y, z, s, converged


def polish(H, g, E, e, C, c, x, z, s):
    """Solve the KKT system with the interior point's active rows (z_i > s_i) as equalities; keep
    the result if it is primal feasible and multipliers of the right signs exist (non-negative
    least squares).  At a foot with zero force four friction faces meet at one vertex, so the
    active rows are dependent: an independent subset (QR with column pivoting) is solved, and
    the multipliers are not unique.  Otherwise return x unchanged."""
    from scipy.linalg import qr
    from scipy.optimize import nnls

    act = z > s if C.shape[0] else np.zeros(0, bool)
    Ca = C[act]
    Aeq = np.vstack([E, Ca])
    beq = np.concatenate([e, c[act]])
    n = g.size
    if Aeq.shape[0]:
        _, Rq, piv = qr(Aeq.T, pivoting=True, mode="economic")
        d = np.abs(np.diag(Rq))
        keep = piv[: int(np.sum(d > 1e-10 * d[0]))] if d.size and d[0] > 0 else piv[:0]
    else:
        keep = np.zeros(0, int)
    Ak, bk = Aeq[keep], beq[keep]
    m = Ak.shape[0]
    K = np.zeros((n + m, n + m))
    K[:n, :n] = H
    K[:n, n:] = -Ak.T
    K[n:, :n] = Ak
    xp = np.linalg.solve(K, np.concatenate([-g, bk]))[:n]
    scale = 1.0 + np.abs(xp).max() + np.abs(g).max()
    if not (np.all(C @ xp - c >= -1e-9 * (1.0 + np.abs(c)))
            and np.abs(E @ xp - e).max(initial=0.0) <= 1e-9 * (1.0 + np.abs(e).max(initial=0.0))):
        return x, False
    grad = H @ xp + g  # = E' y + Ca' za with za >= 0
    M = np.hstack([E.T, -E.T, Ca.T])
    lam, res = nnls(M, grad, maxiter=50 * M.shape[1])
    if res > 1e-7 * scale:
        return x, False
    return xp, True


def solve(H, g, A, lbA, ubA):
    """(x, status) of the reference's QP by phase-1 LP + interior point + polish."""
    ok, _ = feasible(A, lbA, ubA)
    if not ok:
        return np.zeros(g.size), QP_INFEASIBLE
    E, e, C, c = _rows(A, lbA, ubA)
    # a weakly active row (z and s both small when the interior point stops) can leave the active
    # set ambiguous: the polish then fails its checks, and the interior point is run tighter
    for tol in (1e-11, 1e-13, 1e-15):
        x, y, z, s, conv = ipm(H, g, E, e, C, c, tol=tol)
        if not conv:
            break
        xp, ok = polish(H, g, E, e, C, c, x, z, s)
        if ok:
            return xp, QP_OK
    return x, (QP_OK if conv else QP_NUMERIC)
