#!/usr/bin/env python3
"""CPU experiment: cold-start working-set guesses for the 12-variable QP.

For every QP of a bench workload, builds the engine's 12-variable problem (oracle/wbc_reduced.py)
and runs the Goldfarb-Idnani method with the kernel's selection rule (slack / |reference row|,
ties to the lowest row id) from several starting working sets:

  cold      the empty set (the engine today);
  guess     the rows violated at the unconstrained optimum x0, most violated first, added as a
            block (dependent rows skipped, at most 12), then the point where they all hold:
            negative multipliers are dropped one at a time (most negative first) until the set
            is dual feasible, and the loop continues from there.

It prints the per-QP working-set operations and the wave cost model: a wave runs its four QPs'
largest count of each phase (block adds, repair drops, loop passes), in the kernel's wave order
(four consecutive robots, or the wave map's buckets for mixed masks).
Test/analysis tooling only; not part of the engine.
"""
from __future__ import annotations

import argparse
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import wbc_np as W  # noqa: E402
import wbc_reduced as WR  # noqa: E402
from quadrupedwholebodycontroller_amd import workloads  # noqa: E402


def problem(args):
    pose, nu, qj, ref, kap, sw = args
    c = W.ReferenceWBC()
    c.set_state(pose, nu, qj)
    c.set_reference(ref, [(kap >> i) & 1 for i in range(4)], bool(sw))
    c.update_state()
    c.assemble_qp()
    rp = WR.reduced_problem(c)
    if rp is None:
        return None
    p = c.params
    tm = p["max_torque"]
    tol = []
    for i in rp["ids"]:
        if i < 16:
            tol.append(1e-10)
        else:
            j, side = divmod(i - 16, 2)
            sg = -1.0 if side else 1.0
            tol.append(1e-10 * max(1.0, abs(-tm - sg * c.bbar[6 + j])))
    return dict(H=rp["H"], g=rp["g"], CI=rp["CI"], ci=rp["ci"], nsel=np.sqrt(np.maximum(rp["nsel"], 1e-300)),
                tol=np.array(tol), ids=np.array(rp["ids"]))


class GI:
    """Dual active set in the J-form (J = L^-T Q, R upper triangular), as the kernel's solve16."""

    def __init__(self, pr):
        self.pr = pr
        H, g = pr["H"], pr["g"]
        L = np.linalg.cholesky(H)
        self.J = np.linalg.inv(L).T
        self.x0 = -np.linalg.solve(H, g)
        self.x = self.x0.copy()
        self.R = np.zeros((12, 12))
        self.q = 0
        self.act = []
        self.u = np.zeros(0)
        self.n_ops = dict(block=0, repair=0, adds=0, drops=0)

    def slacks(self):
        return self.pr["CI"] @ self.x - self.pr["ci"]

    def add_col(self, d):
        q = self.q
        v = d[q:].copy()
        nrm = np.linalg.norm(v)
        if nrm <= 1e-13 * max(1.0, np.linalg.norm(d)):
            return False
        alpha = -nrm if v[0] >= 0 else nrm
        v[0] -= alpha
        vv = v @ v
        self.J[:, q:] -= np.outer(self.J[:, q:] @ v, v) * (2.0 / vv)
        self.R[:q, q] = d[:q]
        self.R[q, q] = alpha
        self.q += 1
        return True

    def drop(self, k):
        q, R, J = self.q, self.R, self.J
        R[:, k:q - 1] = R[:, k + 1:q]
        R[:, q - 1] = 0.0
        for j in range(k, q - 1):
            a, b = R[j, j], R[j + 1, j]
            h = np.hypot(a, b)
            c, s = (a / h, b / h) if h > 0 else (1.0, 0.0)
            rj, rj1 = R[j, j:q - 1].copy(), R[j + 1, j:q - 1].copy()
            R[j, j:q - 1] = c * rj + s * rj1
            R[j + 1, j:q - 1] = -s * rj + c * rj1
            Jj, Jj1 = J[:, j].copy(), J[:, j + 1].copy()
            J[:, j] = c * Jj + s * Jj1
            J[:, j + 1] = -s * Jj + c * Jj1
        self.q -= 1
        del self.act[k]
        self.u = np.delete(self.u, k)

    def point(self):
        """x, u with every active row tight: R^T v = -s_A(x0), u = R^-1 v, x = x0 + J1 v."""
        q = self.q
        CI, ci = self.pr["CI"], self.pr["ci"]
        sa = np.array([CI[p] @ self.x0 - ci[p] for p in self.act])
        Rq = self.R[:q, :q]
        v = np.linalg.solve(Rq.T, -sa)
        self.u = np.linalg.solve(Rq, v)
        self.x = self.x0 + self.J[:, :q] @ v

    def warm(self, rows, repair=True):
        for p in rows:
            if self.q >= 12:
                break
            d = self.J.T @ self.pr["CI"][p]
            if self.add_col(d):
                self.act.append(p)
                self.n_ops["block"] += 1
        if self.q == 0:
            return True
        self.point()
        while self.q and self.u.min() < -1e-10:
            if not repair:
                return False
            k = int(np.argmin(self.u))
            self.drop(k)
            self.n_ops["repair"] += 1
            if self.q:
                self.point()
            else:
                self.x = self.x0.copy()
                self.u = np.zeros(0)
        self.u = np.maximum(self.u, 0.0)
        return True

    def select(self):
        s = self.slacks()
        pr = self.pr
        w = np.where(s < -pr["tol"], s / pr["nsel"], np.inf)
        for p in self.act:
            w[p] = np.inf
        m = w.min()
        if not np.isfinite(m):
            return -1
        return int(np.nonzero(w <= m * (1.0 - 1e-9))[0][0])  # near-ties: the lowest id (WBC_TIE_BAND)

    def loop(self, max_iter=100):
        CI = self.pr["CI"]
        p = self.select()
        while p >= 0:
            npv = CI[p]
            sp = npv @ self.x - self.pr["ci"][p]
            up = 0.0
            while True:
                if self.n_ops["adds"] + self.n_ops["drops"] >= max_iter:
                    return "max_iter"
                q = self.q
                d = self.J.T @ npv
                z = self.J[:, q:] @ d[q:]
                r = np.linalg.solve(self.R[:q, :q], d[:q]) if q else np.zeros(0)
                t1, l = np.inf, -1
                for k in range(q):
                    if r[k] > 1e-14 and self.u[k] / r[k] < t1:
                        t1, l = self.u[k] / r[k], k
                zn = d[q:] @ d[q:]
                t2 = -sp / zn if zn > 1e-14 else np.inf
                t = min(t1, t2)
                if not np.isfinite(t):
                    return "infeasible"
                if np.isfinite(t2):
                    self.x = self.x + t * z
                    sp += t * (z @ npv)
                self.u = self.u - t * r
                up += t
                if np.isfinite(t2) and t2 <= t1:
                    self.u = np.append(self.u, up)
                    self.add_col(d)
                    self.act.append(p)
                    self.n_ops["adds"] += 1
                    break
                self.drop(l)
                self.n_ops["drops"] += 1
            p = self.select()
        return "ok"


def run_one(pr, mode):
    g = GI(pr)
    if mode == "guess":
        s = g.slacks()
        viol = np.where(s < -pr["tol"], s / pr["nsel"], np.inf)
        order = [int(i) for i in np.argsort(viol, kind="stable") if np.isfinite(viol[i])]
        g.warm(order)
    st = g.loop()
    return st, g.n_ops, g.x, sorted(g.act)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="stance_cold_b4096")
    ap.add_argument("--n", type=int, default=4096)
    args = ap.parse_args()
    if args.workload.startswith("stance"):
        inp = workloads.stance_cold(args.n, 1)
    else:
        inp = workloads.rl_random(args.n, 3)
    B = args.n
    jobs = [(inp["base_pose"][b], inp["nu"][b], inp["qj"][b], inp["ref"][b], int(inp["contacts"][b]),
             int(inp["switching"][b])) for b in range(B)]
    with Pool(8) as pool:
        probs = pool.map(problem, jobs, chunksize=64)
    res = {m: [] for m in ("cold", "guess")}
    for b, pr in enumerate(probs):
        for m in res:
            res[m].append(None if pr is None else run_one(pr, m))
    # per-QP stats and a wave cost model (ticks, pass = 2.9 k): block re-add f_add x pass, repair
    # drop f_rep x pass, the point 1.0 k; a wave runs its four QPs' largest count of each phase
    C_PASS, C_PT = 2900, 1000
    for m, rr in res.items():
        ok = [r for r in rr if r is not None]
        it = np.array([r[1]["adds"] + r[1]["drops"] for r in ok])
        blk = np.array([r[1]["block"] for r in ok])
        rep = np.array([r[1]["repair"] for r in ok])
        print(f"[{m}] QPs {len(ok)}: loop iters mean {it.mean():.2f} max {it.max()}  block mean {blk.mean():.2f} "
              f"max {blk.max()}  repair mean {rep.mean():.2f} max {rep.max()}")
        for f_add, f_rep in ((0.3, 1.0), (0.5, 1.0), (0.7, 1.0)):
            wave_cost = []
            for w0 in range(0, B, 4):
                grp = [rr[b] for b in range(w0, min(w0 + 4, B)) if rr[b] is not None]
                if not grp:
                    continue
                mi = max(r[1]["adds"] + r[1]["drops"] for r in grp) + 1
                mb = max(r[1]["block"] for r in grp)
                mr = max(r[1]["repair"] for r in grp)
                wave_cost.append(C_PASS * (mi + f_add * mb + f_rep * mr) + (C_PT if mb else 0))
            wc = np.array(wave_cost)
            print(f"    f_add {f_add} f_rep {f_rep}: wave solve cost mean {wc.mean():.0f} p99 {np.percentile(wc, 99):.0f} "
                  f"max {wc.max():.0f}")
    # agreement
    diffs = [np.abs(a[2] - b[2]).max() / (1 + np.abs(a[2]).max()) for a, b in zip(res["cold"], res["guess"])
             if a is not None and a[0] == "ok" and b[0] == "ok"]
    same = sum(a[0] == b[0] for a, b in zip(res["cold"], res["guess"]) if a is not None)
    print(f"status equal {same}, max rel x diff {max(diffs):.2e}")


if __name__ == "__main__":
    main()
