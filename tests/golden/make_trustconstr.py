#!/usr/bin/env python3
"""Independent-solver fixture for the NLP optimum (SURVEY.md §8(c) golden item 4).

TEST INFRASTRUCTURE.  The reference solves its NLP with CasADi + IPOPT (quad_OC.py:170-174), neither of
which exists in this image.  This script re-solves the same NLP with a solver that shares no code with the
oracle or the HIP kernels -- scipy.optimize.minimize(method="trust-constr") -- on the problem built in torch
fp64 by tests/kkt.py (objective, multiple-shooting defects and their derivatives by autograd), from the
reference's own initial guess (quad_OC.py:142,158: u = midpoint of [0, 2.44], x_1..x_N = 0), and stores its
optimum next to the oracle's for the same inputs:

    python3 tests/golden/make_trustconstr.py        # up to ~45 min on 8 cores, writes tests/golden/trustconstr.npz

tests/test_oracle_golden.py::test_oracle_optimum_matches_trust_constr then requires the oracle's cost to
agree with trust-constr's to <= 1e-6 relative on every instance where both reach the same KKT point, and
lists the instances that land in other local optima (the NLP is nonconvex; at generation time 3 of 16, see
the printed table).  Limits per instance: maxiter 3000 or 20 minutes (status 3).
"""
from __future__ import annotations

import math
import os
import sys
import time

import numpy as np
import torch
from scipy.optimize import Bounds, NonlinearConstraint, minimize

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(HERE))
from kkt import U_UB, W_UB, kkt_residual, objective_and_defects  # noqa: E402
from learningagileflight_se3_amd import scenario as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

N, NX, NU = 50, 13, 4
NV = N * NX + N * NU


def unpack(z):
    x = z[: N * NX].reshape(N, NX)
    u = z[N * NX:].reshape(N, NU)
    return x, u


def solve_trust_constr(ini, goal, ptra, qtra, t, maxiter=3000, max_seconds=1200.0):
    dt = torch.float64
    args = [torch.tensor(a, dtype=dt) for a in (ini, goal, ptra, qtra)]
    tt = torch.tensor(float(t), dtype=dt)
    ul = torch.zeros(4, dtype=dt)

    def parts(zt):
        x, u = zt[: N * NX].reshape(N, NX), zt[N * NX:].reshape(N, NU)
        X = torch.cat([args[0][None], x], 0)
        return objective_and_defects(X, u, args[0], args[1], args[2], args[3], tt, ul)

    def fun(z):
        return float(parts(torch.tensor(z, dtype=dt))[0])

    from torch.func import grad as fgrad, hessian as fhess, jacrev
    obj = lambda q: parts(q)[0]
    con = lambda q: parts(q)[1].reshape(-1)

    def grad(z):
        return fgrad(obj)(torch.tensor(z, dtype=dt)).numpy()

    def hess(z):
        return fhess(obj)(torch.tensor(z, dtype=dt)).numpy()

    def cons(z):
        return con(torch.tensor(z, dtype=dt)).detach().numpy()

    def cjac(z):
        return jacrev(con)(torch.tensor(z, dtype=dt)).numpy()

    def chess(z, v):
        vt = torch.tensor(v, dtype=dt)
        return fhess(lambda q: (con(q) * vt).sum())(torch.tensor(z, dtype=dt)).numpy()

    lb = np.full(NV, -np.inf)
    ub = np.full(NV, np.inf)
    xl, ul_ = lb[: N * NX].reshape(N, NX), ub[: N * NX].reshape(N, NX)
    xl[:, 10:13], ul_[:, 10:13] = -W_UB, W_UB
    lb[N * NX:], ub[N * NX:] = 0.0, U_UB
    z0 = np.zeros(NV)
    z0[N * NX:] = 0.5 * U_UB                                           # quad_OC.py:142
    t_start = time.time()

    def stop(xk, state):   # wall-clock cap (status 3): the fixture records it as not converged
        return time.time() - t_start > max_seconds

    res = minimize(fun, z0, method="trust-constr", jac=grad, hess=hess,
                   constraints=[NonlinearConstraint(cons, 0.0, 0.0, jac=cjac, hess=chess)],
                   bounds=Bounds(lb, ub, keep_feasible=False), callback=stop,
                   options=dict(maxiter=maxiter, gtol=1e-10, xtol=1e-14, barrier_tol=1e-10, verbose=0))
    x, u = unpack(res.x)
    X = np.concatenate([ini[None], x], 0)
    return X, u, float(res.fun), int(res.status), int(res.nit), float(res.constr_violation)


def _one(job):
    torch.set_num_threads(1)
    i, (ini, goal, p, q, t) = job
    t0 = time.time()
    out = solve_trust_constr(ini, goal, p, q, t)
    print(f"  instance {i} done in {time.time() - t0:.0f} s (status {out[3]}, {out[4]} iterations)", flush=True)
    return out + (time.time() - t0,)


def main(n=16, seed=11, workers=8):
    import multiprocessing as mp
    # one BLAS / OpenMP thread per worker (inherited by the spawned workers): with the default thread pools
    # eight workers oversubscribe the cores ~60x and trust-constr crawls
    for v in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[v] = "1"
    sb = S.synthetic_batch(n, seed=seed)
    p = sb["dnn_out"][:, :3].astype(np.float64)
    a = sb["dnn_out"][:, 3:6].astype(np.float64)
    t = sb["dnn_out"][:, 6].astype(np.float64)
    q = np.stack([O.rd2quat(ai) for ai in a])
    ref = O.solve(sb["ini"], sb["goal"], p, q, t)
    rec = {k: [] for k in ("x_tc", "u_tc", "J_tc", "status_tc", "nit_tc", "cv_tc", "kkt_tc")}
    jobs = [(sb["ini"][i], sb["goal"][i], p[i], q[i], t[i]) for i in range(n)]
    with mp.get_context("spawn").Pool(min(workers, n)) as pool:
        results = pool.map(_one, list(enumerate(jobs)), chunksize=1)
    print(" i   J_oracle           J_trust-constr     rel diff   tc status nit  constr_viol  KKT dual (oracle lam)")
    for i, (X, U, J, st, nit, cv, sec) in enumerate(results):
        # the trust-constr point certified with the oracle's multipliers (same optimum => small dual residual)
        k = kkt_residual(X, U, ref["lam"][i], sb["ini"][i], sb["goal"][i], p[i], q[i], t[i])
        rec["x_tc"].append(X); rec["u_tc"].append(U); rec["J_tc"].append(J)
        rec["status_tc"].append(st); rec["nit_tc"].append(nit); rec["cv_tc"].append(cv); rec["kkt_tc"].append(k["dual"])
        Jo = float(ref["cost"][i])
        print(f"{i:2d}  {Jo:.12e}  {J:.12e}  {abs(J - Jo) / abs(Jo):.2e}   {st}  {nit:5d}  {cv:.2e}  {k['dual']:.2e}"
              f"   ({sec:.0f} s)", flush=True)
    out = dict(ini=sb["ini"], goal=sb["goal"], p=p, q=q, t=t,
               x_oracle=ref["x"], u_oracle=ref["u"], lam_oracle=ref["lam"], J_oracle=ref["cost"],
               **{k: np.asarray(v) for k, v in rec.items()})
    np.savez_compressed(os.path.join(HERE, "trustconstr.npz"), **out)
    print("wrote trustconstr.npz")


if __name__ == "__main__":
    main(int(os.environ.get("N_INST", "16")))
