"""TEST INFRASTRUCTURE: the rounding yardstick of the iteration-path agreement tests.

The device factorises the same Newton systems as the oracle with another operation order (the MFMA Riccati stage,
riccati_mfma.inc), so device and oracle agree to rounding, and on long, ill-conditioned solves rounding alone
moves IPOPT's near-tie decisions (an inertia correction one factor of kappa apart, a filter entry, one backtracking
halving; tools/resto_diverge.py).  How often it does is measured here on the same jobs with the oracle against
itself: its -O3 / FMA-contraction build (liblafse3_oracle_fast.so, other rounding, same source) against its strict
parity build (liblafse3_oracle.so).  A device test then asks for at least that many exact paths minus 2 % of the
jobs, instead of a fixed fraction that a change of the device's rounding alone could flip.  Reference: IPOPT's
default options at /root/reference/quad_OC.py:170-174.
"""
import numpy as np


def grad_paths(args, status_strict, iters_strict, **kw):
    """sol_gradient jobs (B x 9 solves): how many the FMA build solves with the strict build's status and iteration
    count."""
    from oracle import oracle as O
    ito = np.zeros_like(iters_strict)
    _, _, so = O.sol_gradient(*args, fast=True, iters=ito, **kw)
    return int(((so == status_strict) & (ito == iters_strict)).sum())


def solve_paths(args, kw, ref_strict):
    """ocp solves: how many the FMA build solves with the strict build's status and iteration count."""
    from oracle import oracle as O
    r = O.solve(*args, fast=True, **kw)
    return int(((r["status"] == ref_strict["status"]) & (r["iters"] == ref_strict["iters"])).sum())
