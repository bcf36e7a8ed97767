"""The barrier parameter update mu_new = max(mu_min, min(0.2 mu, mu^1.5)) (IPOPT's monotone mu strategy,
kappa_mu = 0.2, theta_mu = 1.5; quad_OC.py:170-174 leaves every algorithmic option at IPOPT's default).

mu^1.5 is the one non-elementary operation whose result becomes solver state: a one-ulp different mu moves every
later iterate.  The oracle (orc_pow15) and the kernel (ipm_kernel.hip pow15) compute it by the same double-double
formula, correctly rounded; the device's libm pow is not (0.02^1.5 one ulp low), which made device and oracle take
different mu sequences (round 4, tools/resto_diverge.py).  Checked here against an exact (80-digit) reference."""
from decimal import Decimal, getcontext

import numpy as np

from oracle import oracle as O


def _exact(x: float) -> float:
    getcontext().prec = 80
    return float((Decimal(x) ** 3).sqrt())   # Decimal -> float rounds to nearest


def test_pow15_is_correctly_rounded():
    L = O.lib()
    rng = np.random.default_rng(7)
    xs = list(10.0 ** rng.uniform(-9.0, 0.0, 4000))
    mu = 0.1   # the solver's own sequence from mu_init = 0.1 down to mu_min = tol / 10
    while mu > 1e-9:
        xs.append(mu)
        mu = max(1e-9, min(0.2 * mu, _exact(mu)))
    bad = [x for x in xs if L.orc_pow15(x) != _exact(x)]
    assert not bad, bad[:5]
