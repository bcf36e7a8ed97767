"""The restoration phase of the oracle (oracle/lafse3_oracle.c: soft restoration + IPOPT's restoration phase) on
tests/golden/resto.npz: NLP instances whose filter line search fails (18 samples of the configs[2] bench batch
holding 26 such sol_gradient jobs, 64 moving-gate MPC solves of configs[4]).  Without the restoration phase
(restoration = 0, round 2's solver) they end in line-search failures; with it every instance reaches a point the
independent torch-autograd certificate (tests/kkt.py) accepts as a KKT point of the reference's NLP."""
import numpy as np
import pytest

from oracle import oracle as O


@pytest.fixture(scope="module")
def g(golden):
    return golden("resto")


def _moving_args(g):
    dn = g["moving_dnn_out"]
    nrm = [np.float64(np.sqrt(np.float32(sum(np.float64(np.float32(c * c)) for c in v)))) for v in dn[:, 3:6]]
    q32 = np.stack([O.rd2quat(v.astype(np.float64), n) for v, n in zip(dn[:, 3:6], nrm)])
    return (g["moving_ini"], g["moving_goal"], dn[:, :3].astype(np.float64), q32, dn[:, 6].astype(np.float64))


def test_fixture_instances_fail_without_restoration(g):
    r = O.solve(*_moving_args(g), ulast=g["moving_u_last"], params=O.default_params(restoration=0))
    assert np.mean(r["status"] == 3) >= 0.9, np.unique(r["status"], return_counts=True)
    _, _, st = O.sol_gradient(g["bench_ini"], g["bench_goal"], g["bench_gate12"], g["bench_dnn_out"],
                              params=O.default_params(restoration=0))
    assert np.sum(st == 3) >= 10


def test_moving_failures_restored_to_kkt_points(g):
    import kkt
    args = _moving_args(g)
    r = O.solve(*args, ulast=g["moving_u_last"])
    assert np.all(r["status"] <= 1), np.unique(r["status"], return_counts=True)
    bad = []
    for i in range(len(r["status"])):
        k = kkt.kkt_residual(r["x"][i], r["u"][i], r["lam"][i], args[0][i], args[1][i], args[2][i], args[3][i],
                             args[4][i], ulast=g["moving_u_last"][i])
        if not (k["primal"] <= 5e-7 and k["dual"] <= 1e-4 * k["s_d"] and k["compl"] <= 1e-6 and k["bound_viol"] <= 0):
            bad.append((i, k))
    assert not bad, bad


def test_bench_failures_restored(g):
    import kkt
    it = np.zeros((18, 9), np.int32)
    _, R, st = O.sol_gradient(g["bench_ini"], g["bench_goal"], g["bench_gate12"], g["bench_dnn_out"], iters=it)
    assert np.all(st <= 1), np.unique(st, return_counts=True)
    assert np.all(np.isfinite(R))
    # the jobs that failed without restoration: certified optima
    _, _, st0 = O.sol_gradient(g["bench_ini"], g["bench_goal"], g["bench_gate12"], g["bench_dnn_out"],
                               params=O.default_params(restoration=0))
    pp, qq, tt, uu = O.grad_params(g["bench_dnn_out"])
    for b, j in np.argwhere(st0 == 3):
        r = O.solve(g["bench_ini"][b:b + 1], g["bench_goal"][b:b + 1], pp[b, j][None], qq[b, j][None], tt[b, j:j + 1])
        assert r["status"][0] <= 1 and r["iters"][0] == it[b, j]
        k = kkt.kkt_residual(r["x"][0], r["u"][0], r["lam"][0], g["bench_ini"][b], g["bench_goal"][b], pp[b, j],
                             qq[b, j], tt[b, j])
        assert k["primal"] <= 5e-7 and k["dual"] <= 1e-4 * k["s_d"] and k["compl"] <= 1e-6, (b, j, k)


def test_watchdog_cuts_the_post_restoration_crawl(g):
    """IPOPT's watchdog (watchdog_shortened_iter_trigger 10, watchdog_trial_iter_max 3; oracle backtrack / orc_ipm):
    bench-fixture job (sample 13, probe 4) crawls for 1226 iterations after its restoration phase without it (short
    steps under repeated inertia correction); with it the solve ends in <= 400 iterations at a certified KKT point.
    Over the whole fixture the watchdog changes no status and lowers the total iteration count."""
    import kkt
    pp, qq, tt, _ = O.grad_params(g["bench_dnn_out"])
    b, j = 13, 4
    args = (g["bench_ini"][b:b + 1], g["bench_goal"][b:b + 1], pp[b, j][None], qq[b, j][None], tt[b, j:j + 1])
    off = O.solve(*args, params=O.default_params(watchdog=0))
    on = O.solve(*args)
    assert off["status"][0] == 0 and off["iters"][0] >= 1000, off["iters"]
    assert on["status"][0] == 0 and on["iters"][0] <= 400, on["iters"]
    k = kkt.kkt_residual(on["x"][0], on["u"][0], on["lam"][0], *(a[0] for a in args))
    assert k["primal"] <= 5e-7 and k["dual"] <= 1e-4 * k["s_d"] and k["compl"] <= 1e-6, k
    it0, it1 = np.zeros((18, 9), np.int32), np.zeros((18, 9), np.int32)
    _, _, s0 = O.sol_gradient(*(g[k] for k in ("bench_ini", "bench_goal", "bench_gate12", "bench_dnn_out")),
                              iters=it0, params=O.default_params(watchdog=0))
    _, _, s1 = O.sol_gradient(*(g[k] for k in ("bench_ini", "bench_goal", "bench_gate12", "bench_dnn_out")),
                              iters=it1)
    assert np.all(s0 <= 1) and np.all(s1 <= 1)
    assert it1.sum() < it0.sum() and it1.max() < it0.max(), (it0.sum(), it1.sum(), it0.max(), it1.max())
