"""GPU tests of the restoration phase (ipm_kernel.hip / resto.inc) against the oracle (oracle/lafse3_oracle.c
orc_restoration) on tests/golden/resto.npz: the NLP instances whose filter line search fails -- 18 samples of the
configs[2] bench batch (synthetic_batch(4096, seed 1000); 162 sol_gradient solves) and 64 moving-gate MPC solves
of configs[4] (lafse3_get_input, quad_policy.py:202-211).

  * restoration = 0 (the 0.4 solver) reproduces the oracle's line-search failures on the device;
  * restoration = 1 (default): no instance ends in a line-search failure, the restoration counters report the
    phase's entries and returns, statuses / iteration counts agree with the oracle's, and where both took the
    same iteration path the rewards / trajectories agree to the A5 tolerances.
The restored solves are certified as KKT points of the reference NLP by tests/test_restoration_host.py (oracle
side); here the device has to follow the oracle onto them.
"""
import numpy as np
import pytest
import yardstick

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g(golden):
    return golden("resto")


def _engine(**overrides):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback by design)")
    from learningagileflight_se3_amd import _lib
    from learningagileflight_se3_amd.engine import Engine
    e = Engine()
    if overrides:
        e.set_params(_lib.default_params(**overrides))
    return e


def _bench_args(g):
    return (g["bench_ini"], g["bench_goal"], g["bench_gate12"], g["bench_dnn_out"])


def test_without_restoration_the_failures_reproduce(g):
    """restoration = 0: the device ends the oracle's line-search failures (restoration = 0) in line-search failures
    too, at least as many of them as the oracle's own FMA-contracted build does (the rounding yardstick,
    tests/yardstick.py: 8 of the 10).  Round 4's VALU stage reproduced 10 of 10, the MFMA stage 9 or 10: a
    line-search failure is the end of a long ill-conditioned path whose near-tie decisions rounding moves."""
    from oracle import oracle as O
    e = _engine(restoration=0)
    _, _, S9 = e.sol_gradient(*_bench_args(g), want_rewards=True)
    e.close()
    S9 = S9.cpu().numpy()
    prm = O.default_params(restoration=0)
    _, _, so = O.sol_gradient(*_bench_args(g), params=prm)
    _, _, sf = O.sol_gradient(*_bench_args(g), params=prm, fast=True)
    fail_o = so == 3
    yard = int((fail_o & (sf == 3)).sum())
    print(f"restoration=0: oracle ls_fail {fail_o.sum()}, device ls_fail {(S9 == 3).sum()}, "
          f"both {(fail_o & (S9 == 3)).sum()} (rounding yardstick: oracle FMA build {yard})")
    assert fail_o.sum() >= 10
    assert (fail_o & (S9 == 3)).sum() >= yard
    # regression bar: the count this kernel measured (9 of 10 since the MFMA stage, profiles/r05_*), so that a
    # drift towards the yardstick's floor shows up as a failure instead of passing silently
    assert (fail_o & (S9 == 3)).sum() >= 9, (fail_o & (S9 == 3)).sum()


def test_bench_failures_restored_on_device(g):
    """restoration = 1 on the 162 bench-fixture solves: every status solved/acceptable (the oracle's are), the
    restoration counters show entries == returns >= 10, and on the solves that take the oracle's iteration count the
    nine rewards agree to 1e-6 (relative).  How many solves take the oracle's exact iteration path is judged against
    the rounding yardstick (tests/yardstick.py): the oracle built with FMA contraction against its strict build on
    the same jobs (157 / 162 measured round 4) -- the device must reach that count minus 2 % of the jobs.  Every
    remaining divergence is preceded by rounding-level drift of theta / phi (tools/resto_diverge.py,
    profiles/r04_resto_diverge.log), so a fixed fraction would judge the rounding, not the solver."""
    from oracle import oracle as O
    e = _engine()
    it = torch.full((18, 9), -1, dtype=torch.int32, device=e.device)
    e.record_iters(it)
    o8, R9, S9 = e.sol_gradient(*_bench_args(g), want_rewards=True)
    rc = e.last_resto_counters()
    e.record_iters(None)
    e.check_device()
    R9, S9, it = R9.cpu().numpy(), S9.cpu().numpy(), it.cpu().numpy()
    e.close()
    ito = np.zeros((18, 9), np.int32)
    o8o, Ro, So = O.sol_gradient(*_bench_args(g), iters=ito)
    same = (S9 == So) & (it == ito)
    yard = yardstick.grad_paths(_bench_args(g), So, ito)
    print(f"device statuses {dict(zip(*np.unique(S9, return_counts=True)))}, resto {rc}, "
          f"same status+iterations {same.sum()}/162 (rounding yardstick: oracle FMA build {yard}/162)")
    _, _, s0 = O.sol_gradient(*_bench_args(g), params=O.default_params(restoration=0))
    restored = s0 == 3
    print(f"restored jobs: device iterations {it[restored].tolist()}, oracle {ito[restored].tolist()}")
    assert np.all(S9 <= 1), dict(zip(*np.unique(S9, return_counts=True)))
    assert np.all(np.isfinite(R9)) and np.all(np.isfinite(o8.cpu().numpy()))
    assert rc["resto_entries"] >= 10 and rc["resto_returns"] == rc["resto_entries"], rc
    assert same.sum() >= yard - 0.02 * same.size, (same.sum(), yard)
    d = np.abs(R9[same] - Ro[same]) / (1.0 + np.abs(Ro[same]))
    assert d.max() < 1e-6, d.max()


def test_moving_gate_failures_restored_on_device(g):
    """The 64 configs[4] get_input solves: restoration = 1 leaves no line-search failure (the round-2 solver failed
    >= 90 % of them); every device trajectory matches the oracle's KKT-certified one to 1e-5 (relative) whatever
    the iteration path, and the count that takes the oracle's iteration path exactly reaches the rounding yardstick
    minus 2 % of the solves (tests/yardstick.py).  These solves run 30-440 iterations through one or more restoration
    phases, and rounding alone moves their paths: the oracle built with FMA contraction takes its own strict build's
    path on only 42 / 64 (tools/resto_diverge.py); the device, with the oracle's float32 input semantics and mu
    sequence bit for bit since round 4, on 40 / 64 (round 3: 36), each divergence after a drift that starts at the
    rounding level (profiles/r04_resto_diverge.log)."""
    from oracle import oracle as O
    e = _engine()
    B = len(g["moving_ini"])
    it = torch.full((B,), -1, dtype=torch.int32, device=e.device)
    e.record_iters(it)
    _, x, st = e.get_input(g["moving_ini"], g["moving_goal"], g["moving_dnn_out"], u_last=g["moving_u_last"],
                           want_x=True)
    rc = e.last_resto_counters()
    e.record_iters(None)
    x, st, it = x.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()
    e.close()
    dn = g["moving_dnn_out"]
    nrm = [np.float64(np.sqrt(np.float32(sum(np.float64(np.float32(c * c)) for c in v)))) for v in dn[:, 3:6]]
    q32 = np.stack([O.rd2quat(v.astype(np.float64), n) for v, n in zip(dn[:, 3:6], nrm)])
    ref = O.solve(g["moving_ini"], g["moving_goal"], dn[:, :3].astype(np.float64), q32, dn[:, 6].astype(np.float64),
                  ulast=g["moving_u_last"])
    same = (st == ref["status"]) & (it == ref["iters"])
    yard = yardstick.solve_paths((g["moving_ini"], g["moving_goal"], dn[:, :3].astype(np.float64), q32,
                                  dn[:, 6].astype(np.float64)), dict(ulast=g["moving_u_last"]), ref)
    print(f"moving: device statuses {dict(zip(*np.unique(st, return_counts=True)))}, resto {rc}, "
          f"same path {same.sum()}/{B} (rounding yardstick: oracle FMA build {yard}/{B})")
    assert np.all(st <= 1), dict(zip(*np.unique(st, return_counts=True)))
    assert rc["resto_entries"] >= 0.5 * B and rc["resto_returns"] == rc["resto_entries"], rc
    assert same.sum() >= yard - 0.02 * B, (same.sum(), yard)
    d = np.abs(x - ref["x"]) / (1.0 + np.abs(ref["x"]))
    assert d.max() < 1e-5, d.max()
