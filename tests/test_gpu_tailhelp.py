"""Tail help (csrc/tailhelp.inc, params.tail_help): once a launch's queue is drained, idle waves factorise the next
inertia-correction trials (IPOPT's PDPerturbationHandler sequence, quad_OC.py:170-174 defaults) of the instances still
running, and an owner skips a trial a helper has already found to have the wrong inertia.  The helpers run the same
table build and factorisation on bit-identical inputs, so every output must equal the tail_help = 0 launch bit for
bit; the help counters show the path ran (requests posted, trials skipped).

  * configs[1] forward solves (lafse3_ocp_solve, B = 1 024, quad_OC.py:104-212): x, u, lam, cost, status, iters and
    the iteration / sweep totals;
  * sol_gradient FD (quad_policy.py:94-112) on the bench scenario (B = 512, 4 608 solves): out8, rewards9, status9;
  * IFT mode (B = 512): out8, rewards9, status9.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _engines():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback by design)")
    from learningagileflight_se3_amd import _lib
    from learningagileflight_se3_amd.engine import Engine
    on, off = Engine(), Engine()
    on.set_params(_lib.default_params(tail_help=1))
    off.set_params(_lib.default_params(tail_help=0))
    return on, off


@pytest.fixture(scope="module")
def engs():
    on, off = _engines()
    yield on, off
    on.close()
    off.close()


def _solve_batch(seed, B):
    from learningagileflight_se3_amd import scenario as S
    sb = S.synthetic_batch(B, seed=seed)
    return [torch.as_tensor(sb["ini"], device="cuda"), torch.as_tensor(sb["goal"], device="cuda"),
            torch.as_tensor(sb["dnn_out"][:, :3].astype(np.float64), device="cuda"),
            torch.as_tensor(sb["dnn_out"][:, 3:6].astype(np.float64), device="cuda"),
            torch.as_tensor(sb["dnn_out"][:, 6].astype(np.float64), device="cuda")]


def test_tail_help_ocp_solve_bit_equal(engs):
    on, off = engs
    a = _solve_batch(77, 1024)
    ref = off.ocp_solve(*a)
    torch.cuda.synchronize()
    c_off = off.last_counters()
    h_off = off.last_help_counters()
    out = on.ocp_solve(*a)
    torch.cuda.synchronize()
    c_on = on.last_counters()
    h_on = on.last_help_counters()
    print(f"configs[1] B=1024: kernel {off.last_kernel_ms():.2f} ms without tail help, {on.last_kernel_ms():.2f} ms "
          f"with; help {h_on}")
    for k in ("x", "u", "lam", "cost", "status", "iters"):
        assert torch.equal(out[k], ref[k]), k
    assert c_on == c_off
    assert all(v == 0 for v in h_off.values())
    assert h_on["requests"] > 0 and h_on["skipped"] > 0


def _grad_batch(B, seed=1000):
    from learningagileflight_se3_amd import scenario as S
    sb = S.synthetic_batch(B, seed=seed)
    return [torch.as_tensor(sb[k], device="cuda") for k in ("ini", "goal", "gate12", "dnn_out")]


@pytest.mark.parametrize("grad_mode", [0, 1])
def test_tail_help_sol_gradient_bit_equal(engs, grad_mode):
    on, off = engs
    g = _grad_batch(512)
    ref = off.sol_gradient(*g, want_rewards=True, grad_mode=grad_mode)
    torch.cuda.synchronize()
    out = on.sol_gradient(*g, want_rewards=True, grad_mode=grad_mode)
    torch.cuda.synchronize()
    h = on.last_help_counters()
    print(f"sol_gradient grad_mode={grad_mode} B=512: kernel {off.last_kernel_ms():.2f} ms without tail help, "
          f"{on.last_kernel_ms():.2f} ms with; help {h}")
    for a, b, name in zip(out, ref, ("out8", "rewards9", "status9")):
        assert torch.equal(a, b), name
    assert h["requests"] > 0


def test_tail_help_two_rounds_repeatable(engs):
    """The same launch twice with tail help: identical outputs (which helper serves which trial differs run to
    run; the results may not)."""
    on, _ = engs
    a = _solve_batch(91, 512)
    r1 = on.ocp_solve(*a)
    torch.cuda.synchronize()
    r2 = on.ocp_solve(*a)
    torch.cuda.synchronize()
    for k in ("x", "u", "lam", "cost", "status", "iters"):
        assert torch.equal(r1[k], r2[k]), k
