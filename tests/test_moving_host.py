"""CPU parity of the moving-gate receding-horizon host logic (learningagileflight_se3_amd/moving_gate.py)
against tests/golden/moving.npz, made by the reference's own gate / quad_moving.solver / run_quad code
(tests/golden/make_golden.py gen_moving; the NLP solves there are the oracle's)."""
import numpy as np
import pytest
import torch

from learningagileflight_se3_amd import moving_gate as MG
from learningagileflight_se3_amd import scenario
from learningagileflight_se3_amd.policy_net import Network

V0, W0 = np.array([1.0, 0.3, 0.4]), np.pi / 2


def dnn2_from_fixture(g):
    net = Network(18, 128, 128, 7)
    sd = {k: torch.as_tensor(g[k.replace(".", "_")]) for k in net.state_dict()}
    net.load_state_dict(sd)
    return net


def per_sample(net):
    """DNN2 evaluated one sample at a time in float32 on the CPU, as quad_nn.network.forward is called."""
    def f(inp):
        with torch.no_grad():
            return np.stack([net(torch.tensor(r, dtype=torch.float)).numpy() for r in np.atleast_2d(inp)])
    return f


def episode_noise(s):
    """np.random.seed(500 + s); nn_sample(); gate.move(...) draw order of make_golden.gen_moving."""
    rs = np.random.RandomState(500 + s)
    sample = scenario.nn_sample(rs)
    return sample, MG.move_noise(rs, 500)


@pytest.fixture(scope="module")
def g(golden):
    return golden("moving")


def test_samples_and_gate_motion_match_reference(g):
    for s in range(g["inputs"].shape[0]):
        sample, noise = episode_noise(s)
        assert np.array_equal(sample, g["inputs"][s])
        gp0, _ = MG.initial_episodes(sample[None])
        gm, V = MG.move(gp0, V0, W0, noise[None])
        assert np.max(np.abs(gm[0] - g["gate_move"][s])) < 1e-12
        assert np.max(np.abs(V[0] - g["V"][s])) < 1e-15


def test_plant_step_matches_reference_dyn_fn(g):
    x, u = g["states"][:, :-1].reshape(-1, 13), g["controls"].reshape(-1, 4)
    xn = MG.plant_step(x, u)
    assert np.max(np.abs(xn - g["states"][:, 1:].reshape(-1, 13))) < 1e-12


def test_traversal_time_solver_and_dnn2_inputs_match_reference(g):
    net = dnn2_from_fixture(g)
    f = per_sample(net)
    n_ep, steps = g["t"].shape
    for s in range(n_ep):
        final = g["inputs"][s, 3:6][None]
        for i in range(steps):
            st = g["states"][s, i][None]
            t, it = MG.solve_t(f, st, final, g["gate_move"][s, i][None], g["V"][s, i][None], W0)
            assert abs(t[0] - g["t"][s, i]) < 1e-9, (s, i, t, g["t"][s, i])
            if i % MG.CTRL_EVERY == 0:
                gn = MG.rotate_y(MG.translate(g["gate_move"][s, i][None], g["V"][s, i][None] * g["t"][s, i]),
                                 np.array([W0 * g["t"][s, i]]))
                inp = MG.dnn2_inputs(gn, st, final)
                assert np.max(np.abs(inp[0] - g["ins18"][s, i // MG.CTRL_EVERY])) < 1e-10
                out = f(g["ins18"][s, i // MG.CTRL_EVERY])
                assert np.array_equal(out[0], g["outs"][s, i // MG.CTRL_EVERY])
