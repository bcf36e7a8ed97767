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


def fixture_episodes(g):
    """(samples, noise) of moving.npz's episodes: episode 0 runs last_inputs.npy's scenario (source 0), the
    others nn_sample (source 1); the gate.move noise follows the same draw order for both."""
    samples, noise = [], []
    for s in range(g["inputs"].shape[0]):
        smp, nz = episode_noise(s)
        samples.append(g["inputs"][s] if g["source"][s] == 0 else smp)
        noise.append(nz)
    return np.stack(samples), np.stack(noise)


def test_dnn2_fixture_is_the_trained_network(golden):
    """dnn2_nn3_1.npz (raw float32 storages of nn3_1.pth) has DNN2's shapes and drives moving.npz; on the
    fixture's DNN2 inputs it predicts traversal times in the trained range (0 < t < 5 s), which a
    random-init network does not."""
    w, g = golden("dnn2_nn3_1"), golden("moving")
    shapes = {"l1_weight": (128, 18), "l1_bias": (128,), "l2_weight": (128, 128), "l2_bias": (128,),
              "l3_weight": (7, 128), "l3_bias": (7,)}
    for k, sh in shapes.items():
        assert w[k].shape == sh and w[k].dtype == np.float32 and np.all(np.isfinite(w[k]))
        assert np.array_equal(w[k], g[k])
    out = per_sample(dnn2_from_fixture(g))(g["ins18"].reshape(-1, 18))
    assert np.array_equal(out, g["outs"].reshape(-1, 7))
    assert np.all((out[:, 6] > 0) & (out[:, 6] < 5))


@pytest.fixture(scope="module", params=["moving", "moving500"])
def g(golden, request):
    """moving.npz (2 episodes x 120 plant steps) and moving500.npz (episode 0 at main.py's full 500 steps)."""
    return golden(request.param)


def test_samples_and_gate_motion_match_reference(g, golden):
    assert g["source"][0] == 0 and np.array_equal(g["inputs"][0], golden("last_inputs")["inputs"])
    for s in range(g["inputs"].shape[0]):
        sample, noise = episode_noise(s)
        if g["source"][s] == 1:
            assert np.array_equal(sample, g["inputs"][s])
        sample = g["inputs"][s]
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


def test_device_kinematics_match_host_restatement():
    """The torch (device-path) kinematics equal the numpy/scipy host path on gate-shaped frames
    (run here on the CPU device: same float64 arithmetic, scipy's quaternion conventions)."""
    rng = np.random.default_rng(0)
    n = 2000
    gp = scenario.gate_corners(rng.uniform(0.5, 1.25, n), rng.uniform(-1.5, 1.5, n)).reshape(-1, 4, 3)
    gp = MG.rotate_y(gp + rng.normal(0, 3, (n, 1, 3)), rng.uniform(-3, 3, n))
    st, fin, u = rng.normal(size=(n, 13)), rng.normal(size=(n, 3)), rng.uniform(0, 2.44, (n, 4))
    T = torch.as_tensor
    assert np.max(np.abs(MG.dnn2_inputs(gp, st, fin) - MG.dnn2_inputs_t(T(gp), T(st), T(fin)).numpy())) < 1e-14
    ang = rng.uniform(-3, 3, n)
    assert np.max(np.abs(MG.rotate_y(gp, ang) - MG.rotate_y_t(T(gp), T(ang)).numpy())) < 1e-14
    assert np.array_equal(MG.plant_step(st, u), MG.plant_step_t(T(st), T(u)).numpy())
    net = Network(18, 32, 32, 7).double()
    f = lambda x: net(torch.as_tensor(x)).detach().numpy()
    t_host, _ = MG.solve_t(f, st[:64], fin[:64], gp[:64], rng.normal(size=(64, 3)) * 0 + 0.3, W0)
    t_dev = MG.solve_t_t(lambda x: net(x.double()).float(), T(st[:64]), T(fin[:64]), T(gp[:64]),
                         T(np.full((64, 3), 0.3)), W0)
    assert np.max(np.abs(t_host - t_dev.numpy())) < 1e-6
