"""CPU tests of the §8(f) host logic around the engine (no device calls):

  * imitation_pairs  == nn_train_2.py:72-84 restated as the reference's per-sample loops;
  * run_rl (reference update order) == deep_learning.py:45-83 replayed sample by sample, with a
    deterministic stand-in for sol_gradient (the GPU path is covered by tests/test_gpu_rows.py).
"""
import numpy as np
import torch

from learningagileflight_se3_amd import scenario
from learningagileflight_se3_amd.imitation import imitation_pairs
from learningagileflight_se3_amd.policy_net import Network
from learningagileflight_se3_amd.rl_loop import run_rl


def test_imitation_pairs_match_reference_loops():
    rng = np.random.default_rng(5)
    B, N = 3, 50
    samples = np.stack([scenario.nn_sample(rng) for _ in range(B)])
    out = rng.uniform(-1, 4, (B, 7)).astype(np.float32)
    x = rng.normal(0, 1, (B, N + 1, 13))
    inp, tgt = imitation_pairs(samples, out, x)
    assert inp.shape == (B * N, 18) and tgt.shape == (B * N, 7) and tgt.dtype == np.float32
    r = 0
    for k in range(B):                                   # nn_train_2.py:72-84
        for i in range(N):
            ref_in = np.zeros(18)
            ref_in[0:13] = x[k, i, :]
            ref_in[13:16] = samples[k][3:6]
            ref_in[16:18] = samples[k][7:9]
            ref_out = np.zeros(7)
            ref_out[0:6] = out[k][0:6]
            ref_out[6] = float(out[k][6]) - i * 0.10     # NumPy 1.x scalar promotion (reference env)
            assert np.array_equal(inp[r], ref_in)
            assert np.array_equal(tgt[r], torch.tensor(ref_out, dtype=torch.float).numpy())
            r += 1


def _fake_grad(samples, out):
    """Deterministic stand-in for sol_gradient: depends on the inputs and on the DNN output."""
    g = np.zeros((samples.shape[0], 8))
    g[:, 0:7] = 0.01 * np.tanh(out.astype(np.float64) + samples[:, 0:7])
    g[:, 7] = samples[:, 0] - out[:, 6]
    return g


def test_run_rl_reference_order_matches_per_sample_replay():
    epochs, batch, cores = 2, 6, 3
    torch.manual_seed(0)
    net = Network(9, 16, 16, 7)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    res = run_rl(net, opt, _fake_grad, epochs, batch, cores, "reference", np.random.default_rng(9))

    torch.manual_seed(0)
    ref = Network(9, 16, 16, 7)
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    rng = np.random.default_rng(9)
    every = np.zeros((epochs, batch))
    for ep in range(epochs):                              # deep_learning.py:41-90
        for i in range(batch // cores):
            ins = [scenario.nn_sample(rng) for _ in range(cores)]
            outs = [ref(torch.tensor(v, dtype=torch.float)).data.numpy() for v in ins]
            gra = [_fake_grad(v[None], o[None])[0] for v, o in zip(ins, outs)]
            for j in range(cores):
                o = ref(torch.tensor(ins[j], dtype=torch.float))
                loss = ref.myloss(o, torch.tensor(gra[j][0:7], dtype=torch.float))
                ropt.zero_grad()
                loss.backward()
                ropt.step()
                every[ep, j + cores * i] = gra[j][7]
    for p, q in zip(net.parameters(), ref.parameters()):
        assert torch.equal(p, q)
    assert np.array_equal(res["every_reward"], every)
    assert np.allclose(res["mean_reward"], every.mean(1), rtol=0, atol=1e-12)


def test_run_rl_batched_update_runs():
    torch.manual_seed(1)
    net = Network(9, 8, 8, 7)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    before = [p.detach().clone() for p in net.parameters()]
    res = run_rl(net, opt, _fake_grad, 1, 4, 2, "batched", np.random.default_rng(2))
    assert res["every_reward"].shape == (1, 4)
    assert any(not torch.equal(a, b) for a, b in zip(before, net.parameters()))


def test_run_rl_writes_the_reference_outputs(tmp_path):
    """deep_learning.py:91-94: Iteration, Mean_Reward{k}, Every_reward{k} after each epoch and the network
    at the end (state_dict here), reloadable with the safe loaders."""
    torch.manual_seed(2)
    net = Network(9, 8, 8, 7)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    res = run_rl(net, opt, _fake_grad, 2, 4, 2, "reference", np.random.default_rng(3), out_dir=str(tmp_path), run=3)
    assert np.array_equal(np.load(tmp_path / "Iteration.npy"), [1, 2])
    assert np.array_equal(np.load(tmp_path / "Mean_Reward3.npy"), res["mean_reward"])
    assert np.array_equal(np.load(tmp_path / "Every_reward3.npy"), res["every_reward"])
    sd = torch.load(tmp_path / "nn_deep2_3.pt", weights_only=True)
    for k, v in net.state_dict().items():
        assert torch.equal(sd[k], v)
