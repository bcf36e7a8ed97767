"""GPU tests of the launch machinery around the solver (C ABI, persistent queue, sharding):

  * configs[1] at full size: B = 1024 lafse3_ocp_solve (OCSys.ocSolver, quad_OC.py:104-212) against the oracle;
  * configs[3]'s 8-GPU split on one GPU: eight contiguous 8 192-sample shards, launched one after another and
    concatenated, equal one 65 536-sample launch bit for bit (the engine's results do not depend on batch
    position or size, so this is what the 8 ranks of bench.py --gpus 8 compute between them);
  * the probe-queue guard: a sample push withheld by the debug hook is reported (LAFSE3_EDEVICE, status 7,
    NaN rewards) instead of leaving a stale out8;
  * lafse3_record_iters refuses a launch larger than its buffer; lafse3_reward scores B > slots trajectories;
  * two contexts on two streams with overlapping launches give the single-launch outputs bit for bit.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback by design)")
    from learningagileflight_se3_amd.engine import Engine
    return Engine()


def test_configs1_full_size_ocp_solve(eng):
    """configs[1]: 1024 random (start, goal, static gate) forward solves in one launch: all outputs finite,
    >= 99 % solved/acceptable, and a seeded 32-instance subset against the oracle with the A5 tolerances of
    test_ocp_solve_matches_oracle_and_is_kkt (same iteration path on >= 90 %: x/u 1e-6, cost 1e-10; all: cost
    1e-6); the subset's rows of the full launch equal the subset solved alone."""
    from learningagileflight_se3_amd import scenario as S
    from oracle import oracle as O
    sb = S.synthetic_batch(1024, seed=77)
    p = sb["dnn_out"][:, :3].astype(np.float64)
    a = sb["dnn_out"][:, 3:6].astype(np.float64)
    t = sb["dnn_out"][:, 6].astype(np.float64)
    out = eng.ocp_solve(sb["ini"], sb["goal"], p, a, t)
    torch.cuda.synchronize()
    g = {k: v.cpu().numpy() for k, v in out.items()}
    for k in ("x", "u", "lam", "cost"):
        assert np.all(np.isfinite(g[k])), k
    assert np.mean(g["status"] <= 1) >= 0.99, np.bincount(g["status"])
    idx = np.sort(np.random.default_rng(1).choice(1024, 32, replace=False))
    alone = eng.ocp_solve(sb["ini"][idx], sb["goal"][idx], p[idx], a[idx], t[idx])
    for k in ("x", "u", "lam", "cost", "iters"):
        assert np.array_equal(alone[k].cpu().numpy(), g[k][idx]), k
    q = np.stack([O.rd2quat(ai) for ai in a[idx]])
    ref = O.solve(sb["ini"][idx], sb["goal"][idx], p[idx], q, t[idx])
    ok = (g["status"][idx] <= 1) & (ref["status"] <= 1)
    same = ok & (g["iters"][idx] == ref["iters"])
    print(f"configs[1] subset: converged {ok.sum()}/32, same iteration path {same.sum()}/32")
    assert same.sum() >= 0.9 * 32
    for k in ("x", "u"):
        d = np.abs(g[k][idx][same] - ref[k][same]) / (1 + np.abs(ref[k][same]))
        assert d.max() < 1e-6, k
    assert np.max(np.abs(g["cost"][idx][same] - ref["cost"][same]) / np.abs(ref["cost"][same])) < 1e-10
    assert np.max(np.abs(g["cost"][idx][ok] - ref["cost"][ok]) / np.abs(ref["cost"][ok])) < 1e-6


def test_eight_shards_equal_one_65536_launch(eng):
    """configs[3] (65 536 samples over 8 GPUs): rank r of bench.py solves the contiguous
    shard_range(65536, r, 8).  Here the eight shards run one after another on one GPU and their out8 / rewards9 /
    status9, concatenated, equal one launch of the whole batch bit for bit."""
    from learningagileflight_se3_amd import scenario as S
    from learningagileflight_se3_amd.rl_step import shard_range
    n, world = 65536, 8
    sb = S.synthetic_batch(n, seed=1000)
    args = [torch.as_tensor(sb[k], device=eng.device) for k in ("ini", "goal", "gate12", "dnn_out")]
    eng.reserve(9 * n)
    whole = eng.sol_gradient(*args, want_rewards=True)
    parts = []
    for r in range(world):
        lo, hi = shard_range(n, r, world)
        assert hi - lo == 8192
        parts.append(eng.sol_gradient(*(x[lo:hi] for x in args), want_rewards=True))
    torch.cuda.synchronize()
    for i, name in enumerate(("out8", "rewards9", "status9")):
        cat = torch.cat([pt[i] for pt in parts]).cpu().numpy()
        w = whole[i].cpu().numpy()
        if name == "out8":
            assert np.all(np.isfinite(w))
        assert np.array_equal(cat, w), name
    st = whole[2].cpu().numpy()
    print(f"65536-sample launch: {np.mean(st <= 1):.5f} of 589824 solves solved/acceptable")
    assert np.mean(st <= 1) >= 0.99


def test_lost_probe_push_is_reported(eng):
    """ipm_kernel.hip sched_next: a claimed probe task whose sample push never lands used to be dropped
    silently.  With lafse3_debug_drop_push the push of sample 3 reserves its queue slot but
    never writes it: its eight probe slots come back NaN / status 7 (ST_DEVICE_ERR), lafse3_last_counters and
    lafse3_check_device raise, and every other sample is unaffected.  The error word survives later launches
    until lafse3_check_device has reported it, and Engine.sol_gradient checks it by default, so a NaN
    row never reaches the DNN1 update silently."""
    from learningagileflight_se3_amd import _lib
    from learningagileflight_se3_amd import scenario as S
    from learningagileflight_se3_amd.engine import Engine
    e = Engine()
    sb = S.synthetic_batch(12, seed=5)
    args = (sb["ini"], sb["goal"], sb["gate12"], sb["dnn_out"])
    ref8, refR, refS = e.sol_gradient(*args, want_rewards=True)
    e.check_device()                                  # a clean launch passes
    e.debug_drop_push(3)
    try:
        with pytest.raises(_lib.Lafse3Error, match="probe task was lost"):
            e.sol_gradient(*args, want_rewards=True)  # verify=True (default) raises
        o8, R9, S9 = e.sol_gradient(*args, want_rewards=True, verify=False)
    finally:
        e.debug_drop_push(-1)
    e.sol_gradient(*args, verify=False)                # a clean launch does not clear the word
    with pytest.raises(_lib.Lafse3Error, match="device error word"):
        e.last_counters()
    with pytest.raises(_lib.Lafse3Error, match="probe task was lost"):
        e.check_device()                              # reported: cleared
    e.check_device()
    e.last_counters()
    R9, S9, o8 = R9.cpu().numpy(), S9.cpu().numpy(), o8.cpu().numpy()
    assert np.all(S9[3, 1:] == 7) and np.all(np.isnan(R9[3, 1:]))
    assert S9[3, 0] == refS.cpu().numpy()[3, 0] and R9[3, 0] == refR.cpu().numpy()[3, 0]
    keep = np.arange(12) != 3
    assert np.array_equal(R9[keep], refR.cpu().numpy()[keep]) and np.array_equal(o8[keep], ref8.cpu().numpy()[keep])
    e.sol_gradient(*args)                             # the hook is off again: a clean launch
    e.close()


def test_reward_launch_keeps_solver_bookkeeping(eng):
    """lafse3_reward is not a solver launch: the last solve's kernel time, counters and restoration
    counts survive a scoring call on the same context."""
    from learningagileflight_se3_amd import scenario as S
    sb = S.synthetic_batch(16, seed=8)
    p = sb["dnn_out"][:, :3].astype(np.float64); a = sb["dnn_out"][:, 3:6].astype(np.float64)
    out = eng.ocp_solve(sb["ini"], sb["goal"], p, a, sb["dnn_out"][:, 6].astype(np.float64))
    ms, cnt, rc = eng.last_kernel_ms(), eng.last_counters(), eng.last_resto_counters()
    assert cnt["iterations"] > 0
    R = eng.reward(out["x"], sb["goal"], sb["gate12"])
    torch.cuda.synchronize()
    assert np.all(np.isfinite(R.cpu().numpy()))
    assert eng.last_kernel_ms() == ms and eng.last_counters() == cnt and eng.last_resto_counters() == rc


def test_record_iters_capacity_and_reward_beyond_slots(eng):
    """lafse3_record_iters stores its buffer's capacity: a launch that would write more entries fails with
    LAFSE3_EINVAL instead of writing past the buffer.  lafse3_reward runs the persistent launch, so
    B larger than the resident slots (1024) scores every trajectory."""
    from learningagileflight_se3_amd import _lib
    from learningagileflight_se3_amd import scenario as S
    from oracle import oracle as O
    sb = S.synthetic_batch(8, seed=6)
    args = (sb["ini"], sb["goal"], sb["gate12"], sb["dnn_out"])
    small = torch.zeros((4, 9), dtype=torch.int32, device=eng.device)
    eng.record_iters(small)
    try:
        with pytest.raises(_lib.Lafse3Error, match="record_iters buffer holds 36 entries"):
            eng.sol_gradient(*args)
        eng.sol_gradient(*(a[:4] for a in args))     # 4 samples = 36 entries: fits
        torch.cuda.synchronize()
        assert np.all(small.cpu().numpy() > 0)
    finally:
        eng.record_iters(None)
    # trajectories: the eight optima of this batch, tiled past the slot count
    p = sb["dnn_out"][:, :3].astype(np.float64)
    a = sb["dnn_out"][:, 3:6].astype(np.float64)
    x = eng.ocp_solve(sb["ini"], sb["goal"], p, a, sb["dnn_out"][:, 6].astype(np.float64))["x"].cpu().numpy()
    B = 1100
    rep = np.arange(B) % 8
    R = eng.reward(x[rep], sb["goal"][rep], sb["gate12"][rep]).cpu().numpy()
    rR, _ = O.reward(x, sb["goal"], sb["gate12"])
    assert np.all(np.isfinite(R)) and np.max(np.abs(R - rR[rep])) < 1e-9


def test_two_launches_in_flight_equal_single_launches(eng):
    """Two solver contexts on two HIP streams with their persistent launches overlapping (bench.py
    ocp_solve_per_s_2streams: the second launch's workgroups take the SIMDs the first one's finished instances
    free): every output equals the same batch solved alone on one context, bit for bit, and a different batch on
    the other stream is unaffected."""
    from learningagileflight_se3_amd import scenario as S
    from learningagileflight_se3_amd.engine import Engine

    def batch(seed):
        sb = S.synthetic_batch(1024, seed=seed)
        return [torch.as_tensor(sb["ini"], device="cuda"), torch.as_tensor(sb["goal"], device="cuda"),
                torch.as_tensor(sb["dnn_out"][:, :3].astype(np.float64), device="cuda"),
                torch.as_tensor(sb["dnn_out"][:, 3:6].astype(np.float64), device="cuda"),
                torch.as_tensor(sb["dnn_out"][:, 6].astype(np.float64), device="cuda")]
    a, b = batch(77), batch(78)
    ref_a, ref_b = eng.ocp_solve(*a), eng.ocp_solve(*b)
    torch.cuda.synchronize()
    e2 = Engine()
    try:
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        outs = []
        for i in range(4):
            with torch.cuda.stream(s1 if i % 2 == 0 else s2):
                outs.append((eng if i % 2 == 0 else e2).ocp_solve(*(a if i % 2 == 0 else b)))
        torch.cuda.synchronize()
    finally:
        e2.close()
    for i, o in enumerate(outs):
        ref = ref_a if i % 2 == 0 else ref_b
        for k in ("x", "u", "lam", "cost", "status", "iters"):
            assert torch.equal(o[k], ref[k]), (i, k)
