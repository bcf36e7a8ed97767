#!/usr/bin/env python3
"""tests/golden/resto.npz: NLP instances on which the solver's filter line search fails (IPOPT would enter its
soft restoration phase, then the restoration phase).  Made without the reference (no reference code involved):

  * bench: the samples of bench.py's configs[2] batch (scenario.synthetic_batch(4096, seed=1000)) holding a
    sol_gradient job that ended in a line-search failure with the pre-restoration oracle (round 2's solver: 26
    jobs in these 18 samples); stored as sol_gradient inputs (ini, goal, gate12, dnn_out float32);
  * moving: MPC instances of the moving-gate loop (configs[4]: synthetic episodes, seed 1000, trained DNN2)
    whose get_input solve ended in a line-search failure with round 2's GPU solver, captured by
    tools/dump_moving_fail.py (gate-frame state, goal, DNN2 output float32, u_last).

    python3 tests/golden/make_resto.py gpurun_out/moving_fail_inputs.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
BENCH_SAMPLES = [245, 308, 479, 977, 984, 1169, 1202, 1228, 1487, 1936, 2127, 2347, 2362, 2377, 2450, 2517, 3377,
                 3833]

if __name__ == "__main__":
    sys.path.insert(0, REPO)
    from learningagileflight_se3_amd import scenario as S
    sb = S.synthetic_batch(4096, seed=1000)
    idx = np.array(BENCH_SAMPLES)
    m = np.load(sys.argv[1])
    np.savez_compressed(os.path.join(HERE, "resto.npz"),
                        bench_index=idx, bench_ini=sb["ini"][idx], bench_goal=sb["goal"][idx],
                        bench_gate12=sb["gate12"][idx], bench_dnn_out=sb["dnn_out"][idx],
                        moving_ini=m["ini"], moving_goal=m["goal"], moving_dnn_out=m["dnn_out"].astype(np.float32),
                        moving_u_last=m["u_last"], moving_step=m["step"], moving_episode=m["episode"])
    print("resto.npz", {k: v.shape for k, v in np.load(os.path.join(HERE, "resto.npz")).items()})
