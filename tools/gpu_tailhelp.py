"""Tail help anatomy (csrc/tailhelp.inc): configs[1] (B = 1 024, seed 77) and the IFT bench batch with tail_help 0
and 1 — kernel time, help counters (owner cycles posting / waiting / copying), and from the placement record
(Engine.debug_timers: start / end in 100 MHz ticks, iterations, sweeps per instance) the longest instances and the
launch's concurrency over time.  -> stdout (gpurun_out/tailhelp.log)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from learningagileflight_se3_amd import _lib  # noqa: E402
from learningagileflight_se3_amd import scenario as S  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402

dev = torch.device("cuda", 0)


def solve_args(B, seed):
    sb = S.synthetic_batch(B, seed=seed)
    return [torch.as_tensor(sb["ini"], device=dev), torch.as_tensor(sb["goal"], device=dev),
            torch.as_tensor(sb["dnn_out"][:, :3].astype(np.float64), device=dev),
            torch.as_tensor(sb["dnn_out"][:, 3:6].astype(np.float64), device=dev),
            torch.as_tensor(sb["dnn_out"][:, 6].astype(np.float64), device=dev)]


def run(th, kind, reps=3):
    e = Engine()
    e.set_params(_lib.default_params(tail_help=th))
    if kind == "ocp":
        a = solve_args(1024, 77)
        n = 1024
        call = lambda: e.ocp_solve(*a)  # noqa: E731
    else:
        sb = S.synthetic_batch(4096, seed=1000)
        g = [torch.as_tensor(sb[k], device=dev) for k in ("ini", "goal", "gate12", "dnn_out")]
        n = 3 * 4096
        e.set_params(_lib.default_params(tail_help=th, grad_mode=1))
        call = lambda: e.sol_gradient(*g)  # noqa: E731
    call()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        call()
        torch.cuda.synchronize()
        ms.append(e.last_kernel_ms())
    buf = torch.zeros((n, 32), dtype=torch.int64, device=dev)
    e.debug_timers(buf)
    call()
    torch.cuda.synchronize()
    e.debug_timers(None)
    h = e.last_help_counters()
    T = buf.cpu().numpy()
    e.close()
    t0 = T[:, 16].min()
    st, en = (T[:, 16] - t0) / 1e5, (T[:, 17] - t0) / 1e5   # ms
    it, sw = T[:, 20], T[:, 21]
    print(f"{kind} tail_help={th}: kernel ms {[round(m, 2) for m in ms]}; help {h}", flush=True)
    if h["requests"]:
        print(f"   per request: post {h['post_cycles'] / h['requests']:.0f} cycles; waits "
              f"{h['wait_cycles'] / max(1, h['adopted'] + h['skipped']):.0f} cycles per answered trial; copy "
              f"{h['copy_cycles'] / max(1, h['adopted']):.0f} cycles per adoption", flush=True)
    order = np.argsort(-(en - st))[:6]
    for i in order:
        print(f"   instance {i}: start {st[i]:.2f} end {en[i]:.2f} ms, {it[i]} iterations, {sw[i]} sweeps "
              f"({sw[i] / max(it[i], 1):.2f}/it, {(en[i] - st[i]) / max(it[i], 1) * 1e3:.0f} us/it)", flush=True)
    span = en.max()
    for f in (0.25, 0.5, 0.75, 0.9, 1.0):
        t = f * span
        print(f"   at {t:.1f} ms: {int(((st <= t) & (en > t)).sum())} instances running", flush=True)
    return T


for kind in ("ocp", "ift"):
    for th in (0, 1):
        run(th, kind)
