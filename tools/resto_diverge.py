"""Where do device and oracle part ways on the restoration fixtures?

  python tools/resto_diverge.py device   (GPU box) per-iteration IPM traces (lafse3_debug_trace, 16 doubles per
                                         iteration: mu e0 th0 ph0 gBD amax az alpha dw accepted nfilt sweeps r0 r1 J lb) of
                                         the tests/golden/resto.npz jobs -> gpurun_out/resto_trace_gpu.npz:
                                           bench  : the 18 samples x 9 probes of sol_gradient, restoration on
                                           bench0 : the same, restoration = 0 (the line-search failures of :54)
                                           moving : the 64 configs[4] get_input solves
  python tools/resto_diverge.py host     (here) the oracle's traces of the same jobs (oracle/: the checker) and, per job
                                         whose status or iteration count differs, the first iteration whose decision
                                         (accepted, delta_w, filter size, mu, restoration gap) differs, with the
                                         largest relative difference of e0 / theta / phi on the iterations before it
                                         -> stdout and gpurun_out/resto_diverge.json

Restoration-phase iterations are not traced (both sides skip their indices), so a job whose restoration phases run
for different lengths shows up as a "gap" divergence at the first index one side skipped."""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
TI = 700   # traced iterations per job (the fixtures' longest solve is < 450)
FIELDS = ["mu", "e0", "th0", "ph0", "gBD", "amax", "az", "alpha", "dw", "accepted", "nfilt", "sweeps"]
OUT = os.path.join(REPO, "gpurun_out")


def fixture():
    return dict(np.load(os.path.join(REPO, "tests", "golden", "resto.npz")))


def device():
    import torch
    from learningagileflight_se3_amd import _lib
    from learningagileflight_se3_amd.engine import Engine
    g = fixture()
    res = {}
    bench = (g["bench_ini"], g["bench_goal"], g["bench_gate12"], g["bench_dnn_out"])
    B = len(g["bench_ini"])
    for tag, resto in (("bench", 1), ("bench0", 0)):
        e = Engine()
        e.set_params(_lib.default_params(restoration=resto))
        it = torch.full((B, 9), -1, dtype=torch.int32, device=e.device)
        tr = torch.zeros((9 * B, TI, 16), dtype=torch.float64, device=e.device)   # instance = probe * B + sample
        e.record_iters(it)
        e.debug_trace(tr, TI)
        _, R9, S9 = e.sol_gradient(*bench, want_rewards=True)
        torch.cuda.synchronize()
        e.debug_trace(None)
        e.record_iters(None)
        res[tag + "_status"] = S9.cpu().numpy()
        res[tag + "_iters"] = it.cpu().numpy()
        res[tag + "_R9"] = R9.cpu().numpy()
        res[tag + "_trace"] = tr.cpu().numpy().reshape(9, B, TI, 16).transpose(1, 0, 2, 3)   # (sample, probe, ...)
        e.close()
    Bm = len(g["moving_ini"])
    e = Engine()
    it = torch.full((Bm,), -1, dtype=torch.int32, device=e.device)
    tr = torch.zeros((Bm, TI, 16), dtype=torch.float64, device=e.device)
    e.record_iters(it)
    e.debug_trace(tr, TI)
    _, x, st = e.get_input(g["moving_ini"], g["moving_goal"], g["moving_dnn_out"], u_last=g["moving_u_last"],
                           want_x=True)
    torch.cuda.synchronize()
    e.debug_trace(None)
    e.record_iters(None)
    res.update(moving_status=st.cpu().numpy(), moving_iters=it.cpu().numpy(), moving_x=x.cpu().numpy(),
               moving_trace=tr.cpu().numpy())
    e.close()
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, "resto_trace_gpu.npz"), **res)
    print({k: v.shape for k, v in res.items()}, flush=True)


def oracle_traces(g, fast=False):
    """The oracle's traces of the same jobs, solve by solve (orc_solve_q with the debug trace armed).  fast=True: the
    oracle's -O3 FMA-contracted build (same algorithm, other rounding) -- the baseline for how often rounding alone
    changes an iteration path on these instances."""
    from oracle import oracle as O
    L = O.lib(fast)

    def arm(buf, n):
        L.orc_debug_trace(None if buf is None else buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), n)
    out = {}
    dn = g["bench_dnn_out"]
    pp, qq, tt, uu = O.grad_params(dn)
    B = len(dn)
    for tag, resto in (("bench", 1), ("bench0", 0)):
        prm = O.default_params(restoration=resto)
        tr = np.zeros((B, 9, TI, 16))
        st = np.zeros((B, 9), np.int32)
        its = np.zeros((B, 9), np.int32)
        for j in range(9):
            buf = np.zeros((B, TI, 16))
            arm(buf, TI)
            # the bench fixture's sol_gradient has no u_last: probes 1-6 see a zero one (orc_sol_gradient)
            r = O.solve(g["bench_ini"], g["bench_goal"], pp[:, j], qq[:, j], tt[:, j], params=prm, fast=fast)
            arm(None, 0)
            tr[:, j] = buf
            st[:, j] = r["status"]
            its[:, j] = r["iters"]
        out[tag] = (tr, st, its)
    nrm = [np.float64(np.sqrt(np.float32(sum(np.float64(np.float32(c * c)) for c in v))))
           for v in g["moving_dnn_out"][:, 3:6]]
    q32 = np.stack([O.rd2quat(v.astype(np.float64), n) for v, n in zip(g["moving_dnn_out"][:, 3:6], nrm)])
    Bm = len(q32)
    buf = np.zeros((Bm, TI, 16))
    arm(buf, TI)
    dm = g["moving_dnn_out"]
    r = O.solve(g["moving_ini"], g["moving_goal"], dm[:, :3].astype(np.float64), q32, dm[:, 6].astype(np.float64),
                ulast=g["moving_u_last"], fast=fast)
    arm(None, 0)
    out["moving"] = (buf, r["status"], r["iters"])
    return out


def first_divergence(td, to, nd, no):
    """First traced iteration whose decision differs; the largest relative e0/th0/ph0 gap on the iterations before."""
    n = min(max(nd, no) + 1, TI)
    worst, drift = 0.0, None   # drift: first iteration whose e0 / theta / phi differ by more than 1e-9 (relative)
    for k in range(n):
        a, b = td[k], to[k]
        gap_d, gap_o = not a.any(), not b.any()
        if gap_d != gap_o:
            return {"it": k, "what": "restoration gap (device %s, oracle %s)" % ("skips" if gap_d else "traces",
                                                                               "skips" if gap_o else "traces"),
                    "prior_rel": worst}
        if gap_d:
            continue
        # the line search's decision: the number of backtracking halvings of alpha_max (not the drift of alpha_max)
        hd, ho = (int(round(np.log2(v[5] / v[7]))) if v[7] > 0 and v[5] > 0 else -1 for v in (a, b))
        for name, dv, ov in (("accepted", a[9], b[9]), ("dw", a[8], b[8]), ("nfilt", a[10], b[10]), ("mu", a[0], b[0]),
                             ("halvings", hd, ho)):
            if dv != ov:
                return {"it": k, "what": name, "device": float(dv), "oracle": float(ov), "prior_rel": worst,
                        "drift_it": drift,
                        "e0": [float(a[1]), float(b[1])], "th0": [float(a[2]), float(b[2])],
                        "ph0": [float(a[3]), float(b[3])], "alpha": [float(a[7]), float(b[7])]}
        rel = np.abs(a[1:4] - b[1:4]) / np.maximum(np.abs(b[1:4]), 1e-6)   # (theta ~ 1e-14 at a feasible point)
        worst = max(worst, float(rel.max()))
        if drift is None and rel.max() > 1e-9:
            drift = k
    return {"it": None, "what": "no decision differs in the traced iterations", "prior_rel": worst, "drift_it": drift}


def host():
    g = fixture()
    d = dict(np.load(os.path.join(OUT, "resto_trace_gpu.npz")))
    o = oracle_traces(g)
    of = oracle_traces(g, fast=True)
    report = {}
    for tag in ("bench", "bench0", "moving"):
        to, so, io = o[tag]
        td, sd, idv = d[tag + "_trace"], d[tag + "_status"], d[tag + "_iters"]
        jobs = list(zip(*np.nonzero((sd != so) | (idv != io))))
        rows = []
        for jb in jobs:
            fd = first_divergence(td[jb], to[jb], int(idv[jb]), int(io[jb]))
            fd.update(job=[int(v) for v in jb], status=[int(sd[jb]), int(so[jb])], iters=[int(idv[jb]), int(io[jb])])
            rows.append(fd)
        same = int(((sd == so) & (idv == io)).sum())
        _, sf, itf = of[tag]
        same_f = int(((sf == so) & (itf == io)).sum())
        print(f"{tag}: device same path {same}/{sd.size}; diverging {len(rows)}; baseline: the oracle's FMA build "
              f"{same_f}/{sd.size}" + (f"; line-search failures oracle {(so == 3).sum()}, device {(sd == 3).sum()} "
                                       f"(both {((so == 3) & (sd == 3)).sum()}), FMA build {(sf == 3).sum()} (both "
                                       f"{((so == 3) & (sf == 3)).sum()})" if tag == "bench0" else ""), flush=True)
        for r in rows:
            print("  ", json.dumps(r), flush=True)
        report[tag] = {"same": same, "same_oracle_fma_build": same_f, "n": int(sd.size), "diverging": rows}
    json.dump(report, open(os.path.join(OUT, "resto_diverge.json"), "w"), indent=1)


if __name__ == "__main__":
    {"device": device, "host": host}[sys.argv[1]]()
