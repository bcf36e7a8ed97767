"""Cut a rocprofv3 kernel trace of tools/gpu_moving_trace.py into its runs (at the cumsum marker kernels) and compare
them: per run the span, ipm_kernel / traversal_time_kernel / torch-kernel durations, and per HIP stream (group) and
per hardware queue the busy time and the gaps between consecutive kernels.

    python3 tools/trace_moving.py run_kernel_trace.csv [--dump out.csv]
"""
import csv
import sys
from collections import defaultdict

import numpy as np

path = sys.argv[1]
rows = []
with open(path, newline="") as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     r.get("Stream_Id", "?"), r.get("Queue_Id", "?")))
rows.sort()
cuts = [i for i, r in enumerate(rows) if "scan" in r[2].lower() or "cumsum" in r[2].lower()]
print(f"{len(rows)} kernels, {len(cuts)} markers")


def kind(name):
    if "ipm_kernel" in name:
        return "ipm"
    if "traversal_time" in name:
        return "tt"
    if "u0_gather" in name:
        return "u0"
    return "torch"


keep = []
for n, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
    seg = rows[a + 1:b]
    if not seg:
        continue
    t0, t1 = seg[0][0], max(r[1] for r in seg)
    print(f"\n== run {n}: {len(seg)} kernels, span {(t1 - t0) / 1e9:.3f} s")
    by = defaultdict(list)
    for s, e, nm, st, q in seg:
        by[kind(nm)].append(e - s)
    for k in ("ipm", "tt", "u0", "torch"):
        v = np.array(by.get(k, [0]), dtype=np.float64)
        print(f"   {k:6s} n {len(by.get(k, [])):7d}  sum {v.sum() / 1e9:8.3f} s  mean {v.mean() / 1e3:10.1f} us  "
              f"p50 {np.median(v) / 1e3:10.1f} us  max {v.max() / 1e3:10.1f} us")
    for key, idx in (("stream", 3), ("queue", 4)):
        grp = defaultdict(list)
        for r in seg:
            grp[r[idx]].append(r)
        for g, rs in sorted(grp.items()):
            busy = sum(e - s for s, e, *_ in rs)
            gaps = np.array([rs[i + 1][0] - rs[i][1] for i in range(len(rs) - 1)], dtype=np.float64)
            ipm = [r for r in rs if kind(r[2]) == "ipm"]
            print(f"   {key} {g:>4s}: {len(rs):7d} kernels ({len(ipm)} ipm), busy {busy / 1e9:7.3f} s, "
                  f"gaps sum {gaps.clip(min=0).sum() / 1e9:7.3f} s  p50 {np.median(gaps) / 1e3 if len(gaps) else 0:8.1f} us"
                  f"  overlap(neg gaps) {(-gaps.clip(max=0)).sum() / 1e9:7.3f} s")
    # concurrency of the two groups' ipm kernels: time with >= 2 ipm kernels in flight
    ev = []
    for s, e, nm, st, q in seg:
        if kind(nm) == "ipm":
            ev += [(s, 1), (e, -1)]
    ev.sort()
    cur, last, both, any_ = 0, None, 0, 0
    for t, d in ev:
        if last is not None:
            if cur >= 2:
                both += t - last
            if cur >= 1:
                any_ += t - last
        cur += d
        last = t
    print(f"   ipm in flight: any {any_ / 1e9:.3f} s, two at once {both / 1e9:.3f} s")
    keep += [r for r in seg if kind(r[2]) != "torch"]
if "--dump" in sys.argv:
    out = sys.argv[sys.argv.index("--dump") + 1]
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["start", "end", "kernel", "stream", "queue"])
        for r in keep:
            w.writerow([r[0], r[1], r[2][:60], r[3], r[4]])
