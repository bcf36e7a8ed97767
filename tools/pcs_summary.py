"""Summarise a rocprofv3 PC-sampling CSV (tools/gpu_pcs.sh): samples per instruction / source line / stall reason.
usage: python tools/pcs_summary.py <pc_sampling.csv> [kernel-substring] > summary.txt
Prints the header, then the sample share of every source line (Instruction_Comment, from a -gline-tables-only build),
of every instruction text and of every low-cardinality column (stall reasons, issue flags) of ipm_kernel's samples."""
import csv
import sys
from collections import Counter, defaultdict

path = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else ""
rows = csv.reader(open(path, newline=""))
head = next(rows)
print("columns:", head)
col = {h: i for i, h in enumerate(head)}


def pick(*names):
    for n in names:
        for h in head:
            if h.lower() == n.lower():
                return col[h]
    for n in names:
        for h in head:
            if n.lower() in h.lower():
                return col[h]
    return None


ci = pick("Instruction")
cc = pick("Instruction_Comment", "Comment")
ck = pick("Kernel_Name", "Kernel")
co = pick("Instruction_Offset", "Code_Object_Offset", "Pc")
small = defaultdict(Counter)
by_line, by_ins, by_off, by_line_stall = Counter(), Counter(), Counter(), defaultdict(Counter)
n = 0
stall_col = pick("Stall_Reason")
for r in rows:
    if ksub and ck is not None and ksub not in r[ck]:
        continue
    n += 1
    line = r[cc] if cc is not None else ""
    ins = r[ci] if ci is not None else ""
    by_line[line] += 1
    by_ins[ins.split()[0] if ins else ""] += 1
    if co is not None:
        by_off[(r[co], ins)] += 1
    for h, i in col.items():
        if h in ("Instruction", "Instruction_Comment") or i in (co,):
            continue
        v = r[i]
        if len(small[h]) < 64 or v in small[h]:
            small[h][v] += 1
    if stall_col is not None:
        by_line_stall[line][r[stall_col]] += 1
print("samples", n)
for h, c in small.items():
    if len(c) < 40:
        print(f"\n== {h}")
        for v, m in c.most_common(20):
            print(f"  {100.0 * m / max(n, 1):6.2f} %  {v}")
print("\n== source lines (top 120)")
for v, m in by_line.most_common(120):
    extra = ""
    if stall_col is not None:
        extra = "  " + ", ".join(f"{k}:{c}" for k, c in by_line_stall[v].most_common(3))
    print(f"  {100.0 * m / max(n, 1):6.2f} %  {v}{extra}")
print("\n== opcodes (top 40)")
for v, m in by_ins.most_common(40):
    print(f"  {100.0 * m / max(n, 1):6.2f} %  {v}")
print("\n== instructions by offset (top 150)")
for (o, ins), m in by_off.most_common(150):
    print(f"  {100.0 * m / max(n, 1):6.2f} %  {o}  {ins}")
