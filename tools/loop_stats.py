"""Instruction mix of the loops of one function in a hipcc -S listing (the factorisation stage loop and friends).
usage: python tools/loop_stats.py <asm.s> [function-substring] [must-contain]"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().split("\n")
fsub = sys.argv[2] if len(sys.argv) > 2 else "linear_solve"
must = sys.argv[3] if len(sys.argv) > 3 else "v_mfma"
a = next(i for i, l in enumerate(src) if re.match(r"^_ZN6lafse3\w*" + fsub + r"\w*:", l))
b = next(i for i in range(a, len(src)) if src[i].strip().startswith(".size"))
body = src[a:b]
labels = {l.split(":")[0]: j for j, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
for j, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", l)
    if not m:
        continue
    t = m.group(1) or m.group(2)
    if t not in labels or labels[t] >= j:
        continue
    lo = body[labels[t]:j + 1]
    if not any(must in x for x in lo):
        continue
    ins = [x.split()[0] for x in lo if x.startswith("\t") and not x.startswith("\t.") and not x.startswith("\t;") and x.split()]
    c = Counter()
    for op in ins:
        k = ("mfma" if "mfma" in op else "f64" if op.endswith("_f64") else "ds_read" if op.startswith("ds_read")
             else "ds_write" if op.startswith("ds_write") else "vmem_load" if re.match(r"(global|buffer)_load", op)
             else "vmem_store" if re.match(r"(global|buffer)_store", op) else "waitcnt" if op == "s_waitcnt"
             else "nop" if op == "s_nop" else "readlane" if "readlane" in op else "permlane" if "permlane" in op
             else "scratch" if op.startswith("scratch") else "salu" if op.startswith("s_") else "valu")
        c[k] += 1
    print(f"loop {t} lines {labels[t]}..{j}: {len(ins)} instructions", dict(sorted(c.items(), key=lambda kv: -kv[1])))
