"""Per-function scratch (spill) traffic of the ipm kernel build: where the spills sit relative to loops.
usage: python tools/spills.py <asm.s>"""
import re, sys
src = open(sys.argv[1]).read().split("\n")
funcs = {}
cur = None
for i, l in enumerate(src):
    m = re.match(r"^(_ZN6lafse3[0-9A-Za-z_]+):", l)
    if m:
        cur = m.group(1); funcs[cur] = [i, None]
    if cur and l.strip().startswith(".size") and cur in l:
        funcs[cur][1] = i; cur = None
for f, (a, b) in funcs.items():
    if b is None or "lane" in f:
        continue
    body = src[a:b]
    # loop bodies: between a label and a backward branch to it
    labels = {l.split(":")[0]: j for j, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
    loops = []
    for j, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", l)
        if m:
            t = m.group(1) or m.group(2)
            if t in labels and labels[t] < j:
                loops.append((labels[t], j))
    inloop = 0
    for j, l in enumerate(body):
        if "scratch_" in l and any(s <= j <= e for s, e in loops):
            inloop += 1
    tot = sum("scratch_" in l for l in body)
    name = re.sub(r"_ZN6lafse3\d+", "", f)[:40]
    print(f"{name:42s} scratch ops {tot:5d}  inside loops {inloop:5d}  loops {len(loops)}")
