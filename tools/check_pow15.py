"""Exact check of tools/ubench_pow15's device results: pow15 (mu^1.5), sqrt, the residual correction, x / 3 against
80-digit references; prints the mismatch counts (correct rounding expected for sqrt / division; pow15's
double-double result should be correctly rounded)."""
import sys
from decimal import Decimal, getcontext

import numpy as np

getcontext().prec = 80
raw = np.fromfile(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pow15.bin", dtype=np.float64)
n = raw.size // 5
x, out = raw[:n], raw[n:].reshape(n, 4)
bad = {"pow15": [], "sqrt": [], "div3": []}
for i in range(n):
    d = Decimal(float(x[i]))
    if out[i, 0] != float((d ** 3).sqrt()):
        bad["pow15"].append(i)
    if out[i, 1] != float(d.sqrt()):
        bad["sqrt"].append(i)
    if out[i, 3] != float(d / 3):
        bad["div3"].append(i)
print({k: len(v) for k, v in bad.items()}, "of", n)
for i in bad["pow15"][:5]:
    print("pow15", repr(float(x[i])), repr(out[i, 0]), "exact", repr(float((Decimal(float(x[i])) ** 3).sqrt())),
          "sqrt", repr(out[i, 1]), "exact", repr(float(Decimal(float(x[i])).sqrt())))
