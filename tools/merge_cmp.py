"""Compare two merge_dump.py files: per array the fraction of elements that differ and the max |diff|."""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
worst = 0.0
for k in sorted(a.files):
    x, y = a[k], b[k]
    d = np.abs(x.astype(np.float64) - y)
    neq = np.count_nonzero((x != y) & ~(np.isnan(x) & np.isnan(y)))
    worst = max(worst, neq / x.size)
    print(f"{k:12s} differ {neq:7d} / {x.size} ({neq / x.size:.2e})  max|d| {np.nanmax(d):.3e}")
print("worst fraction", worst)
