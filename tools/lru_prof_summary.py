"""Per-kernel summary of a rocprofv3 --kernel-trace database (the exact-LRU rounds' kernels):
calls, total and median duration."""
import glob
import sqlite3
import sys

import numpy as np

db = glob.glob(sys.argv[1] + "/*.db")[0] if not sys.argv[1].endswith(".db") else sys.argv[1]
c = sqlite3.connect(db)
rows = list(c.execute("select name, end - start from kernels"))
by = {}
for name, d in rows:
    by.setdefault(name.split("(")[0], []).append(d / 1e3)
tot = sum(sum(v) for v in by.values())
for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    v = np.array(v)
    print(f"{name[:40]:40s} {len(v):6d} {v.sum() / 1e3:9.2f} ms  p50 {np.median(v):8.1f} us  p90 {np.percentile(v, 90):8.1f} us")
print(f"total {tot / 1e3:.2f} ms")
