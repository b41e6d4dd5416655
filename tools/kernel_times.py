"""Median duration (us) per kernel name from a rocprofv3 rocpd database, in
dispatch order groups: tools/kernel_times.py DB [GROUPS]"""
import sqlite3
import sys

import numpy as np

db = sys.argv[1]
rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
if len(sys.argv) > 3 and sys.argv[2] == "--last":
    # the last N dispatches in order, one line each
    for nm, s, e in rows[-int(sys.argv[3]):]:
        print(f"{nm.split('(')[0][-40:]:40s} {(e - s) / 1e3:9.1f}")
    sys.exit(0)
groups = int(sys.argv[2]) if len(sys.argv) > 2 else 1
names = sorted({r[0] for r in rows})
for nm in names:
    d = [(r[2] - r[1]) / 1e3 for r in rows if r[0] == nm]
    k = max(1, len(d) // groups)
    print(f"{nm[:40]:40s} n={len(d):5d} " + " ".join(f"{np.median(d[i * k:(i + 1) * k]):8.1f}" for i in range(groups)))
