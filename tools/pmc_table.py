"""Per-kernel mean of every PMC counter in a rocprofv3 rocpd database:
tools/pmc_table.py DB"""
import re
import sqlite3
import sys
from collections import defaultdict

con = sqlite3.connect(sys.argv[1])
acc = defaultdict(lambda: defaultdict(list))
for name, cn, val in con.execute("select kernel_name, counter_name, value from counters_collection"):
    m = re.search(r"(k_\w+)", name)
    acc[m.group(1) if m else name[:30]][cn].append(float(val))
cnames = sorted({c for k in acc.values() for c in k})
print(f"{'kernel':<22}" + "".join(f"{c[-22:]:>24}" for c in cnames))
for k, d in sorted(acc.items()):
    print(f"{k:<22}" + "".join(f"{(sum(d[c]) / len(d[c]) if d[c] else 0):>24.4g}" for c in cnames))
