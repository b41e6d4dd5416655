"""Per-kernel duration medians and the median gap between consecutive
dispatches from a rocprofv3 --kernel-trace database (rocpd .db):
    python tools/trace_stats.py gpurun_out/prof_x/*.db"""
import glob
import sqlite3
import statistics as st
import sys

for db in sys.argv[1:] or glob.glob("gpurun_out/*/*.db"):
    c = sqlite3.connect(db)
    t = {n.split("_0000")[0]: n for (n,) in c.execute("select name from sqlite_master where type='table'")}
    rows = list(c.execute(f"select d.start, d.end, k.kernel_name from {t['rocpd_kernel_dispatch']} d "
                          f"join {t['rocpd_info_kernel_symbol']} k on d.kernel_id = k.id order by d.start"))
    by = {}
    for s, e, n in rows:
        by.setdefault(n, []).append((e - s) / 1000)
    print(db)
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n[:90]:<90s} {len(v):6d}  median {st.median(v):9.2f} us  min {min(v):9.2f} us")
    if len(rows) > 1:
        print(f"  median gap between dispatches {st.median(rows[i + 1][0] - rows[i][1] for i in range(len(rows) - 1)) / 1000:.2f} us")
