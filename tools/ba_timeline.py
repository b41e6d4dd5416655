"""Local BA call timeline from a rocprofv3 --kernel-trace database (rocpd .db):
per call (a call starts at its k_ba_edges dispatch) the span, the kernel busy
time, the idle time between dispatches, the busy time per kernel and the
largest gaps with the kernel before them.
    python tools/ba_timeline.py gpurun_out/r6o_ba/*.db"""
import glob
import sqlite3
import sys

for db in sys.argv[1:] or glob.glob("gpurun_out/*/*.db"):
    c = sqlite3.connect(db)
    t = {n.split("_0000")[0]: n for (n,) in c.execute("select name from sqlite_master where type='table'")}
    rows = list(c.execute(f"select d.start, d.end, k.kernel_name from {t['rocpd_kernel_dispatch']} d "
                          f"join {t['rocpd_info_kernel_symbol']} k on d.kernel_id = k.id order by d.start"))
    starts = [i for i, r in enumerate(rows) if "k_ba_edges" in r[2]]
    print(db, len(starts), "calls")
    for ci, s in enumerate(starts):
        e = starts[ci + 1] if ci + 1 < len(starts) else len(rows)
        call = rows[s:e]
        span = (call[-1][1] - call[0][0]) / 1e3
        busy = sum(r[1] - r[0] for r in call) / 1e3
        gaps = [((call[i + 1][0] - call[i][1]) / 1e3, call[i][2][:40], call[i + 1][2][:40]) for i in range(len(call) - 1)]
        nchol = sum("chol" in r[2] for r in call)
        print(f"call {ci}: {len(call)} dispatches, {nchol} factorisations, span {span:.1f} us, busy {busy:.1f} us, "
              f"idle {sum(g[0] for g in gaps):.1f} us")
        if ci == len(starts) - 1:
            by = {}
            for r in call:
                k = r[2].split("(")[0][:48]
                by[k] = by.get(k, 0) + (r[1] - r[0]) / 1e3
            for k, v in sorted(by.items(), key=lambda kv: -kv[1]):
                print(f"    {k:<48s} {v:9.1f} us")
            gp = {}
            for g, a, b in gaps:
                gp[(a, b)] = gp.get((a, b), 0) + g
            print("  idle by transition (top 12):")
            for (a, b), v in sorted(gp.items(), key=lambda kv: -kv[1])[:12]:
                print(f"    {v:8.1f} us  {a} -> {b}")
