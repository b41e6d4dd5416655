"""Per-kernel averages of every counter in rocprofv3 --pmc databases (one
table; counters per dispatch, and per wave when SQ_WAVES is present).
    python tools/pmc_table.py DB [DB ...] [--kernels k_describe k_fast]"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?)\(", name) or re.search(r"(\w+)\(", name)
    return m.group(1) if m else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--kernels", nargs="*", default=None)
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))
    for db in a.dbs:
        con = sqlite3.connect(db)
        for name, cn, v in con.execute("select kernel_name, counter_name, value from counters_collection"):
            vals[short(name)][cn].append(float(v))
    for k in sorted(vals):
        if a.kernels and not any(k.startswith(x) for x in a.kernels):
            continue
        c = vals[k]
        waves = sum(c["SQ_WAVES"]) / len(c["SQ_WAVES"]) if "SQ_WAVES" in c else None
        print(k)
        for cn in sorted(c):
            avg = sum(c[cn]) / len(c[cn])
            extra = f"   {avg / waves:12.2f} per wave" if waves and cn != "SQ_WAVES" else ""
            print(f"    {cn:32s} {avg:16.0f}{extra}")


if __name__ == "__main__":
    main()
