#!/usr/bin/env python3
"""Summarise rocprofv3 rocpd databases (kernel trace + PMC passes) into the
text files committed under profiles/.

usage: prof_summary.py --trace gpurun_out/prof_r1/trace_results.db
                       [--fetch gpurun_out/pmc_fetch/pmc_results.db]
                       [--write gpurun_out/pmc_write/pmc_results.db]
                       --out profiles/r01_bench_vga_b256

FETCH_SIZE / WRITE_SIZE are reported in KB per dispatch as rocprofv3 gives
them, plus the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE is
doubled (wide coalesced reads are tallied at half their bytes); WRITE_SIZE is
taken as is.  Both are per-dispatch averages over every dispatch of a kernel.
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_\w+(?:<[^>]*>)?)\(", name) or re.search(r"(\w+)\(", name)
    return m.group(1) if m else name


def kernel_stats(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    return [(short(r[0]), int(r[1]), float(r[2]), float(r[3]), float(r[4])) for r in rows]


def pmc(db, counter):
    con = sqlite3.connect(db)
    acc = defaultdict(list)
    for name, val in con.execute("select kernel_name, value from counters_collection where counter_name = ?",
                                 (counter,)):
        acc[short(name)].append(float(val))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--sq", help="pmc db with SQ_* counters")
    ap.add_argument("--json", help="also write per-kernel HBM bytes per dispatch here")
    ap.add_argument("--frames-per-dispatch", type=float, default=0.0)
    ap.add_argument("--out", required=True)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    lines = []
    if a.title:
        lines.append(f"# {a.title}")
    lines.append("## rocprofv3 --kernel-trace --stats (durations in ms)")
    lines.append(f"{'kernel':<20} {'calls':>6} {'total_ms':>12} {'avg_ms':>10} {'pct':>7}")
    for n, c, tot, avg, pct in kernel_stats(a.trace):
        lines.append(f"{n:<20} {c:>6} {tot / 1e3:>12.1f} {avg / 1e3:>10.2f} {pct:>7.2f}")
    if a.fetch or a.write:
        f = pmc(a.fetch, "FETCH_SIZE") if a.fetch else {}
        w = pmc(a.write, "WRITE_SIZE") if a.write else {}
        lines.append("")
        lines.append("## PMC per dispatch (separate --pmc passes; KB as reported, FETCH x2 = gfx950-corrected)")
        lines.append(f"{'kernel':<20} {'dispatches':>10} {'FETCH_KB':>12} {'FETCHx2_MB':>11} {'WRITE_KB':>12} "
                     f"{'HBM_MB':>9}")
        for k in sorted(set(f) | set(w)):
            fk, fn = f.get(k, (float('nan'), 0))
            wk, _ = w.get(k, (float('nan'), 0))
            hbm = (2 * fk + wk) / 1024.0
            lines.append(f"{k:<20} {fn:>10} {fk:>12.1f} {2 * fk / 1024:>11.2f} {wk:>12.1f} {hbm:>9.2f}")
    if a.sq:
        names = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
                 "SQ_WAIT_INST_ANY", "SQ_BUSY_CYCLES"]
        c = {n: pmc(a.sq, n) for n in names}
        lines.append("")
        lines.append("## SQ counters per dispatch (per-wave instruction counts; cycle shares of SQ_WAVE_CYCLES)")
        lines.append(f"{'kernel':<20} {'waves':>9} {'VALU/w':>8} {'SALU/w':>8} {'LDS/w':>7} {'wait_any':>9} "
                     f"{'wait_inst':>9}")
        for k in sorted(c["SQ_WAVES"]):
            wv = c["SQ_WAVES"][k][0]
            if wv <= 0:
                continue
            g = lambda n: c[n].get(k, (float("nan"), 0))[0]   # noqa: E731
            wc = g("SQ_WAVE_CYCLES")
            lines.append(f"{k:<20} {wv:>9.0f} {g('SQ_INSTS_VALU') / wv:>8.0f} {g('SQ_INSTS_SALU') / wv:>8.0f} "
                         f"{g('SQ_INSTS_LDS') / wv:>7.0f} {g('SQ_WAIT_ANY') / wc:>9.2f} {g('SQ_WAIT_INST_ANY') / wc:>9.2f}")
    if a.json and a.fetch and a.write:
        import json
        f = pmc(a.fetch, "FETCH_SIZE")
        w = pmc(a.write, "WRITE_SIZE")
        out = {"source": a.out, "frames_per_dispatch": a.frames_per_dispatch,
               "note": "FETCH_SIZE x2 (gfx950) + WRITE_SIZE, KB x 1024, averaged over dispatches",
               "kernels": {k: {"hbm_bytes_per_dispatch": (2 * f[k][0] + w.get(k, (0.0, 0))[0]) * 1024.0,
                               "fetch_kb": f[k][0], "write_kb": w.get(k, (0.0, 0))[0]} for k in f}}
        if a.sq:   # VALU wave-instructions per dispatch (whole device), for the issue roofline
            vi = pmc(a.sq, "SQ_INSTS_VALU")
            for k, d in out["kernels"].items():
                if k in vi:
                    d["valu_insts_per_dispatch"] = vi[k][0]
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)
    text = "\n".join(lines) + "\n"
    with open(a.out, "w") as fh:
        fh.write(text)
    print(text)


if __name__ == "__main__":
    main()
