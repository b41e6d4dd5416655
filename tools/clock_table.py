"""Clock and VALU issue table from tools/gpu_clock_pass.sh's databases:
tools/clock_table.py OUTDIR

Per kernel (mean over its dispatches in the PMC pass):
  clock  = GRBM_GUI_ACTIVE / 8 / duration   (rocprofv3 sums GRBM over the 8 XCDs;
           MI355X_MICROARCH.md 'DVFS give-back')
  cyc/wi = 1024 SIMDs x duration x clock / SQ_INSTS_VALU
           (cycles one SIMD spends per VALU wave-instruction, if VALU issue were
           the only thing the kernel did; the ceiling is the ubench's figure)
  issue  = SQ_INSTS_VALU / duration in G wave-instr/s
The kernel-trace pass gives the duration without counters attached (trace_us)."""
import re
import sqlite3
import sys
from collections import defaultdict
from pathlib import Path


def base(name):
    m = re.search(r"(k_\w+(?:<[^>(]*>)?)", name)
    return m.group(1) if m else name.split("(")[0][:40]


out = Path(sys.argv[1])


def db(sub):
    c = sorted((out / sub).rglob("*.db"))
    return sqlite3.connect(str(c[0])) if c else None


for tag, pmc, tr in (("valu_rate micro-benchmark", "ubpmc", "ubtrace"), ("bench.py VGA B=1024 unsplit", "pmc", "trace")):
    con = db(pmc)
    if con is None:
        print(f"# {tag}: no PMC database")
        continue
    per = defaultdict(lambda: defaultdict(float))
    for did, name, cn, val, dur, grid in con.execute(
            "select dispatch_id, kernel_name, counter_name, value, duration, grid_size from counters_collection"):
        d = per[did]
        # the micro-benchmark launches each kind at several grid sizes
        d["name"] = base(name) + (f"/{int(grid) // 65536}W" if pmc == "ubpmc" else "")
        d[cn] = float(val)
        d["dur"] = float(dur)
        d["grid"] = float(grid)
    trace = defaultdict(list)
    tcon = db(tr)
    if tcon is not None:
        for name, s, e in tcon.execute("select name, start, end from kernels"):
            trace[base(name)].append((e - s) / 1e3)
    agg = defaultdict(list)
    for did in sorted(per):
        agg[per[did]["name"]].append(per[did])
    print(f"# {tag}")
    print(f"{'kernel':<24}{'n':>4}{'pmc_us':>10}{'trace_us':>10}{'clock_GHz':>10}{'VALU/wave':>10}"
          f"{'cyc/wi':>8}{'Gwi/s':>8}{'busy/dur':>9}")
    for k, ds in sorted(agg.items()):
        n = len(ds)
        dur = sum(d["dur"] for d in ds) / n * 1e-9
        grbm = sum(d.get("GRBM_GUI_ACTIVE", 0) for d in ds) / n
        valu = sum(d.get("SQ_INSTS_VALU", 0) for d in ds) / n
        waves = sum(d.get("SQ_WAVES", 0) for d in ds) / n
        busy = sum(d.get("SQ_BUSY_CYCLES", 0) for d in ds) / n
        clk = grbm / 8 / dur if dur > 0 else 0
        cyc = 1024 * dur * clk / valu if valu else 0
        tus = sum(trace[k]) / len(trace[k]) if trace.get(k) else 0
        print(f"{k[:24]:<24}{n:>4}{dur * 1e6:>10.1f}{tus:>10.1f}{clk / 1e9:>10.3f}{valu / waves if waves else 0:>10.1f}"
              f"{cyc:>8.2f}{valu / dur / 1e9 if dur else 0:>8.1f}{busy / 8 / dur / 1e9 if dur else 0:>9.3f}")
    print()
