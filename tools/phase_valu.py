"""Per-phase instruction split of k_fast / k_describe from the stop-after-phase
builds of tools/phase_valu.sh: a phase = counts(its stop build) - counts(the
previous one), the last phase = counts(product) - counts(the last stop build);
per wave of the product.
    python tools/phase_valu.py gpurun_out/phase_valu_TAG"""
import sqlite3
import sys
from collections import defaultdict
from pathlib import Path

# kernel: (build tag, [(stop build, phase name)]; the last phase ends at the product)
PHASES = {
    "k_fast": ("f", [(1, "prologue + staging"), (2, "iniThFAST compass + compaction"), (3, "iniThFAST arc scores"),
                     (4, "iniThFAST NMS + output"), (None, "minThFAST pass (cells left empty)")]),
    "k_describe": ("d", [(1, "prologue + staging"), (2, "moments + row pass (int8 MFMA)"),
                         (4, "orientation + sample offsets + column pass"), (None, "rounding + bit tests + records")]),
}
CTRS = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_MFMA", "SQ_WAVE_CYCLES"]


def counts(db):
    v = defaultdict(lambda: defaultdict(list))
    for name, cn, val in sqlite3.connect(db).execute(
            "select kernel_name, counter_name, value from counters_collection"):
        for k in PHASES:
            if k + "<false" in name:
                v[k][cn].append(float(val))
    return {k: {cn: sum(x) / len(x) for cn, x in c.items()} for k, c in v.items()}


def main():
    root = Path(sys.argv[1])
    run = {}
    for d in sorted(root.iterdir()):
        dbs = list(d.rglob("*results.db")) if d.is_dir() else []
        if dbs:
            run[d.name] = counts(dbs[0])
    for k, (tag, names) in PHASES.items():
        full = run["full"][k]
        waves = full["SQ_WAVES"]
        print(f"{k}: {waves:.0f} waves per launch; counts per wave")
        print(f"    {'phase':46s}" + "".join(f"{c[8:]:>12s}" for c in CTRS))
        prev = {c: 0.0 for c in CTRS}
        for i, (stop, nm) in enumerate(names):
            cur = run[f"{tag}{stop}"][k] if stop else full
            row = [(cur.get(c, 0.0) - prev[c]) / waves for c in CTRS]
            print(f"    {str(i + 1) + '. ' + nm:46s}" + "".join(f"{x:12.1f}" for x in row))
            prev = {c: cur.get(c, 0.0) for c in CTRS}
        print(f"    {'total':46s}" + "".join(f"{full.get(c, 0.0) / waves:12.1f}" for c in CTRS))


if __name__ == "__main__":
    main()
