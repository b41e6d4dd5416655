"""Run one bench extra at other stream counts (batch sweeps):
    python tools/sweep_extra.py KEY N1 [N2 ...] [--steps K]"""
import subprocess
import sys

key, rest = sys.argv[1], sys.argv[2:]
steps = "10"
if "--steps" in rest:
    i = rest.index("--steps")
    steps = rest[i + 1]
    rest = rest[:i] + rest[i + 2:]
code = """
import sys
sys.path.insert(0, '.')
import bench
bench.EXTRAS = [(k, m, w, h, nf, int(sys.argv[2]) if k == sys.argv[1] else b, u) for k, m, w, h, nf, b, u in bench.EXTRAS]
sys.argv = ['bench.py', '--extra', sys.argv[1], '--steps', sys.argv[3]]
sys.exit(bench.main())
"""
for n in rest:
    # one process per size (each sets up its own device state)
    r = subprocess.run([sys.executable, "-c", code, key, n, steps], capture_output=True, text=True)
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    print(n, line[-1] if line else r.stderr[-400:], flush=True)
