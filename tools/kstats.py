"""Print a rocprofv3 kernel_stats.csv compactly: short name, calls, avg us, total ms, %."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    name = re.sub(r"\(.*", "", r["Name"].replace("orbx::(anonymous namespace)::", "").replace("void ", ""))
    print(f"{name[:48]:48s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} us {float(r['TotalDurationNs']) / 1e6:9.3f} ms {float(r['Percentage']):6.2f}%")
