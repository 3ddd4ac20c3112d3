"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels by total time (short names)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in rows[:n]:
    name = r["Name"]
    m = re.match(r"(?:void )?(?:\(anonymous namespace\)::)?([\w:<>, ]+?)\(", name)
    short = (m.group(1) if m else name)[:70]
    if short.startswith("Cijk"):
        short = name[:40]
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms  calls={int(r["Calls"]):5d}  avg={float(r["AverageNs"])/1e3:9.2f} us  '
          f'{float(r["Percentage"]):5.1f}%  {short}')
