"""Average duration per (kernel, grid) from a rocprofv3 kernel trace CSV, in trace order."""
import csv
import re
import sys
from collections import OrderedDict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
agg = OrderedDict()
for r in rows:
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    name = re.sub(r"\(.*", "", name)[:60]
    key = (name, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg.setdefault(key, [0, 0.0])
    a[0] += 1
    a[1] += d
for (name, grid), (n, t) in agg.items():
    print(f"{t / n:8.1f} us  x{n:4d}  grid {grid:6d}  {name}")
