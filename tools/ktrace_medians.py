#!/usr/bin/env python3
"""Median duration of each kernel (matching a substring) in a rocprofv3 kernel trace, split
into K consecutive equal parts (one per benchmark configuration run in order).

    python tools/ktrace_medians.py gpurun_out/tbe/kt_kernel_trace.csv tbe 3
"""
import collections
import csv
import re
import statistics
import sys


def main(path, sub="", parts=1):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = collections.OrderedDict()
    for r in rows:
        n = r["Kernel_Name"]
        if sub not in n:
            continue
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        n = n[:n.index("(")] if "(" in n else n
        d.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in d.items():
        m = max(1, len(v) // parts)
        meds = [round(statistics.median(v[i * m:(i + 1) * m]), 2) for i in range(parts)
                if v[i * m:(i + 1) * m]]
        print(f"{k[-72:]:72s} {len(v):6d} {meds}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "",
         int(sys.argv[3]) if len(sys.argv) > 3 else 1)
