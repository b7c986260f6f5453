#!/usr/bin/env python3
"""Per-kernel timeline of one training step from a rocprofv3 kernel trace (kt_kernel_trace.csv):
finds the last run of consecutive dispatches between two step-opening launches - the lookup
launch (tbe_fwd*) or, with the sort deferred, the bottom-MLP chain (mlp_chain_kernel) - i.e.
one hipGraph replay,
prints each kernel with its grid, duration and the idle gap before it."""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(\(.*", "", name)
    return name[:70]


def main(path, which=-2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "tbe_fwd" in r["Kernel_Name"]]
    if len(starts) < 3:  # the sort deferred: steps open with the bottom-MLP chain
        starts = [i for i, r in enumerate(rows)
                  if re.search(r"\bmlp_chain_kernel\b", r["Kernel_Name"])]
    a, b = starts[which - 1], starts[which]
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    prev_end = t0
    tot = 0
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gx = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        gy = int(r["Grid_Size_Y"]) // max(1, int(r["Workgroup_Size_Y"]))
        print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev_end) / 1e3:5.1f} dur {(e - s) / 1e3:6.1f}  "
              f"grid {gx}x{gy} wg {r['Workgroup_Size_X']}  vgpr {r['VGPR_Count']}+{r['Accum_VGPR_Count']}  "
              f"{short(r['Kernel_Name'])}")
        tot += e - s
        prev_end = e
    print(f"step span {(prev_end - t0) / 1e3:.1f} us, kernel sum {tot / 1e3:.1f} us, "
          f"{len(step)} kernels")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else -2)
