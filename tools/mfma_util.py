#!/usr/bin/env python3
"""MFMA utilisation per kernel from one rocprofv3 --pmc pass of the bench step
(SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES).

SQ_VALU_MFMA_BUSY_CYCLES = sum over SIMDs of MFMA busy cycles (= N_mfma x cycles per MFMA:
checked against SQ_INSTS_MFMA x 32 for v_mfma_f32_16x16x4_f32); GRBM_GUI_ACTIVE is summed
over the 8 XCDs, so the dispatch lasts GRBM_GUI_ACTIVE / 8 cycles and the chip offers
1024 SIMDs x that many MFMA cycles.  util = MFMA_BUSY / (1024 x GRBM_GUI_ACTIVE / 8).

    python tools/mfma_util.py <counter_collection.csv>
"""
import collections
import csv
import re
import sys

SIMDS = 1024  # 256 CUs x 4
XCDS = 8


def main(path):
    rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        key = n[:n.index("(")] if "(" in n else n
        key = re.sub(r"^void ", "", key)
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[key].add(r["Dispatch_Id"])
    out = []
    for k, c in per.items():
        nd = len(disp[k])
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / nd
        gui = c.get("GRBM_GUI_ACTIVE", 0.0) / nd
        ins = c.get("SQ_INSTS_MFMA", 0.0) / nd
        if busy <= 0 or gui <= 0:
            continue
        cyc = gui / XCDS
        out.append((busy / (SIMDS * cyc), k, nd, ins, busy, cyc))
    print(f"{'util':>6} {'disp':>5} {'mfma/disp':>10} {'busy cyc/disp':>14} {'dur cyc':>9}  kernel")
    for u, k, nd, ins, busy, cyc in sorted(out, key=lambda x: -x[4] * x[2]):
        print(f"{u:6.3f} {nd:5d} {ins:10.0f} {busy:14.0f} {cyc:9.0f}  {k[:90]}")


if __name__ == "__main__":
    main(sys.argv[1])
