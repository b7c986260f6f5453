#!/usr/bin/env python3
"""Average per-dispatch counter values of the kernels in a rocprofv3 --pmc
counter_collection.csv, grouped by kernel name (optionally filtered by a substring), plus
derived MFMA utilisation and clock figures.

    python tools/pmc_kernel_summary.py gpurun_out/gp1/p1/p1_counter_collection.csv [gemm]
"""
import collections
import csv
import re
import sys


def main(path, sub=""):
    rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        if sub not in n:
            continue
        key = n[:n.index("(")] if "(" in n else n
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[key].add(r["Dispatch_Id"])
    for k, c in per.items():
        nd = len(disp[k])
        avg = {n: v / nd for n, v in c.items()}
        print(f"{k[-80:]}  dispatches {nd}")
        for n in sorted(avg):
            print(f"   {n:28s} {avg[n]:16.0f}")
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if n in avg:
                    print(f"   {n} / WAVE_CYCLES = {avg[n] / wc:.3f}")
        busy, cu = avg.get("SQ_VALU_MFMA_BUSY_CYCLES"), avg.get("SQ_BUSY_CU_CYCLES")
        if busy and cu:
            # MFMA_BUSY counts cycles summed over SIMDs; BUSY_CU_CYCLES quad-cycles per CU
            print(f"   MFMA busy / (4 SIMD x CU busy cycles) = {busy / (4 * 4 * cu):.3f} "
                  "(if BUSY_CU_CYCLES is in quad-cycles)")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
