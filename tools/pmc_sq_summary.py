"""Per-kernel SQ counter summary of a rocprofv3 --pmc csv (SQ_WAVE_CYCLES, SQ_WAIT_ANY,
SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, SQ_VALU_MFMA_BUSY_CYCLES, SQ_LDS_BANK_CONFLICT,
SQ_LDS_IDX_ACTIVE, SQ_WAIT_INST_LDS): fractions of wave cycles and the LDS conflict share.

    python tools/pmc_sq_summary.py <pmc_counter_collection.csv>
"""
import collections
import csv
import re
import sys


def main(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = re.sub(r"\(.*", "", name)
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r["Dispatch_Id"])
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"])
    tot = sum(v["SQ_WAVE_CYCLES"] for _, v in rows)
    print(f"{'kernel':58s} {'waveCyc%':>8s} {'waitAny':>7s} {'waitIns':>7s} {'active':>7s} "
          f"{'ldsConf':>7s} {'waitLds':>7s}")
    for k, v in rows:
        w = v["SQ_WAVE_CYCLES"] or 1
        if v["SQ_WAVE_CYCLES"] / tot < 0.002:
            continue
        print(f"{k[:58]:58s} {100 * v['SQ_WAVE_CYCLES'] / tot:8.1f} {v['SQ_WAIT_ANY'] / w:7.2f} "
              f"{v['SQ_WAIT_INST_ANY'] / w:7.2f} {v['SQ_ACTIVE_INST_ANY'] / w:7.2f} "
              f"{v['SQ_LDS_BANK_CONFLICT'] / max(1, v['SQ_LDS_IDX_ACTIVE']):7.2f} "
              f"{v['SQ_WAIT_INST_LDS'] / w:7.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
