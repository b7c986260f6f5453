"""Per-step HBM traffic per kernel group from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE, counter unit KB) of `bench.py --no-graph --steps S --warmup W`.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half the bytes of
wide coalesced reads -> doubled; WRITE_SIZE taken as is.

Usage: python tools/pmc_summary.py <dir with pmc_FETCH_SIZE/ pmc_WRITE_SIZE/> <steps + warmup of the pass>
                                   [bench --config name, default terabyte]
"""
import csv
import json
import sys
from collections import defaultdict

GROUPS = [
    # gemm_role_kernel: GEMM launches that also carry a deferred TBE / head pass
    ("gemm", ("gemm_group_kernel", "gemm_role_kernel", "gemm_generic_kernel", "gemm_rowsum_kernel",
              "gemm_f32_", "gemm_splitk_reduce_kernel")),
    ("tbe_fwd", ("tbe_fwd_kernel", "tbe_fwd_presort_kernel", "mlp_chain_kernel")),  # + sort, bottom MLP
    ("tbe_bwd", ("tbe_bwd_", "tbe_tiled_", "tbe_keys_hist_", "tbe_update_pass_", "rocprim")),
    ("qr", ("qr_",)),
    ("interaction", ("interact_",)),
    ("colsum", ("colsum_",)),
    ("head", ("head_", "mean_kernel", "outer_drelu_kernel")),
    ("relu_bwd", ("relu_bwd_kernel",)),
]


def group_of(name):
    for g, keys in GROUPS:
        if any(k in name for k in keys):
            return g
    return None


def load(path, counter):
    per = defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        g = group_of(r["Kernel_Name"])
        if g is None:
            continue
        per[g][0] += float(r["Counter_Value"]) * 1024.0
        per[g][1] += 1
    return per


def main():
    d, steps = sys.argv[1], int(sys.argv[2])
    config = sys.argv[3] if len(sys.argv) > 3 else "terabyte"
    f = load(f"{d}/pmc_FETCH_SIZE/pmc_counter_collection.csv", "FETCH_SIZE")
    w = load(f"{d}/pmc_WRITE_SIZE/pmc_counter_collection.csv", "WRITE_SIZE")
    out = {"_config": config}
    for g, _ in GROUPS:
        if g not in f:
            continue
        # launches before the timed loop (init, warmup) share the same kernels: average
        # over all launches of the group and scale to the per-step launch count
        n = f[g][1]
        per_launch_read = 2.0 * f[g][0] / n
        per_launch_write = w[g][0] / max(1, w[g][1])
        launches_per_step = n / steps
        out[g] = {"launches": n, "read_bytes_per_launch": round(per_launch_read),
                  "write_bytes_per_launch": round(per_launch_write),
                  "hbm_bytes_per_launch": round(per_launch_read + per_launch_write),
                  "launches_per_step_approx": round(launches_per_step, 2),
                  "hbm_bytes_per_step": round((2.0 * f[g][0] + w[g][0]) / steps)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
