"""Turn a tools/gpu_profile.sh run (gpurun_out/prof_trace, gpurun_out/prof_pmc) into the committed
summaries under profiles/:

    python tools/summarize_prof.py --tag r01 [--config cfg2]

profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
profiles/<tag>_pmc.json           per-kernel PMC averages; for the timed render kernel the HBM
                                  traffic per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 B
                                  (FETCH_SIZE/WRITE_SIZE are in KiB; gfx950 FETCH_SIZE counts
                                  half of the bytes of wide reads -- MI355X_MICROARCH.md, HBM)
"""
import argparse
import csv
import glob
import json
import os
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    """Kernel name without return type, namespaces and arguments ("render_fast_kernel_w6<30, false, 17>")."""
    base = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    return base.replace("rtk::", "").replace("rtfast::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--kernel", default=None, help="default: the timed render kernel with the most time")
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)

    stats = os.path.join(a.src, "prof_trace", "run_kernel_stats.csv")
    if a.kernel is None and os.path.exists(stats):
        rows = [r for r in csv.DictReader(open(stats)) if short(r["Name"]).startswith("render_fast_kernel")
                and ", false," in short(r["Name"])]
        a.kernel = short(max(rows, key=lambda r: float(r["TotalDurationNs"]))["Name"]) if rows else None
    summary = {"config": a.config, "kernel": a.kernel}
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(out, f"{a.tag}_kernel_stats.csv"))
        for row in csv.DictReader(open(stats)):
            if short(row["Name"]) == a.kernel:
                summary["rocprof_avg_ms"] = float(row["AverageNs"]) / 1e6
                summary["rocprof_calls"] = int(row["Calls"])

    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    meta = {}
    for path in sorted(glob.glob(os.path.join(a.src, "prof_pmc", "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(path)):
            k = short(row["Kernel_Name"])
            per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            meta[k] = {"vgpr": int(row["VGPR_Count"]), "sgpr": int(row["SGPR_Count"]),
                       "lds_bytes": int(row["LDS_Block_Size"]), "workgroup": int(row["Workgroup_Size"]),
                       "grid": int(row["Grid_Size"])}
    kernels = {}
    for k, cs in per.items():
        kernels[k] = {"resources": meta[k], "counters": {c: sum(v) / len(v) for c, v in cs.items()}}
    summary["kernels"] = kernels
    r = kernels.get(a.kernel)
    if r and "FETCH_SIZE" in r["counters"] and "WRITE_SIZE" in r["counters"]:
        c = r["counters"]
        summary["fetch_kib_per_launch"] = c["FETCH_SIZE"]
        summary["write_kib_per_launch"] = c["WRITE_SIZE"]
        summary["hbm_bytes_per_launch"] = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            summary["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    path = os.path.join(out, f"{a.tag}_pmc.json")
    json.dump(summary, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in summary.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
