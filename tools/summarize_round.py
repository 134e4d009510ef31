"""Committed summaries of a tools/gpu_profiles.sh run (gpurun_out/) under profiles/<tag>_*:

    python tools/summarize_round.py --tag r02

profiles/<tag>_<cfg>_bench.json        the bench line of that config (roofline with the in-run PMC
                                       counters of the production render kernel)
profiles/<tag>_<cfg>_pmc.json          per-pass rocprofv3 --pmc counters of the production render
                                       kernel (mean per dispatch) + derived figures
profiles/<tag>_<cfg>_kernel_stats.csv  rocprofv3 --kernel-trace --stats of the bench (cfg2, cfg4)
profiles/<tag>_foreign_hip_api.json    HIP API calls of the --foreign bench: whole run and the timed
                                       frames (no synchronising call may appear there)
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out")
OUT = os.path.join(ROOT, "profiles")
SYNC = ("hipStreamSynchronize", "hipDeviceSynchronize", "hipMemcpy", "hipEventSynchronize", "hipMemcpyWithStream",
        "hipMemset", "hipFree", "hipHostFree", "hipStreamWaitEvent")


def short(name):
    """Kernel name without return type, namespaces and arguments ("render_fast_kernel_w6<30, false, 17>")."""
    base = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    return base.replace("rtk::", "").replace("rtfast::", "")


def bench_line(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def pmc_summary(cfg):
    """Per pass, the counters of the render-kernel variant with the most dispatches (a probe frame
    at the other occupancy is left out, as bench.read_pmc_pass does)."""
    out = {"config": cfg, "passes": {}}
    for d in sorted(glob.glob(os.path.join(SRC, f"pmc_{cfg}", "pass*"))):
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        meta = {}
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                k = short(r["Kernel_Name"])
                if not k.startswith("render_fast_kernel"):
                    continue
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta[k] = {"kernel": k, "vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]),
                           "lds_bytes": int(r["LDS_Block_Size"]), "scratch_bytes": int(r.get("Scratch_Size", 0) or 0),
                           "grid": int(r["Grid_Size"])}
        k = max(vals, key=lambda x: max(len(v) for v in vals[x].values())) if vals else None
        v = vals[k] if k else {}
        out["passes"][os.path.basename(d)] = {"kernel": meta.get(k), "dispatches": max((len(x) for x in v.values()), default=0),
                                             "counters_mean": {c: sum(x) / len(x) for c, x in sorted(v.items())}}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    a = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    for cfg in ("cfg1", "cfg2", "cfg3", "cfg4", "cfg5"):
        b = os.path.join(SRC, f"bench_{a.tag}_{cfg}.log")
        if os.path.exists(b):
            line = bench_line(b)
            json.dump(line, open(os.path.join(OUT, f"{a.tag}_{cfg}_bench.json"), "w"), indent=1)
            s = pmc_summary(cfg)
            r = line["roofline"]
            s["derived"] = {k: r.get(k) for k in ("frac", "achieved", "peak", "unit", "lane_utilization", "clock_ghz",
                                                  "frac_at_clock", "kernel_ms", "profiled_kernel_ms", "traffic",
                                                  "valu_wave_instructions_per_launch")}
            s["derived"]["hbm"] = r.get("hbm")
            json.dump(s, open(os.path.join(OUT, f"{a.tag}_{cfg}_pmc.json"), "w"), indent=1)
            print(cfg, "frac", r.get("frac"), "kernel_ms", r.get("kernel_ms"), "lanes", r.get("lane_utilization"))
        tl = os.path.join(SRC, f"trace_{cfg}.log")
        if os.path.exists(tl) and bench_line(tl):
            # the bench line printed by the profiled command itself (PMC pass skipped under a profiler)
            json.dump(bench_line(tl), open(os.path.join(OUT, f"{a.tag}_{cfg}_trace_bench.json"), "w"), indent=1)
        t = os.path.join(SRC, f"trace_{cfg}", "run_kernel_stats.csv")
        if os.path.exists(t):
            shutil.copy(t, os.path.join(OUT, f"{a.tag}_{cfg}_kernel_stats.csv"))
            for row in csv.DictReader(open(t)):
                if short(row["Name"]).startswith("render_fast_kernel") and ", false," in short(row["Name"]):
                    print(cfg, "rocprof", short(row["Name"]), "calls", row["Calls"], "avg ms", float(row["AverageNs"]) / 1e6)
    api = os.path.join(SRC, "hiptrace_foreign", "run_hip_api_trace.csv")
    ker = os.path.join(SRC, "hiptrace_foreign", "run_kernel_trace.csv")
    if os.path.exists(api) and os.path.exists(ker):
        calls = [r for r in csv.DictReader(open(api)) if not r["Function"].startswith("__hip")]
        rf = [r for r in csv.DictReader(open(ker)) if "render_fast" in r["Kernel_Name"] and ", false," in r["Kernel_Name"]]
        timed = set(r["Correlation_Id"] for r in rf[-10:])
        ts = sorted(int(c["Start_Timestamp"]) for c in calls if c["Correlation_Id"] in timed)
        win = [c for c in calls if ts and ts[0] <= int(c["Start_Timestamp"]) <= ts[-1]]
        res = {"source": "rocprofv3 --hip-trace --kernel-trace -- python3 bench.py --foreign --steps 10 --warmup 2",
               "whole_run": dict(collections.Counter(c["Function"] for c in calls).most_common()),
               "timed_frames": len(ts),
               "timed_window_calls": dict(collections.Counter(c["Function"] for c in win).most_common()),
               "timed_window_synchronising_calls": sum(1 for c in win if c["Function"] in SYNC)}
        json.dump(res, open(os.path.join(OUT, f"{a.tag}_foreign_hip_api.json"), "w"), indent=1)
        print("foreign: timed frames", len(ts), "synchronising calls in the timed window:",
              res["timed_window_synchronising_calls"])


if __name__ == "__main__":
    main()
