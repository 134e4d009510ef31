"""The GPU box's host CPU for the bench's cpu_baseline (analysis aid): cgroup quota, affinity,
model, and the oracle's config-2 frame time at several thread counts, so a change of the baseline
between rounds can be traced to the host rather than the code.

    python tools/cpu_probe.py [--rows 270] [--threads 8,16,32]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import rt_testlib as T  # noqa: E402


def read(path):
    try:
        return open(path).read().strip()
    except OSError as e:
        return f"<{e.strerror}>"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=270)
    ap.add_argument("--threads", default="8,16,32")
    args = ap.parse_args()
    info = {"cpu": bench.cpu_model(), "os_cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "usable_cpus": bench.usable_cpus(), "cpu.max": read("/sys/fs/cgroup/cpu.max"),
            "omp_env": os.environ.get("OMP_NUM_THREADS"), "loadavg": read("/proc/loadavg")}
    print(json.dumps(info), flush=True)
    w, h, spp, b = 1920, 1080, 8, 6
    osc = T.OracleScene("bunny")
    r0 = (h - args.rows) // 2
    for th in map(int, args.threads.split(",")):
        rng = T.oracle_rng_frame(bench.SEED, w, h, th)
        stat0 = read("/sys/fs/cgroup/cpu.stat")
        t = time.perf_counter()
        _, st = osc.render(w, h, spp, b, rng=rng, rows=(r0, r0 + args.rows), threads=th, stats=True)
        dt = time.perf_counter() - t
        stat1 = read("/sys/fs/cgroup/cpu.stat")
        print(json.dumps({"threads": th, "rows": args.rows, "s": round(dt, 2), "mrays_s": round(float(st[0]) / dt / 1e6, 3),
                          "cpu.stat_before": stat0.replace("\n", "; "), "cpu.stat_after": stat1.replace("\n", "; ")}),
              flush=True)


if __name__ == "__main__":
    main()
