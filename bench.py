"""Benchmark of the hot path: one "step" = one progressive frame of the per-pixel path tracer
(RayTracing/main_raytracing.cu:162-200 via raytracing_process) over the whole frame.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2]

N = 1 runs BASELINE.json configs[1] (Stanford bunny scene, 1920x1080, 8 spp, 6 bounces), its 16x16
tiles launched heaviest first (--plan cost: one untimed probe frame's per-wave clocks order them;
the pixels, RNG layout and output are the reference's -- only the launch order changes).
N > 1: one process per GPU.  Launched without a launcher (WORLD_SIZE unset), bench.py starts the
N rank processes itself before touching the GPU and forwards rank 0's line; under
torch.distributed.run it is one of the ranks.  The frame's 16x16 tiles are dealt over the ranks
(--plan cost, the default: a probe frame's per-wave clocks, longest processing time first, each
rank's heaviest tiles first; --plan rr: round-robin), each rank renders its tiles into a compact
shard, and ONE gather per frame (rt_gather_shards: RCCL over xGMI, from librt_hip.so) brings the
shards to rank 0, where rt_unshard_tiles scatters them into the pitched surface.  The gather of
frame i runs on its own stream, overlapped with the render of frame i+1.
  --scaling strong (default): the BASELINE frame itself split N ways (the metric's
      "bunny 1920x1080x8spp @1/2/4/8 GPU"; --config cfg3 is BASELINE configs[2], 4K 64 spp).
  --scaling weak: per-GPU work fixed -- the same camera at sqrt(N) x the resolution per axis.
Timing: barrier + synchronize on both sides of exactly K steps, max over ranks; every rank's own
render-kernel time is reported (rank_kernel_ms).

Rank 0 prints one JSON line.  value = ray segments traced (GetRayHit calls, counted exactly by
the kernel) per second over the whole job, in Mrays/s.

roofline: the render kernel is issue-bound (its ~23 MB scene lives in L2 / Infinity Cache, so HBM
sees a few GB per frame), so the bound is VALU issue: achieved = SQ_INSTS_VALU per launch (a
rocprofv3 --pmc pass of this same workload, run by this script as a child process) / the
kernel's HIP-event time; peak = 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction
(MI355X_MICROARCH.md: v_fma_f32 wave64 = 2 cycles per SIMD).  Beside it: lane utilisation, the
effective clock, HBM bytes from FETCH_SIZE x 2 + WRITE_SIZE (the guide's gfx950 correction), and
the SURVEY.md 8(d) algorithmic-bytes demand figure.
cpu_baseline = the CPU restatement of the reference (oracle/, "port") on every core this process
may use on the host (cgroup quota and affinity), same scene and seed; the CPU model is reported.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (scene, width, height, spp, bounces, description)
    "cfg1": ("bunny", 256, 256, 1, 1, "stanford-bunny 256x256 1spp primary rays (BASELINE configs[0])"),
    "cfg2": ("bunny", 1920, 1080, 8, 6, "stanford-bunny 1920x1080 8spp (BASELINE configs[1])"),
    "cfg3": ("bunny", 3840, 2160, 64, 6, "stanford-bunny 3840x2160 64spp (BASELINE configs[2])"),
    "cfg4": ("bunny4", 1920, 1080, 8, 6, "4x instanced bunny 1920x1080 8spp (BASELINE configs[3])"),
    "cfg5": ("plane1m", 1920, 1080, 1, 6, "1M-triangle plane 1920x1080 1spp (BASELINE configs[4])"),
}
SEED = 0xDEADBEEF
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, memory hierarchy)
SIMDS = 1024           # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4        # peak engine clock
VALU_CYCLES = 2        # wave64 fp32 VALU instruction per SIMD (v_fma_f32: 2 cycles, MI355X_MICROARCH.md)
VALU_PEAK = SIMDS * CLOCK_GHZ / VALU_CYCLES  # G wave-instructions per second
# PMC passes (rocprofv3 does not split counters over passes; block limits: 8 SQ, 4 TCC, 2 GRBM)
PMC_PASSES = [
    ["SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_SALU", "SQ_WAVES",
     "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "GRBM_COUNT"],
    ["FETCH_SIZE"],
    ["WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"],
]
# optional pass (round 6): the issue side -- LDS instructions and bank-conflict cycles, scalar-memory instructions,
# the CU's one scalar ALU (quad-cycles), and where wave cycles go (issue stall / waiting / issuing); a failure
# here leaves the required passes' numbers in place
PMC_PASSES_OPTIONAL = [
    ["SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_SMEM", "SQ_INST_CYCLES_SALU", "SQ_ACTIVE_INST_SCA",
     "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"],
]


def algorithmic_bytes(stats, sphere_count, pixels):
    """per segment 32 B per BVH node visited, 56 B per triangle test
    (4 B index + 16 B face + 3 x 12 B positions), 32 B per sphere tested, 64 B material per
    accepted hit, 36 B (3 normals) per accepted triangle hit; per pixel 48 B RNG state
    read+write and 32 B surface read+write."""
    seg, nodes, tris, tacc, sacc = (int(stats[i]) for i in range(5))
    return (32 * nodes + 56 * tris + 32 * sphere_count * seg + 64 * (tacc + sacc) + 36 * tacc + 80 * pixels)


def usable_cpus():
    """Cores this process may run on: affinity, capped by the cgroup CPU quota (the GPU box gives
    a 16-CPU quota on a 256-thread host)."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def weak_size(width, height, world):
    """The weak-scaled frame for N ranks: sqrt(N) x the resolution per axis, width a multiple of
    the 16-pixel tile, aspect kept (1920x1080: N=2 2720x1530, N=4 3840x2160, N=8 5424x3051)."""
    if world <= 1:
        return width, height
    w = int(round(width * world ** 0.5 / 16.0)) * 16
    return w, int(round(w * height / width))


def cpu_baseline_child(cfg, sample_rows=None, timeout_s=300):
    """cpu_baseline in a fresh child process (no torch, no HIP runtime in it): the oracle's OpenMP
    threads then share the box's CPU quota with nothing of the benchmark process."""
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", "--config", cfg,
           "--cpu-rows", str(sample_rows or 0)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
    if r.returncode != 0:
        return {"error": f"exit {r.returncode}: {r.stderr[-300:]}"}
    return json.loads(r.stdout.strip().splitlines()[-1])


def cpu_baseline(cfg, sample_rows=None):
    """Oracle ("port") on this host's cores: bounded sample of the same frame (rows)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rt_testlib as T

    scene_name, w, h, spp, bounces, _ = CONFIGS[cfg]
    threads = usable_cpus()
    osc = T.OracleScene(scene_name)
    rows = sample_rows or h
    if rows >= h:
        r0, r1 = 0, h
    else:
        r0 = (h - rows) // 2
        r1 = r0 + rows
    rng = T.oracle_rng_frame(SEED, w, h, threads)
    t = time.perf_counter()
    _, st = osc.render(w, h, spp, bounces, rng=rng, rows=(r0, r1), threads=threads, stats=True)
    dt = time.perf_counter() - t
    samples = (r1 - r0) * w * spp
    try:
        load = open("/proc/loadavg").read().split()[:3]
    except OSError:
        load = None
    return {"value": round(float(st[0]) / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "cpu": cpu_model(), "host_threads": os.cpu_count(), "host_loadavg": load, "process": "child (oracle only)",
            "sample": f"{cfg} rows [{r0},{r1}) of {h} ({samples} camera samples, {int(st[0])} segments), {dt:.1f} s",
            "samples_per_s": round(samples / dt, 1)}


# ------------------------------------------------------------------------------------------
# launcher: N rank processes started before any GPU call
# ------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, cmd=None, deadline_s=480.0, poll_s=0.05):
    """bench.py --gpus N without a launcher: start N rank processes of this script (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set), forward rank 0's stdout, and return the first failing
    exit code (stopping the other ranks then: a dead rank leaves the others waiting in a
    collective).  A job still running after `deadline_s` -- a rank stuck in communicator set-up or
    in a collective -- is killed whole: the ranks still alive are named on stderr and the launcher
    returns 124.  The launcher itself never touches the GPU."""
    port = _free_port()
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = {}
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs[r] = subprocess.Popen(cmd, env=env, stdout=None if r == 0 else subprocess.DEVNULL)
    t0 = time.monotonic()
    rc = 0
    while procs:
        for r, p in list(procs.items()):
            code = p.poll()
            if code is None:
                continue
            del procs[r]
            if code != 0 and rc == 0:
                rc = code
                print(f"bench.py launcher: rank {r} exited with {code}; stopping ranks {sorted(procs)}", file=sys.stderr)
                for q in procs.values():
                    q.kill()
        if procs and deadline_s and time.monotonic() - t0 > deadline_s:
            print(f"bench.py launcher: ranks {sorted(procs)} still running after {deadline_s:.0f} s; killing all ranks",
                  file=sys.stderr, flush=True)
            for q in procs.values():
                q.kill()
            for q in procs.values():
                q.wait()
            return 124
        time.sleep(poll_s)
    return rc


class Watchdog:
    """Per-rank deadline for N > 1 jobs under any launcher (torch.distributed.run has none of its
    own): if the rank is still running after `deadline_s`, it names the phase it is stuck in and
    ends its process with 124, which ends the job (the other ranks fail their next collective or
    hit their own deadline)."""

    def __init__(self, rank, deadline_s):
        import threading

        self.rank, self.phase = rank, "start"
        self.timer = threading.Timer(deadline_s, self._fire) if deadline_s else None
        if self.timer:
            self.timer.daemon = True
            self.timer.start()

    def _fire(self):
        print(f"bench.py rank {self.rank}: deadline exceeded in phase '{self.phase}'; exiting", file=sys.stderr, flush=True)
        os._exit(124)

    def cancel(self):
        if self.timer:
            self.timer.cancel()


# ------------------------------------------------------------------------------------------
# PMC pass (rocprofv3 child process running this script with --pmc-child)
# ------------------------------------------------------------------------------------------
def under_profiler():
    return any(k.startswith("ROCPROF") for k in os.environ)


def _short(name):
    """Kernel name without return type, namespaces and arguments ("render_fast_kernel_w6<30, false, 17>")."""
    base = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    return base.replace("rtk::", "").replace("rtfast::", "")


def read_pmc_pass(d):
    """One rocprofv3 --pmc output directory: {counter: [value per dispatch]} of the production
    render kernel, its name, and its dispatch durations (s) from the kernel trace.  When the run
    dispatched more than one render-kernel variant (a probe at the other occupancy), the variant
    with the most dispatches is the one reported."""
    per = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            k = _short(row["Kernel_Name"])
            if k.startswith("render_fast_kernel"):
                per.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    if not per:
        return {}, None, []
    kernel = max(per, key=lambda k: max(len(v) for v in per[k].values()))
    durations = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if _short(row["Kernel_Name"]) == kernel:
                durations.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return per[kernel], kernel, durations


def pmc_pass(args, out_dir, timeout_s=150):
    """Counters of the production render kernel for this workload, one rocprofv3 run per pass;
    returns {counter: mean per dispatch}, the kernel name and the profiled dispatch time."""
    rocprof = shutil.which("rocprofv3")
    if rocprof is None:
        return None, "rocprofv3 not found"
    out_dir = os.path.abspath(out_dir)  # the child runs in the temp directory
    counters, kernel, durations = {}, None, []
    optional_error = None
    for i, cs in enumerate(PMC_PASSES + PMC_PASSES_OPTIONAL):
        optional = i >= len(PMC_PASSES)
        d = os.path.join(out_dir, f"pass{i}")
        cmd = [rocprof, "--kernel-trace", "--pmc", *cs, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--config", args.config,
               "--plan", args.plan, "--tune", str(args.tune), "--refill", str(args.refill),
               "--lanes", args.lanes, "--lane-units", str(args.lane_units), "--occupancy", str(args.occupancy_chosen)]
        if args.foreign:
            cmd.append("--foreign")
        if getattr(args, "lane_map_np", None) is not None:
            os.makedirs(out_dir, exist_ok=True)
            mp = os.path.join(out_dir, "lane_map.npy")
            np.save(mp, args.lane_map_np)
            cmd += ["--lane-map-file", mp]
        if args.build_options:
            cmd += ["--build-options", args.build_options]
        try:
            r = subprocess.run(cmd, cwd=tempfile.gettempdir(), capture_output=True, text=True, timeout=timeout_s,
                               env=dict(os.environ, TMPDIR=tempfile.gettempdir()))
        except subprocess.TimeoutExpired:
            if optional:
                optional_error = f"pass {i} timed out"
                break
            return None, f"pass {i} timed out"
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "child.log"), "w") as fh:
            fh.write(r.stdout + "\n---- stderr ----\n" + r.stderr)
        if r.returncode != 0:
            err = [l for l in r.stderr.splitlines() if "Error" in l or "error" in l or "Traceback" in l]
            msg = f"pass {i} exit {r.returncode}: {' | '.join(err[-3:])[-400:]}"
            if optional:
                optional_error = msg
                break
            return None, msg
        vals, k, dur = read_pmc_pass(d)
        kernel = k or kernel
        if i == 0:
            durations = dur
        if not vals:
            if optional:
                optional_error = f"pass {i}: no render_fast_kernel rows"
                break
            return None, f"pass {i}: no render_fast_kernel rows"
        # rows are per dispatch and counter (summed over XCDs by rocprofv3's csv); mean per dispatch
        for c, v in vals.items():
            counters[c] = sum(v) / len(v)
    return {"counters": counters, "kernel": kernel, "optional_error": optional_error,
            "profiled_kernel_s": float(np.mean(durations)) if durations else None}, None


def roofline(pmc, kern_s, bytes_alg, err=None):
    out = {"bound": "valu", "unit": "Gwave-instr/s", "peak": round(VALU_PEAK, 1), "achieved": None, "frac": None,
           "traffic": None, "kernel_ms": round(kern_s * 1e3, 3),
           "peak_basis": f"{SIMDS} SIMDs x {CLOCK_GHZ} GHz / {VALU_CYCLES} cycles per wave64 VALU instruction",
           "algorithmic_bytes_per_launch": int(bytes_alg),
           "algorithmic_demand_gbs": round(bytes_alg / kern_s / 1e9, 1)}
    if pmc is None:
        out["pmc_error"] = err
        return out
    c = pmc["counters"]
    valu = c["SQ_INSTS_VALU"]
    out["kernel"] = pmc["kernel"]
    out["valu_wave_instructions_per_launch"] = int(valu)
    out["achieved"] = round(valu / kern_s / 1e9, 1)
    out["frac"] = round(valu / kern_s / 1e9 / VALU_PEAK, 4)
    out["lane_utilization"] = round(c["SQ_THREAD_CYCLES_VALU"] / max(1.0, c["SQ_ACTIVE_INST_VALU"] * 64), 4)
    out["salu_instructions_per_launch"] = int(c["SQ_INSTS_SALU"])
    tp = pmc.get("profiled_kernel_s")
    if tp:
        clk = c["GRBM_GUI_ACTIVE"] / 8 / tp / 1e9  # summed over the 8 XCDs
        out["clock_ghz"] = round(clk, 3)
        out["frac_at_clock"] = round(valu * VALU_CYCLES / (SIMDS * clk * 1e9 * tp), 4)
        out["profiled_kernel_ms"] = round(tp * 1e3, 3)
    hbm = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)  # KiB; gfx950 FETCH_SIZE counts half
    out["traffic"] = hbm
    out["hbm"] = {"bytes_per_launch": hbm, "achieved_gbs": round(hbm / kern_s / 1e9, 1), "peak_gbs": HBM_PEAK_GBS,
                  "frac": round(hbm / kern_s / 1e9 / HBM_PEAK_GBS, 4),
                  "l2_hit_rate": round(c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)}
    if "SQ_INSTS_LDS" in c:  # the optional issue-side pass
        wc = max(1.0, c["SQ_WAVE_CYCLES"])
        out["issue"] = {"lds_instructions_per_launch": int(c["SQ_INSTS_LDS"]),
                        "lds_bank_conflict_cycles": int(c["SQ_LDS_BANK_CONFLICT"]),
                        "smem_instructions_per_launch": int(c["SQ_INSTS_SMEM"]),
                        "salu_wave_cycles": int(4 * c["SQ_INST_CYCLES_SALU"]),  # waves' cycles in SALU instructions
                        # per-SE aggregates over the waves (SQ_WAVE_CYCLES' basis): where a wave's cycles go
                        "wave_frac_issuing": round(c["SQ_ACTIVE_INST_ANY"] / wc, 4),
                        "wave_frac_issue_stalled": round(c["SQ_WAIT_INST_ANY"] / wc, 4),
                        "wave_frac_waiting": round(c["SQ_WAIT_ANY"] / wc, 4)}
    elif pmc.get("optional_error"):
        out["issue"] = {"error": pmc["optional_error"]}
    out["pmc_counters"] = {k: round(v, 1) for k, v in sorted(c.items())}
    return out


# ------------------------------------------------------------------------------------------
# ranks
# ------------------------------------------------------------------------------------------
def setup_dist(backend, same_device):
    """One process per GPU (RANK / LOCAL_RANK / WORLD_SIZE from the launcher); the "nccl" backend
    is RCCL on ROCm and only carries set-up and timing collectives (the frame's gather is
    rt_gather_shards).  --backend gloo --same-device rehearses the N > 1 path with every rank on
    GPU 0 (a one-GPU box), staging the gather through host memory."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world


CLOCK_HZ = 100e6  # wave_clock ticks: the device's constant 100 MHz clock (s_memrealtime)


def sanitize_wave_clocks(clocks, wall_s=None, k=4096.0):
    """Per-wave probe clocks (int64 view of the kernel's unsigned s_memrealtime deltas) -> float64
    costs and the number of entries flagged invalid.  The clock is the device's one 100 MHz time
    base, so a valid delta lies in [0, probe wall time]; this stays as a guard that logs: a delta
    that is negative, longer than the probe frame's wall time (`wall_s`, when given), or more than
    `k` x the median of the others is replaced by that median (rt_shard_plan rejects costs < 0,
    and an inflated outlier would pull a mean up).  k is far above any real spread: a sky-only wave
    and the heaviest floor wave of config 3 differ by a few hundred times."""
    c = np.asarray(clocks, dtype=np.int64).astype(np.float64)
    bad = c < 0
    if wall_s is not None:
        bad |= c > wall_s * CLOCK_HZ * 1.05 + 1e3
    if (~bad).any():
        med = float(np.median(c[~bad]))
        if med > 0:
            bad |= c > k * med
    if bad.any():
        good = c[~bad]
        c[bad] = float(np.median(good)) if good.size else 1.0
    return c, int(bad.sum())


def gather_layout(counts, cap):
    """The frame gather's bookkeeping (rt_gather_shards): rank r sends its first counts[r] tiles of
    256 float4 slots (recv_bytes[r] bytes); the root lays rank r's bytes at r * stride, stride = the
    plan capacity's worth of tiles.  Slots past counts[r] * 256 in row r are padding that
    rt_unshard_tiles never reads (their tile-list entries are -1)."""
    return [int(c) * 256 * 16 for c in counts], int(cap) * 256 * 16


def make_plan(rt, scene, W, H, SPP, BOUNCES, rank, world, plan_kind, dev):
    """(tile_lists [world, cap] int32 numpy, counts, probe info).  'cost': every rank renders its
    round-robin tiles once with per-wave clocks (set-up, untimed, throw-away RNG), the per-tile
    costs are summed over ranks, and rt_shard_plan deals them longest-first."""
    import torch
    import torch.distributed as dist

    if plan_kind == "rr" or world == 1 and plan_kind != "cost":
        lists, counts = rt.shard_plan(W, H, world)
        return lists, counts, None
    rr, rc = rt.shard_plan(W, H, world)
    mine = torch.from_numpy(rr[rank, : rc[rank]]).to(dev)
    rng = rt.alloc_rng(int(rc[rank]) * 256)
    rt.init_rng_tiles(rng, W, H, mine, SEED)
    scene.upload(rng.data_ptr())  # the probe's own states (the caller re-uploads with the run's)
    shard = torch.zeros((int(rc[rank]) * 256, 4), dtype=torch.float32, device=dev)
    clocks = torch.zeros(int(rc[rank]) * 4, dtype=torch.int64, device=dev)
    t0 = time.perf_counter()
    rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, rank, world, out_shard=shard, tile_list=mine,
              wave_clock=clocks)
    torch.cuda.synchronize()
    probe_s = time.perf_counter() - t0
    per_wave, nbad = sanitize_wave_clocks(clocks.cpu().numpy(), wall_s=probe_s)
    if nbad:
        print(f"[rank {rank}] probe frame: {nbad} of {per_wave.size} wave clocks invalid, replaced by the median",
              file=sys.stderr)
    cost = np.zeros(rt.sharding.tiles_total(W, H), dtype=np.float64)
    cost[rr[rank, : rc[rank]]] = per_wave.reshape(-1, 4).sum(1)
    if world > 1:
        both = np.concatenate([cost, [float(nbad)]])
        t = torch.from_numpy(both).to(dev) if dist.get_backend() == "nccl" else torch.from_numpy(both)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        both = t.cpu().numpy()
        cost, nbad = both[:-1], int(both[-1])
    lists, counts = rt.shard_plan(W, H, world, cost)
    del rng, shard, clocks
    return lists, counts, {"probe_frame_s": round(probe_s, 4), "kind": "cost (probe-frame wave clocks, LPT)",
                           "invalid_wave_clocks": nbad}


def make_lane_map(rt, render, rng, slots, units, dev, refine=0, theta=0.85, waves_per_simd=6):
    """rt_lane_plan for this rank's list: one probe frame of per-pixel work (timing variant of the
    production kernel, set-up, untimed) on a copy of the RNG states, then the split plan, then up to
    `refine` rounds of measured refinement (refine_lane_map).  Returns (device int32 lane map, info)."""
    import torch

    rng_saved = rng.clone()
    cost = torch.zeros(slots, dtype=torch.int32, device=dev)  # one per slot of the tile list
    t0 = time.perf_counter()
    render(lane_cost=cost)
    torch.cuda.synchronize()
    probe_s = time.perf_counter() - t0
    rng.copy_(rng_saved)
    del rng_saved
    cost_np = cost.cpu().numpy()
    lm, nlong = rt.lane_plan(cost_np, units, 1.0)
    info = {"lane_probe_s": round(probe_s, 4), "waves": int(lm.size // 64), "long_waves": nlong, "parallel_units": units}
    if refine > 0:
        lm, info["refine"] = refine_lane_map(rt, render, rng, lm, cost_np, refine, theta, dev, waves_per_simd)
        if lm is None:  # the plain tile order won
            info["waves"] = 0
            return None, info
        info["waves"] = int(lm.size // 64)
    return torch.from_numpy(lm).to(dev), info


def refine_lane_map(rt, render, rng, lm, cost, rounds, theta, dev, waves_per_simd, frames=3):
    """Measured lane-plan refinement (rt_lane_refine): time `frames` consecutive frames of the map
    (production kernel, HIP events, the RNG chain advancing from a saved copy of the states as the
    run's frames will), sum each wave's clocks over the same frames (timing variant), split the waves
    within `theta` of the longest, and keep the new map only while those frames get faster.  Several
    frames, not one: which waves are slow changes from frame to frame with the random paths, and a
    plan fitted to one frame's tail does not carry over.  Every candidate is a permutation of the
    shard's slots, so the frames are the same bit for bit."""
    import torch

    saved = rng.clone()

    def timed(m_dev):
        total = 0.0
        for _ in range(frames):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            render(lane_slots=m_dev, waves_per_simd=waves_per_simd)
            e1.record()
            torch.cuda.synchronize()
            total += e0.elapsed_time(e1)
        rng.copy_(saved)
        return total / frames

    def clocks(m_dev):
        acc = np.zeros(m_dev.numel() // 64, dtype=np.int64)
        clk = torch.zeros(m_dev.numel() // 64, dtype=torch.int64, device=dev)
        for _ in range(frames):
            render(lane_slots=m_dev, wave_clock=clk)
            torch.cuda.synchronize()
            acc += sanitize_wave_clocks(clk.cpu().numpy())[0].astype(np.int64)
        rng.copy_(saved)
        return acc

    t0 = time.perf_counter()
    cur, cur_dev = lm, torch.from_numpy(lm).to(dev)
    best_ms = timed(cur_dev)
    hist, kept = [round(best_ms, 3)], 0
    for _ in range(rounds):
        new, nsplit = rt.lane_refine(cur, cost, clocks(cur_dev), theta)
        new_dev = torch.from_numpy(new).to(dev)
        ms = timed(new_dev)
        hist.append(round(ms, 3))
        if not nsplit or ms >= best_ms:
            break
        cur, cur_dev, best_ms, kept = new, new_dev, ms, kept + 1
    # the plain tile order over the same frames: a lane map is kept only if it beats it
    plain_ms = timed(None)
    if plain_ms <= best_ms:
        del saved
        return None, {"theta": theta, "frames": frames, "waves_per_simd": waves_per_simd, "frame_ms": hist, "rounds_kept": kept,
                      "plain_ms": round(plain_ms, 3), "map": "dropped (the plain tile order is faster)",
                      "s": round(time.perf_counter() - t0, 3)}
    # where the kept map's time goes: its longest waves (summed clocks over the frames, ms per frame)
    # and how many pixels each holds
    ticks = clocks(cur_dev)
    top = np.argsort(-ticks)[:6]
    mw = cur.reshape(-1, 64)
    longest = [[round(float(ticks[w]) / frames / CLOCK_HZ * 1e3, 3), int((mw[w] >= 0).sum())] for w in top]
    del saved
    return cur, {"theta": theta, "frames": frames, "waves_per_simd": waves_per_simd, "frame_ms": hist, "rounds_kept": kept,
                 "plain_ms": round(plain_ms, 3), "longest_waves_ms_pixels": longest,
                 "s": round(time.perf_counter() - t0, 3)}


def production_counts(t):
    """The production kernel's own work on one frame, from its timing variant's counters (`t`: STAT_NAMES ->
    value): where the wave cycles go (small steps / big-leaf rounds / the rest: shading, sky, RNG,
    output), small-step wave iterations and their active lanes, and the big leaves' tests by twins
    (mirror.h quads / units: unit triangles tested, twins decided from their partner's values, twins
    tested).  frame0_counts beside it counts the reference's own work (statistics variant)."""
    tot = max(1, t["cycles_total"])
    out = {"cycles_frac": {"small": round(t["cycles_small"] / tot, 4), "big": round(t["cycles_big"] / tot, 4),
                           "rest": round(1 - (t["cycles_small"] + t["cycles_big"]) / tot, 4)},
           "wave_small_iters": t["wave_small_iters"], "lane_small": t["lane_small"],
           "small_lanes_per_iter": round(t["lane_small"] / max(1, t["wave_small_iters"]), 2),
           "rounds_coop": t["rounds_coop"], "rounds_shared": t["rounds_shared"], "coop_rays": t["coop_rays"],
           "big_unit_tests": t["big_tests"], "twins_decided": t["twin_decided"], "twins_tested": t["twin_tests"],
           "wave_big_iters": t["wave_big_iters"]}
    if t["cycles_tree_cut"]:
        out["cycles_frac"]["tree_walk"] = round(t["cycles_tree_cut"] / tot, 4)
        out["defer_end2"], out["defer_redo"] = t["defer_end2"], t["defer_redo"]
    return out


def settle_occupancy(probe_occupancy, lane_slots, refine_occ, world, cdev):
    """The frames' occupancy with this rank's lane map (or None), and whether the map survives.
    probe_occupancy(map) -> (waves per SIMD, {wps: ms}) times each candidate and max-reduces over ranks,
    so EVERY rank must make the same probe calls: whether a rank kept its lane map is its own
    decision (refine_lane_map drops a map that loses to the plain order on its shard), so the re-probe
    of the plain order below runs when ANY rank holds a map (a MAX-reduced flag), and when the plain
    order wins every rank drops its map.  Returns (wps, best, lane_slots, note or None)."""
    import torch
    import torch.distributed as dist

    wps, best = probe_occupancy(lane_slots)
    any_map = lane_slots is not None
    if world > 1:
        t = torch.tensor([1 if any_map else 0], dtype=torch.int32, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        any_map = bool(t.item())
    if any_map and refine_occ is not None and wps != refine_occ:
        # a map was kept against the plain order at another occupancy: compare again at this one
        plain_wps, plain_best = probe_occupancy(None)
        if plain_best[plain_wps] <= best[wps]:
            return plain_wps, plain_best, None, f"dropped at {wps} waves per SIMD (the plain tile order is faster)"
    return wps, best, lane_slots, None


def run(args):
    import torch
    import torch.distributed as dist
    import __graft_entry__ as G

    multi = int(os.environ.get("WORLD_SIZE", "1")) > 1
    wd = Watchdog(int(os.environ.get("RANK", "0")), args.rank_deadline if multi else 0)
    wd.phase = "rendezvous"
    rank, world = setup_dist(args.backend, args.same_device)
    wd.phase = "scene set-up and plans"
    assert world == args.gpus or args.pmc_child, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    rt = G.load_package()
    build_opts = {k: float(v) if k == "split_angle" else int(v)
                  for k, v in (kv.split("=") for kv in args.build_options.split(","))} if args.build_options else {}
    # A/B render paths (librt_hip_exp.so; the production path never needs it): the tracers, refill, the
    # RT_TUNE A/B families, and the big-leaf screen variants a mirror with screen records asks for
    # (rt_kernel.hip needs_experimental)
    if args.tracer != "fast" or args.refill or (args.tune & 0x1030) or build_opts.get("leaf_screens", 0):
        rt.load_experimental()
    if build_opts:  # exact-preserving mirror / BVH builder knobs (rt_set_build_options)
        rt.set_build_options(**build_opts)
    scene_name, W, H, SPP, BOUNCES, desc = CONFIGS[args.config]
    if world > 1 and args.scaling == "weak":
        W, H = weak_size(W, H, world)
        desc = f"{desc}, weak-scaled to {W}x{H} for {world} GPUs (same camera)"
    dev = torch.device("cuda", torch.cuda.current_device())
    stream = torch.cuda.current_stream()

    t0 = time.perf_counter()
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    sharded = world > 1
    tile_list = None
    plan_info = None
    if sharded:
        # the scene must be uploaded before the probe; RNG pointer is set per buffer below
        probe_rng = rt.alloc_rng(256)
        scene.upload(probe_rng.data_ptr())
        lists, counts, plan_info = make_plan(rt, scene, W, H, SPP, BOUNCES, rank, world, args.plan, dev)
        cap = lists.shape[1]
        count = int(counts[rank])
        tile_list = torch.from_numpy(lists[rank, :count]).to(dev)
        lists_dev = torch.from_numpy(lists).to(dev)
        rng = rt.alloc_rng(cap * 256)
        rt.init_rng_tiles(rng, W, H, tile_list, SEED)
        bufs = [torch.zeros((cap * 256, 4), dtype=torch.float32, device=dev) for _ in range(2)]
        gathered = torch.empty((world, cap * 256, 4), dtype=torch.float32, device=dev) if rank == 0 else None
        frame = rt.alloc_surface(W, H) if rank == 0 else None
        pixels_rank = count * 256
    else:
        if args.plan == "cost":
            probe_rng = rt.alloc_rng(256)
            scene.upload(probe_rng.data_ptr())
            lists, counts, plan_info = make_plan(rt, scene, W, H, SPP, BOUNCES, 0, 1, "cost", dev)
            tile_list = torch.from_numpy(lists[0, : int(counts[0])]).to(dev)
        rng = rt.alloc_rng(W * H)
        rt.init_rng_states(rng, W, H, SEED)
        rng_init = rng.clone() if args.foreign else None
        bufs = [rt.alloc_surface(W, H) for _ in range(2)]
        pixels_rank = W * H
    scene.upload(rng.data_ptr())
    target = scene
    if args.foreign:
        # the reference host's own Scene::Upload: its arrays in its own allocations, no mirror
        # registered -- rendered through the fingerprint-gated path (rt_render, no host sync)
        assert not sharded, "--foreign is a single-GPU measurement"
        target = foreign_copy(rt, scene)
        rt.render(target, bufs[0], bufs[1], W, H, SPP, BOUNCES, 0, tile_list=tile_list)  # first frame starts the build
        rt.foreign_mirror_wait(target)
        rng.copy_(rng_init)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0

    lane_slots = None

    def render(i, cur, prev, **kw):
        ls = kw.pop("lane_slots", lane_slots)
        tune = kw.pop("tune", args.tune)
        if sharded:
            rt.render(scene, None, prev, W, H, SPP, BOUNCES, i, rank, world, out_shard=cur, tile_list=tile_list,
                      tune=tune, lane_slots=ls, **refill(kw))
        else:
            rt.render(target, cur, prev, W, H, SPP, BOUNCES, i, tile_list=tile_list, tune=tune,
                      lane_slots=ls, **refill(kw))

    occupancy = {"waves_per_simd": 0 if args.occupancy == "auto" else int(args.occupancy)}

    def refill(kw):  # the probe (lane_cost) runs without refill
        if "lane_cost" in kw:
            return kw
        if args.tracer != "fast" and "wave_clock" not in kw and "stats" not in kw:  # counts: production kernel
            kw = dict(kw, tracer=args.tracer)
        kw = dict(occupancy, **kw)
        return kw if args.foreign else dict(kw, refill_lanes=args.refill)

    # occupancy (rt_render_params.waves_per_simd): time one untimed frame at 5, 6 and 7 waves per
    # SIMD (twice each, on a copy of the RNG states) and keep the fastest; a strong-scaled shard
    # (N > 1) also tries the 5-wave build capped at 3 and 4 resident waves per SIMD (dynamic LDS):
    # config 2 at N = 8, 6.36 ms at 4 vs 6.66 ms at 6 (profiles/r03e_capped_shards.jsonl)
    cands = (5, 6, 7) if world == 1 else (3, 4, 5, 6, 7)

    def probe_occupancy(ls):
        rng_saved = rng.clone()
        best = {}
        for wps in cands + cands:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            render(0, bufs[0], None, waves_per_simd=wps, lane_slots=ls)
            e1.record(stream)
            torch.cuda.synchronize()
            rng.copy_(rng_saved)
            best[wps] = min(best.get(wps, 1e30), e0.elapsed_time(e1))
        del rng_saved
        if world > 1:
            # one variant for the whole job: every rank takes the setting whose slowest rank is fastest
            cdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
            t = torch.tensor([best[w] for w in cands], dtype=torch.float64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            best = {w: float(x) for w, x in zip(cands, t.tolist())}
        return min(best, key=best.get), best

    auto_occ = args.occupancy == "auto" and not args.pmc_child
    lanes_on = args.lanes in ("on", "auto") and not args.foreign and tile_list is not None
    refine_occ = None if args.occupancy == "auto" else int(args.occupancy)
    if auto_occ and lanes_on and not args.lane_map_file and args.lane_refine > 0:
        # the lane map is refined (and compared with the plain tile order) at the occupancy the
        # frames will run at: a first probe on the plain order picks it
        t1 = time.perf_counter()
        refine_occ, first = probe_occupancy(None)
        setup_s += time.perf_counter() - t1
        plan_info = dict(plan_info or {}, occupancy_plain_order={"waves_per_simd": refine_occ,
                                                                 "probe_ms": {str(k): round(v, 3) for k, v in first.items()}})

    # lane plan (rt_lane_plan): split the waves whose pixels form the frame's serial tail
    if lanes_on and args.lane_map_file:
        # PMC child: the parent's final lane map, so the counters are of exactly the frames it timed
        lane_slots = torch.from_numpy(np.load(args.lane_map_file)).to(dev)
    elif lanes_on:
        t1 = time.perf_counter()
        lane_slots, lane_info = make_lane_map(rt, lambda **kw: render(0, bufs[0], None, **kw), rng,
                                              tile_list.numel() * 256, args.lane_units, dev,
                                              refine=args.lane_refine, theta=args.lane_theta,
                                              waves_per_simd=refine_occ or 6)
        setup_s += time.perf_counter() - t1
        plan_info = dict(plan_info or {}, lanes=lane_info)

    if auto_occ:
        t1 = time.perf_counter()
        cdev = dev if world > 1 and dist.get_backend() == "nccl" else torch.device("cpu")
        occupancy["waves_per_simd"], best, lane_slots, note = settle_occupancy(probe_occupancy, lane_slots, refine_occ,
                                                                               world, cdev)
        if note:
            plan_info["lanes"]["map"] = note
        setup_s += time.perf_counter() - t1
        plan_info = dict(plan_info or {}, occupancy={"waves_per_simd": occupancy["waves_per_simd"],
                                                     "probe_ms": {str(k): round(v, 3) for k, v in best.items()},
                                                     "agreed": "max over ranks" if world > 1 else "single rank"})
    args.lane_map_np = lane_slots.cpu().numpy() if lane_slots is not None else None
    args.occupancy_chosen = occupancy["waves_per_simd"] or 5

    if args.pmc_child:  # under rocprofv3 --pmc: a warm-up and two frames of the production kernel
        for i in range(3):
            render(i, bufs[i & 1], bufs[(i + 1) & 1])
        torch.cuda.synchronize()
        return 0

    # --- exact traversal counts of one frame (stats kernel variant) on a copy of the RNG state
    rng_saved = rng.clone()
    stats = torch.zeros(rt.STAT_COUNT, dtype=torch.int64, device=dev)
    render(0, bufs[0], bufs[1], stats=stats)
    torch.cuda.synchronize()
    rng.copy_(rng_saved)
    del rng_saved
    stats0 = stats.cpu().numpy().astype(np.uint64)
    # --- the production kernel's own work on the same frame and launch shape: its timing variant (RT_TUNE
    #     bit 8: per-wave phase clocks, small-step iterations and lane-steps, big-leaf tests by twins)
    prod0 = None
    if not args.foreign and args.tracer == "fast" and not args.refill:
        rng_saved = rng.clone()
        tst = torch.zeros(rt.STAT_COUNT, dtype=torch.int64, device=dev)
        render(0, bufs[0], bufs[1], stats=tst, tune=args.tune | 256)
        torch.cuda.synchronize()
        rng.copy_(rng_saved)
        del rng_saved
        prod0 = production_counts(dict(zip(rt.STAT_NAMES, tst.cpu().numpy().astype(np.int64).tolist())))
    gpu = scene.gpu.contents
    bytes0 = algorithmic_bytes(stats0, gpu.sphere_count, pixels_rank)
    if args.foreign and rt.foreign_last_tracer(target) != 1:
        raise RuntimeError("--foreign: the production tracer did not render the frame")

    # --- the frame-end gather: rt_gather_shards (RCCL) unless rehearsing on gloo
    comm = None
    gather_kind = None
    if sharded:
        if args.backend == "nccl" and args.gather == "rccl":
            obj = [rt.Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            comm_err = None
            try:
                comm = rt.Comm(world, rank, obj[0])
            except rt.RTError as e:  # every rank must agree before any frame: MIN-reduce an ok flag
                comm, comm_err = None, str(e)
            ok = torch.tensor([0 if comm_err else 1], dtype=torch.int32, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()):
                gather_kind = "rt_gather_shards (RCCL send/recv group, librt_hip.so)"
            else:  # the library's own communicator failed on some rank: gather through torch.distributed instead
                if comm is not None:
                    comm.close()
                comm = None
                gather_kind = f"torch.distributed.gather (nccl; rt_comm_init_rank failed: {comm_err or 'on another rank'})"
                print(f"bench.py: rank {rank}: {gather_kind}", file=sys.stderr, flush=True)
        else:
            gather_kind = f"torch.distributed.gather ({args.backend})"
    recv_bytes = gather_layout(counts, lists.shape[1])[0] if sharded else None

    seg_counter = torch.zeros(1, dtype=torch.int64, device=dev)
    n_total = args.warmup + args.steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_total)]
    comm_stream = torch.cuda.Stream() if comm is not None else None
    rendered = torch.cuda.Event()
    gathered_ev = [torch.cuda.Event(), torch.cuda.Event()]  # the gather that last read bufs[j]
    gather_pending = [False, False]

    # per-frame gather + unshard time: HIP events on comm_stream around rt_gather_shards and (rank 0)
    # rt_unshard_tiles; the host clock around the synchronous gloo rehearsal gather
    gev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_total)]
    gather_host_ms = [0.0] * n_total

    def step(i):
        cur, prev = bufs[i & 1], bufs[(i + 1) & 1]
        if comm is not None and gather_pending[i & 1]:
            stream.wait_event(gathered_ev[i & 1])  # frame i-2's gather still reads `cur`
        ev[i][0].record(stream)
        render(i, cur, prev, segment_counter=seg_counter if i >= args.warmup else None)
        ev[i][1].record(stream)
        if comm is not None:
            rendered.record(stream)
            comm_stream.wait_event(rendered)
            gev[i][0].record(comm_stream)
            comm.gather(cur, recv_bytes[rank], gathered, cur.numel() * 4, recv_bytes, 0, comm_stream)
            if rank == 0:
                rt.unshard_tiles(frame, W, H, gathered, lists_dev, stream=comm_stream)
            gev[i][1].record(comm_stream)
            gathered_ev[i & 1].record(comm_stream)
            gather_pending[i & 1] = True
        elif sharded:
            th = time.perf_counter()
            got = rt.sharding.gather_shards(cur, rank, world, out=gathered)
            if rank == 0:
                rt.unshard_tiles(frame, W, H, got, lists_dev)
                torch.cuda.synchronize()
            gather_host_ms[i] = (time.perf_counter() - th) * 1e3

    wd.phase = "warm-up frames"
    fixture = None
    for i in range(args.warmup):
        step(i)
        if i == 0 and args.check and not sharded and not args.foreign and rank == 0:
            torch.cuda.synchronize()  # frame 0 of the timed launch shape against the oracle's (untimed)
            fixture = check_oracle_fixture(rt, args.config, W, H, bufs[0], rng)
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    torch.cuda.synchronize()
    wd.phase = "timed frames"
    t_start = time.perf_counter()
    for i in range(args.warmup, n_total):
        step(i)
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start

    wd.phase = "report"
    exit_code = 0
    segs = int(seg_counter.item())
    kern_ms = [ev[i][0].elapsed_time(ev[i][1]) for i in range(args.warmup, n_total)]
    kern_avg_s = float(np.mean(kern_ms)) / 1e3
    rank_kernel_ms = [kern_avg_s * 1e3]
    if sharded:
        cdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        s = torch.tensor([segs], dtype=torch.int64, device=cdev)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        segs_total = int(s.item())
        km = torch.zeros(world, dtype=torch.float64, device=cdev)
        km[rank] = kern_avg_s * 1e3
        dist.all_reduce(km, op=dist.ReduceOp.SUM)
        rank_kernel_ms = km.cpu().tolist()
    else:
        segs_total = segs
    gather_info = None
    if sharded:
        # this rank's gather (+ unshard on rank 0) per timed frame; the line reports rank 0's and the
        # slowest rank's mean
        if comm is not None:
            g_ms = [gev[i][0].elapsed_time(gev[i][1]) for i in range(args.warmup, n_total)]
        else:
            g_ms = gather_host_ms[args.warmup:n_total]
        gm = torch.tensor([float(np.mean(g_ms)), float(np.max(g_ms))], dtype=torch.float64, device=cdev)
        gmax = gm.clone()
        dist.all_reduce(gmax, op=dist.ReduceOp.MAX)
        gather_info = {"gather_ms": round(float(np.mean(g_ms)), 4), "gather_ms_max_frame": round(float(np.max(g_ms)), 4),
                       "gather_ms_slowest_rank": round(float(gmax[0].item()), 4),
                       "clock": "HIP events on the gather stream (rt_gather_shards + rt_unshard_tiles on rank 0)"
                       if comm is not None else "host clock around the synchronous gather + unshard (rehearsal)",
                       "overlapped_with_next_frame": comm is not None}

    seg_per_launch = segs / args.steps
    bytes_per_launch = bytes0 * (seg_per_launch / max(1, int(stats0[0])))
    final = frame if sharded else bufs[(n_total - 1) & 1]
    result = None
    if rank == 0:
        img = rt.surface_view(final, W)
        bad = (~torch.isfinite(img)).any(-1).nonzero()
        finite = bad.shape[0] == 0
        pmc, err = None, "PMC pass runs at N = 1 only (the rank-0 shard's counters are not the job's)"
        if world == 1:
            if args.no_pmc or under_profiler():
                err = "skipped (--no-pmc or already under a profiler)"
            else:
                with tempfile.TemporaryDirectory() as td:
                    pmc, err = pmc_pass(args, args.pmc_dir or td)
        roof = roofline(pmc, kern_avg_s, bytes_per_launch, err)
        roof["frame0_counts"] = {k: int(v) for k, v in zip(rt.STAT_NAMES, stats0) if k and int(v)}
        if prod0:
            roof["frame0_production"] = prod0
        result = {
            "metric": "Mrays/s + achieved HBM GB/s, Stanford bunny 1920x1080x8spp @1/2/4/8 GPU",
            "value": round(segs_total / elapsed / 1e6, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling if sharded else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference scene: Cornell box + Stanford bunny + HDR sky, seed 0xDEADBEEF)",
            "config": {"workload": desc, "scene": scene_name, "width": W, "height": H, "spp": SPP,
                       "bounces": BOUNCES, "parallelism": f"tiles{world}" if sharded else "single",
                       "camera_samples_per_s": round(W * H * SPP * args.steps / elapsed, 1),
                       "segments_per_step": round(segs_total / args.steps, 1), "tracer": args.tracer},
            "roofline": roof,
            "rank_kernel_ms": [round(x, 3) for x in rank_kernel_ms],
            "setup_s": round(setup_s, 2),
            "image_finite": finite,
        }
        if plan_info or sharded:
            result["plan"] = dict(plan_info or {"kind": "round-robin"},
                                  tiles_per_rank=[int(c) for c in counts] if sharded else None)
        if gather_kind:
            result["gather"] = gather_kind
            result.update(gather_info)
        if not finite:  # (y, x) of non-finite pixels; the reference arithmetic can produce them too
            result["nonfinite_pixels"] = bad[:8].tolist()
        if args.foreign:
            result["config"]["scene_path"] = "foreign GPUScene (fingerprint-gated private mirror)"
        if args.check:
            t_chk = time.perf_counter()
            result["check_equal"] = check_unsharded(rt, scene_name, W, H, SPP, BOUNCES, n_total, final)
            result["check"] = {"frames": n_total, "s": round(time.perf_counter() - t_chk, 2),
                               "against": "the same frames rendered unsharded in plain tile order (no cost order, "
                                          "no lane map) on this GPU, final surface compared bit for bit"}
            if fixture is not None:
                result["check_oracle_fixture"] = fixture
        if world == 1 and not args.no_cpu_baseline:
            auto_rows = {"cfg1": 256, "cfg2": 1080, "cfg3": 64, "cfg4": 540, "cfg5": 1080}[args.config]
            result["cpu_baseline"] = cpu_baseline_child(args.config, args.cpu_rows or auto_rows)
        print(json.dumps(result), flush=True)
        if args.check and not result["check_equal"]:
            print("bench.py: the timed frame differs from the unsharded plain render", file=sys.stderr, flush=True)
            exit_code = 3
        if fixture is not None and not fixture["equal"]:
            print("bench.py: frame 0 of the timed launch shape differs from the oracle fixture", file=sys.stderr, flush=True)
            exit_code = 3
    if comm is not None:
        torch.cuda.synchronize()
        comm.close()
    if sharded:
        dist.barrier()
        dist.destroy_process_group()
    wd.cancel()
    return exit_code


def foreign_copy(rt, scene):
    """A GPUScene whose arrays are fresh exact-size device allocations (as the reference's
    CUDA::DeviceMemory holds them) with the same contents: a scene this library never built."""
    import ctypes

    ha = scene.host_arrays()
    g = scene.gpu.contents
    f = rt.GPUScene()
    ctypes.pointer(f)[0] = g
    sizes = {"gpu_bvh_nodes": ha["nodes"].nbytes, "gpu_bvh_face_indices": ha["face_indices"].nbytes,
             "gpu_vertices": ha["vertices"].nbytes, "gpu_faces": ha["faces"].nbytes,
             "gpu_spheres": 32 * g.sphere_count, "gpu_materials": 64 * g.material_count}
    for k, n in sizes.items():
        p = ctypes.c_void_p()
        if rt.lib().rt_malloc(ctypes.byref(p), n) or rt.lib().rt_memcpy_d2d(p, ctypes.c_void_p(getattr(g, k)), n):
            raise RuntimeError(rt.lib().rt_last_error().decode())
        setattr(f, k, p.value)
    return f


FIXTURE = os.path.join(ROOT, "tests", "golden", "fullframe_oracle.json")


def fixture_rows(a):
    """Row hashes as tools/make_fullframe_golden.py makes them (NaN values as one canonical quiet NaN)."""
    import hashlib
    a = np.array(a, copy=True)
    if a.dtype == np.float32:
        a = a.view(np.uint32)
        a[(a & 0x7FFFFFFF) > 0x7F800000] = 0x7FC00000
    return [hashlib.sha256(np.ascontiguousarray(r).tobytes()).hexdigest()[:16] for r in a]


def check_oracle_fixture(rt, cfg, W, H, surface, rng):
    """Frame 0 of the timed launch shape itself (cost-ordered tiles, the measured lane map, the probed occupancy;
    its first warm-up frame, from the seeded RNG states) against the CPU oracle's own full frame: the row hashes
    of the frame and of every pixel's final RNG state in tests/golden/fullframe_oracle.json (data written once by
    tools/make_fullframe_golden.py from oracle/rt_oracle.c).  None when there is no fixture for this config."""
    if not os.path.exists(FIXTURE):
        return None
    g = json.load(open(FIXTURE)).get(cfg)
    if not g or (g["width"], g["height"]) != (W, H):
        return None
    img = rt.surface_view(surface, W).cpu().numpy().reshape(H, W, 4)
    st = rng.view(-1, 12)[:, :6].cpu().numpy().view(np.uint32).reshape(H, W, 6)
    bad = sum(a != b for a, b in zip(fixture_rows(img), g["rows"]))
    bad_rng = sum(a != b for a, b in zip(fixture_rows(st), g["rng_rows"]))
    return {"equal": bad == 0 and bad_rng == 0, "frame": 0, "rows": H, "differing_rows": int(bad),
            "differing_rng_rows": int(bad_rng), "against": "tests/golden/fullframe_oracle.json (the oracle's full frame 0)"}


def check_unsharded(rt, scene_name, W, H, spp, bounces, frames, final):
    """Render the same frames on this GPU without sharding (fresh RNG) and compare bit for bit."""
    import torch

    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    rng = rt.alloc_rng(W * H)
    rt.init_rng_states(rng, W, H, SEED)
    scene.upload(rng.data_ptr())
    bufs = [rt.alloc_surface(W, H) for _ in range(2)]
    for i in range(frames):
        rt.render(scene, bufs[i & 1], bufs[(i + 1) & 1], W, H, spp, bounces, i)
    torch.cuda.synchronize()
    # bitwise (same GPU, so NaNs from the reference arithmetic carry the same bits too)
    a = rt.surface_view(bufs[(frames - 1) & 1], W).contiguous().view(torch.int32)
    return bool(torch.equal(a, rt.surface_view(final, W).contiguous().view(torch.int32)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 --pmc pass (roofline.frac = null)")
    ap.add_argument("--pmc-dir", default=None, help="keep the PMC pass's rocprofv3 output here")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-rows", type=int, default=0, help="rows of the frame the CPU baseline renders (0 = auto)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--gather", default="rccl", choices=["rccl", "torch"],
                    help="frame gather: rt_gather_shards over RCCL (C-ABI) or torch.distributed.gather")
    ap.add_argument("--same-device", action="store_true", help="every rank on GPU 0 (rehearsal on a one-GPU box)")
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="N > 1: strong = the BASELINE frame split N ways; weak = sqrt(N) x resolution per axis")
    ap.add_argument("--plan", default=None, choices=["cost", "rr"],
                    help="tile order / deal: cost (default: a probe frame's per-wave clocks, heaviest tiles first, "
                         "longest-processing-time deal over ranks) or round-robin in row-major order")
    ap.add_argument("--refill", type=int, default=0,
                    help="rt_render refill_lanes: a wave refills this many idle lanes from the frame's queue (0 = off)")
    ap.add_argument("--occupancy", default="auto", choices=["auto", "1", "2", "3", "4", "5", "6", "7"],
                    help="rt_render waves_per_simd (1-4: the 5-wave build capped at that residency by dynamic LDS); "
                         "auto = time one untimed frame at 5 / 6 / 7 (N > 1: also 3 / 4) and keep the fastest")
    ap.add_argument("--lanes", default="auto", choices=["auto", "on", "off"],
                    help="lane plan (rt_lane_plan: split the waves of the frame's costliest pixels, then --lane-refine "
                         "rounds of measured refinement); auto = on (config 2 at N = 1: 14.1-14.3 vs 15.5-15.8 ms)")
    ap.add_argument("--lane-map-file", default=None, help=argparse.SUPPRESS)  # PMC child: the parent's lane map
    ap.add_argument("--lane-refine", type=int, default=5,
                    help="rounds of measured lane-plan refinement whenever a lane plan is on (rt_lane_refine; 0 = the model's plan only)")
    ap.add_argument("--lane-theta", type=float, default=0.85,
                    help="rt_lane_refine theta: waves measured within this fraction of the longest are split")
    ap.add_argument("--lane-units", type=float, default=48000.0,
                    help="rt_lane_plan parallel_units (MI355X: 48000 measured best for configs 2 and 3 at N = 2-8)")
    ap.add_argument("--tune", type=lambda s: int(s, 0), default=0, help="diagnostic A/B knobs (0 = production)")
    ap.add_argument("--tracer", default="fast", choices=["fast", "wavefront"],
                    help="render path of the timed frames: the production kernel or the wavefront tracer (A/B)")
    ap.add_argument("--foreign", action="store_true",
                    help="render a GPUScene filled outside this library (the reference's Scene::Upload pattern): "
                         "fingerprint-gated mirror, no host synchronisation per frame")
    ap.add_argument("--build-options", default="",
                    help="rt_set_build_options fields, e.g. leaf_tree_min=300,cluster_max=16 (exact-preserving A/B)")
    ap.add_argument("--rank-deadline", type=float, default=480.0,
                    help="N > 1: seconds after which a still-running job is killed whole (0 = none)")
    ap.add_argument("--check", dest="check", action="store_true", default=True,
                    help="(default) after timing, rank 0 re-renders the same frames unsharded, plain tile order, "
                         "and compares the final frame bit for bit with the timed one (N > 1: the gathered frame)")
    ap.add_argument("--no-check", dest="check", action="store_false", help="skip the bit-exact check")
    ap.add_argument("--cpu-baseline-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.cpu_baseline_child:  # the CPU baseline's own process (see cpu_baseline_child)
        print(json.dumps(cpu_baseline(args.config, args.cpu_rows or None)), flush=True)
        return 0
    if args.plan is None:
        args.plan = "cost"
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.pmc_child:
        return launch_ranks(args.gpus, deadline_s=args.rank_deadline)
    return run(args)


if __name__ == "__main__":
    sys.exit(main())
