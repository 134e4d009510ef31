"""Benchmark of the hot path: one "step" = one progressive frame of the per-pixel path tracer
(RayTracing/main_raytracing.cu:162-200 via raytracing_process) over the whole frame.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2]

N = 1 runs BASELINE.json configs[1] (Stanford bunny scene, 1920x1080, 8 spp, 6 bounces).
N > 1 (launched by torch.distributed.run, one process per GPU): the frame is cut into 16x16
tiles dealt round-robin over the ranks; each rank renders its tiles into a compact shard, and
one RCCL gather over xGMI assembles the frame on rank 0, where a kernel un-permutes it into the
pitched surface.  The gather of frame i runs on its own stream, overlapped with the render of
frame i+1 (each rank keeps its own shard history, so the next frame does not wait for it).
  --scaling weak (default): per-GPU work fixed -- the same camera at sqrt(N) x the resolution
      per axis (N = 4: 3840x2160), so each rank renders about one 1920x1080 frame of tiles.
  --scaling strong: the 1920x1080 frame itself split N ways.  Its speedup is capped by the
      heaviest pixel: samples of a pixel share one RNG stream and run in order, and the
      costliest pixel's 8 samples take ~11 ms alone ("Multi-GPU").
Timing: barrier + synchronize on both sides of exactly K steps, max over ranks.

Rank 0 prints one JSON line.  value = ray segments traced (GetRayHit calls, counted exactly by
the kernel) per second over the whole job, in Mrays/s.  roofline = the render kernel's
algorithmic bytes per launch (SURVEY.md section 8(d) formula, from an exact traversal count)
over its HIP-event-timed average duration, against the 8 TB/s HBM peak.  cpu_baseline = the
CPU restatement of the reference (oracle/, "port") on this host's cores, same scene and seed.
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402

CONFIGS = {
    # name: (scene, width, height, spp, bounces, description)
    "cfg1": ("bunny", 256, 256, 1, 1, "stanford-bunny 256x256 1spp primary rays (BASELINE configs[0])"),
    "cfg2": ("bunny", 1920, 1080, 8, 6, "stanford-bunny 1920x1080 8spp (BASELINE configs[1])"),
    "cfg3": ("bunny", 3840, 2160, 64, 6, "stanford-bunny 3840x2160 64spp (BASELINE configs[2])"),
    "cfg4": ("bunny4", 1920, 1080, 8, 6, "4x instanced bunny 1920x1080 8spp (BASELINE configs[3])"),
    "cfg5": ("plane1m", 1920, 1080, 1, 6, "1M-triangle plane 1920x1080 1spp (BASELINE configs[4])"),
}
SEED = 0xDEADBEEF
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def algorithmic_bytes(stats, sphere_count, pixels):
    """per segment 32 B per BVH node visited, 56 B per triangle test
    (4 B index + 16 B face + 3 x 12 B positions), 32 B per sphere tested, 64 B material per
    accepted hit, 36 B (3 normals) per accepted triangle hit; per pixel 48 B RNG state
    read+write and 32 B surface read+write."""
    seg, nodes, tris, tacc, sacc = (int(stats[i]) for i in range(5))
    return (32 * nodes + 56 * tris + 32 * sphere_count * seg + 64 * (tacc + sacc) + 36 * tacc + 80 * pixels)


def setup_dist(backend="nccl", same_device=False):
    """One process per GPU (torch.distributed.run sets RANK / LOCAL_RANK / WORLD_SIZE); the
    "nccl" backend is RCCL on ROCm.  --backend gloo --same-device rehearses the N > 1 path with
    every rank on GPU 0 (a one-GPU box), staging the gather through host memory."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if same_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return rank, world


def weak_size(width, height, world):
    """The weak-scaled frame for N ranks: sqrt(N) x the resolution per axis, width a multiple of
    the 16-pixel tile, aspect kept (1920x1080: N=2 2720x1530, N=4 3840x2160, N=8 5424x3051)."""
    if world <= 1:
        return width, height
    w = int(round(width * world ** 0.5 / 16.0)) * 16
    return w, int(round(w * height / width))


def cpu_baseline(cfg, sample_rows=None):
    """Oracle ("port") on this host's cores: bounded sample of the same frame (rows)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rt_testlib as T

    scene_name, w, h, spp, bounces, _ = CONFIGS[cfg]
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
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
    return {"value": round(float(st[0]) / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{cfg} rows [{r0},{r1}) of {h} ({samples} camera samples, {int(st[0])} segments), {dt:.1f} s",
            "samples_per_s": round(samples / dt, 1)}


def check_unsharded(rt, scene_name, W, H, spp, bounces, frames, final):
    """Render the same frames on this GPU without sharding (fresh RNG) and compare bit for bit."""
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


def load_issue(cfg):
    """The render kernel's issue-side counters from the committed PMC summary: the path is
    VALU-issue bound (the scene lives in L2 / Infinity Cache), so the HBM fraction alone does not
    say how close the kernel is to its limit."""
    out = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(path))
            c = d["kernels"][d["kernel"]]["counters"]
        except Exception:
            continue
        if d.get("config") == cfg:
            out = {"bound": "valu", "valu_busy": round(c["VALUBusy"] / 100.0, 3),
                   "lane_utilization": round(c["VALUUtilization"] / 100.0, 3),
                   "valu_wave_instructions_per_launch": int(c["SQ_INSTS_VALU"]),
                   "l2_hit_rate": round(d.get("l2_hit_rate", 0.0), 3),
                   "source": os.path.relpath(path, ROOT)}
    return out


def load_traffic(cfg):
    """HBM bytes per render launch from a committed PMC summary (profiles/*pmc*.json), if any."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("config") == cfg and "hbm_bytes_per_launch" in d:
            best = d["hbm_bytes_per_launch"]
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=0, help="rows of the frame the CPU baseline renders (0 = auto)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--same-device", action="store_true", help="every rank on GPU 0 (rehearsal on a one-GPU box)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N > 1: weak = sqrt(N) x resolution per axis (per-GPU work fixed); strong = same frame")
    ap.add_argument("--check", action="store_true",
                    help="after timing, rank 0 re-renders the same frames unsharded and compares the final frame")
    args = ap.parse_args()

    rank, world = setup_dist(args.backend, args.same_device)
    assert world == args.gpus or world == 1, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    rt = G.load_package()
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
    if sharded:
        tiles = rt.shard_tiles(W, H, rank, world)
        per_shard = max(rt.shard_tiles(W, H, r, world) for r in range(world))
        rng = rt.alloc_rng(per_shard * 256)
        rt.init_rng_states(rng, W, H, SEED, rank, world)
        bufs = [torch.zeros((per_shard * 256, 4), dtype=torch.float32, device=dev) for _ in range(2)]
        gathered = torch.empty((world, per_shard * 256, 4), dtype=torch.float32, device=dev) if rank == 0 else None
        frame = rt.alloc_surface(W, H) if rank == 0 else None
    else:
        tiles = rt.shard_tiles(W, H, 0, 1)
        per_shard = tiles
        rng = rt.alloc_rng(W * H)
        rt.init_rng_states(rng, W, H, SEED)
        bufs = [rt.alloc_surface(W, H) for _ in range(2)]
    scene.upload(rng.data_ptr())
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    pixels_rank = tiles * 256 if sharded else W * H

    # --- exact traversal counts of one frame (stats kernel variant) on a copy of the RNG state
    rng_saved = rng.clone()
    stats = torch.zeros(24, dtype=torch.int64, device=dev)
    if sharded:
        rt.render(scene, None, bufs[1], W, H, SPP, BOUNCES, 0, rank, world, out_shard=bufs[0], stats=stats)
    else:
        rt.render(scene, bufs[0], bufs[1], W, H, SPP, BOUNCES, 0, stats=stats)
    torch.cuda.synchronize()
    rng.copy_(rng_saved)
    del rng_saved
    stats0 = stats.cpu().numpy().astype(np.uint64)
    gpu = scene.gpu.contents
    bytes0 = algorithmic_bytes(stats0, gpu.sphere_count, pixels_rank)

    seg_counter = torch.zeros(1, dtype=torch.int64, device=dev)
    n_total = args.warmup + args.steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_total)]

    # gather/render overlap (RCCL only; the gloo rehearsal stages through host memory in line)
    comm = torch.cuda.Stream() if sharded and args.backend == "nccl" else None
    rendered = torch.cuda.Event()
    gathered_ev = [torch.cuda.Event(), torch.cuda.Event()]  # the gather that last read bufs[j]
    gather_pending = [False, False]

    def step(i):
        cur, prev = bufs[i & 1], bufs[(i + 1) & 1]
        if comm is not None and gather_pending[i & 1]:
            stream.wait_event(gathered_ev[i & 1])  # frame i-2's gather still reads `cur`
        ev[i][0].record(stream)
        if sharded:
            rt.render(scene, None, prev, W, H, SPP, BOUNCES, i, rank, world, out_shard=cur,
                      segment_counter=seg_counter if i >= args.warmup else None)
        else:
            rt.render(scene, cur, prev, W, H, SPP, BOUNCES, i,
                      segment_counter=seg_counter if i >= args.warmup else None)
        ev[i][1].record(stream)
        if comm is not None:
            rendered.record(stream)
            comm.wait_event(rendered)
            with torch.cuda.stream(comm):
                rt.sharding.gather_shards(cur, rank, world, out=gathered)
                if rank == 0:
                    rt.unshard(frame, W, H, world, gathered, per_shard)
                gathered_ev[i & 1].record(comm)
            gather_pending[i & 1] = True
        elif sharded:
            rt.sharding.gather_shards(cur, rank, world, out=gathered)
            if rank == 0:
                rt.unshard(frame, W, H, world, gathered, per_shard)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.warmup, n_total):
        step(i)
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start

    segs = int(seg_counter.item())
    kern_ms = [ev[i][0].elapsed_time(ev[i][1]) for i in range(args.warmup, n_total)]
    kern_avg_s = float(np.mean(kern_ms)) / 1e3
    if sharded:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        s = torch.tensor([segs], dtype=torch.int64, device=dev)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        segs_total = int(s.item())
    else:
        segs_total = segs

    # algorithmic bytes per timed launch: frame-0 exact counts scaled by the exact segment ratio
    seg_per_launch = segs / args.steps
    bytes_per_launch = bytes0 * (seg_per_launch / max(1, int(stats0[0])))
    achieved = bytes_per_launch / kern_avg_s / 1e9
    final = (frame if sharded else bufs[(n_total - 1) & 1])
    if rank == 0:
        img = rt.surface_view(final, W)
        bad = (~torch.isfinite(img)).any(-1).nonzero()
        finite = bad.shape[0] == 0
        result = {
            "metric": "Mrays/s + achieved HBM GB/s, Stanford bunny 1920x1080x8spp @1/2/4/8 GPU",
            "value": round(segs_total / elapsed / 1e6, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling if sharded else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference scene: Cornell box + Stanford bunny + HDR sky, seed 0xDEADBEEF)",
            "config": {"workload": desc, "scene": scene_name, "width": W, "height": H, "spp": SPP,
                       "bounces": BOUNCES, "parallelism": f"tiles{world}" if sharded else "single",
                       "camera_samples_per_s": round(W * H * SPP * args.steps / elapsed, 1),
                       "segments_per_step": round(segs_total / args.steps, 1)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(args.config),
                         "issue": load_issue(args.config),
                         "kernel": "render_fast_kernel", "kernel_ms": round(kern_avg_s * 1e3, 3),
                         "algorithmic_bytes_per_launch": int(bytes_per_launch),
                         "frame0_counts": {k: int(v) for k, v in zip(rt.STAT_NAMES, stats0) if k}},
            "setup_s": round(setup_s, 2),
            "image_finite": finite,
        }
        if not finite:  # (y, x) of non-finite pixels; the reference arithmetic can produce them too
            result["nonfinite_pixels"] = bad[:8].tolist()
        if args.check:
            result["check_equal"] = check_unsharded(rt, scene_name, W, H, SPP, BOUNCES, n_total, final)
        if world == 1 and not args.no_cpu_baseline:
            auto_rows = {"cfg1": 256, "cfg2": 1080, "cfg3": 64, "cfg4": 540, "cfg5": 1080}[args.config]
            result["cpu_baseline"] = cpu_baseline(args.config, args.cpu_rows or auto_rows)
        print(json.dumps(result), flush=True)
    if sharded:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
