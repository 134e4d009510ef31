"""Per-wave critical-path model of the strong-scaled frame.

A wave of the production kernel is one serial instruction chain (a lane's samples run back to back,
main_raytracing.cu:188-193; the wave steps through the union of its lanes' chains).  The model:

    duration of wave w  =  integral of  dt / max(1, k(t) / k0)   until  A(w)  has been consumed,

A(w) = the wave's chain measured ALONE on its SIMD (the 5-wave build capped at one resident wave per
SIMD by dynamic LDS, rt_render_params.waves_per_simd = 1: its per-wave s_memrealtime clock), k(t) =
the waves resident on its SIMD at time t, and k0 = the residency at which one SIMD's issue saturates:
alone, a wave issues a dependent VALU instruction every ~8.2 cycles, and the SIMD issues one every
~1.8 cycles once ~5 waves share it (profiles/r03a_valu_microbench.txt), so k0 = 8.2 / 1.8 = 4.6 --
a wave slows by k / k0 once more than k0 waves share its SIMD.  Waves are dispatched in workgroup
order, wave g to SIMD g mod 1024, up to `slots` per SIMD (7 at the 7-wave build), and a finished wave's
slot takes the next one.  The shard time is the last finish.

    python tools/wave_model.py --measure --ns 1,2,4,8 --out gpurun_out/wave_model.npz   (GPU box)
    python tools/wave_model.py --model profiles/r04_wave_model.npz                        (anywhere)

--measure renders each rank's shard of the bench's cost plan with the bench's refined lane map
(rt_lane_plan + 5 rounds of rt_lane_refine, theta 0.85) and records over the same 3 frames: the shard
time at 7 waves per SIMD (HIP events), every wave's clock at 7 waves per SIMD, and every wave's clock
alone (cap 1).
"""
import argparse
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

SIMDS = 1024
CLOCK_HZ = 100e6  # wave_clock ticks (s_memrealtime)


DISPATCH = "rr"  # initial placement: "rr" wave g -> SIMD g mod 1024; "fill" 7 per SIMD in order; "xcd" see below


def initial_simd(i):
    """SIMD of the i-th dispatched wave (i < slots x SIMDs)."""
    if DISPATCH == "fill":
        return i // SLOTS
    if DISPATCH == "xcd":  # round-robin over the 8 XCDs, then over each XCD's 32 CUs, then a CU's 4 SIMDs
        x, j = i % 8, i // 8
        cu, k = j % 32, j // 32
        return ((x * 32 + cu) * 4 + k % 4) % SIMDS
    return i % SIMDS


SLOTS = 7
C0 = 1e9  # CU-level saturation (waves per CU at which the CU's shared memory path saturates); off by default


def simulate(alone_ms, k0, slots, order=None):
    """Processor-sharing simulation of one launch: `alone_ms[g]` = wave g's chain alone (ms), waves
    dispatched in order g = 0, 1, ... to SIMD g mod SIMDS while slots last, then into freed slots.
    Returns (finish time of every wave, the SIMD each ran on)."""
    n = len(alone_ms)
    order = np.arange(n) if order is None else order
    rem = np.asarray(alone_ms, dtype=np.float64).copy()
    finish = np.zeros(n)
    simd_of = np.full(n, -1)
    resident = [[] for _ in range(SIMDS)]
    t_last = np.zeros(SIMDS)  # time of the SIMD's last update
    nxt = 0
    heap = []  # (predicted finish, simd, version)
    version = np.zeros(SIMDS, dtype=np.int64)

    cu_n = np.zeros(SIMDS // 4, dtype=np.int64)  # waves resident per CU (4 SIMDs)

    def rate(s):
        return 1.0 / max(1.0, len(resident[s]) / k0, cu_n[s // 4] / C0)

    def advance(s, t):
        r = rate(s) if resident[s] else 0.0
        for w in resident[s]:
            rem[w] -= (t - t_last[s]) * r
        t_last[s] = t

    def schedule(s):
        version[s] += 1
        if resident[s]:
            w = min(resident[s], key=lambda x: rem[x])
            heapq.heappush(heap, (t_last[s] + max(rem[w], 0.0) / rate(s), s, version[s]))

    # initial dispatch (DISPATCH), `slots` deep
    global SLOTS
    SLOTS = slots
    while nxt < n and nxt < slots * SIMDS:
        s = initial_simd(nxt)
        if len(resident[s]) >= slots:  # placement collision: the next SIMD with a free slot
            s = next(t % SIMDS for t in range(s, s + SIMDS) if len(resident[t % SIMDS]) < slots)
        g = order[nxt]
        resident[s].append(g)
        simd_of[g] = s
        nxt += 1
    for s in range(SIMDS):
        cu_n[s // 4] += len(resident[s])
    for s in range(SIMDS):
        schedule(s)
    while heap:
        t, s, v = heapq.heappop(heap)
        if v != version[s]:
            continue
        cu = s // 4
        for q in range(4 * cu, 4 * cu + 4):  # the CU's SIMDs share the CU term: bring them all to t
            advance(q, t)
        done = [w for w in resident[s] if rem[w] <= 1e-12]
        if not done:  # numerical slack
            done = [min(resident[s], key=lambda x: rem[x])]
        for w in done:
            resident[s].remove(w)
            finish[w] = t
            cu_n[cu] -= 1
            if nxt < n:  # the freed slot takes the next wave in dispatch order
                g = order[nxt]
                resident[s].append(g)
                simd_of[g] = s
                cu_n[cu] += 1
                nxt += 1
        for q in range(4 * cu, 4 * cu + 4):
            schedule(q)
    return finish, simd_of


GDEV = 0.0  # device-load term (--c-dev): rate / ((1 + GDEV D) / (1 + GDEV / slots)), D = resident / (SIMDS x slots)


def simulate_dt(alone_ms, k0, slots, order=None, dt=0.004):
    """simulate() as a time-stepped, vectorised processor-sharing simulation (steps of `dt` ms), which
    also carries the device-load term: a wave on a SIMD with k resident waves progresses at
    1 / max(1, k / k0), divided by (1 + GDEV D) / (1 + GDEV / slots) where D is the fraction of the
    device's wave slots in use -- the alone measurement (one wave per SIMD) is the reference point.
    Same placement as simulate(): wave i of the dispatch order to SIMD i mod SIMDS, `slots` deep, a
    freed slot takes the next wave.  Returns the finish time of every wave (in `order`'s numbering)."""
    n = len(alone_ms)
    order = np.arange(n) if order is None else np.asarray(order)
    rem = np.asarray(alone_ms, dtype=np.float64)[order].copy()  # dispatch order
    slot = np.full((SIMDS, slots), -1, dtype=np.int64)
    m = min(n, slots * SIMDS)
    i = np.arange(m)
    slot[i % SIMDS, i // SIMDS] = i
    nxt, t = m, 0.0
    fin = np.zeros(n)
    ref = 1.0 + GDEV / slots
    while True:
        occ = slot >= 0
        k = occ.sum(1)
        tot = int(k.sum())
        if tot == 0:
            break
        r = 1.0 / (np.maximum(1.0, k / k0) * (1.0 + GDEV * tot / (SIMDS * slots)) / ref)
        ids = slot[occ]
        rem[ids] -= dt * np.broadcast_to(r[:, None], slot.shape)[occ]
        t += dt
        done = ids[rem[ids] <= 0]
        if done.size:
            fin[done] = t
            pos = np.argwhere(np.isin(slot, done))
            slot[pos[:, 0], pos[:, 1]] = -1
            take = min(len(pos), n - nxt)
            if take > 0:
                slot[pos[:take, 0], pos[:take, 1]] = np.arange(nxt, nxt + take)
                nxt += take
    out = np.zeros(n)
    out[order] = fin
    return out


def xcd_order(waves):
    """Logical wave index of hardware workgroup g (rt_fast_body.h xcd_block, runs of 32 per XCD)."""
    S = 32
    full = waves // (8 * S) * (8 * S)
    g = np.arange(waves)
    i, x = g >> 3, g & 7
    lb = np.where(g < full, ((i // S) * 8 + x) * S + i % S, g)
    return lb


def measure(args):
    import torch

    import __graft_entry__ as G
    import bench
    import shard_timing as ST

    rt = G.load_package()
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    cost = ST.probe(rt, scene, W, H, SPP, BOUNCES)
    ST.REFINE, ST.THETA, ST.WPS = args.refine, args.theta, args.wps
    out = {}
    for n in map(int, args.ns.split(",")):
        lists, counts = rt.shard_plan(W, H, n, cost)
        for r in range(n):
            mine = torch.from_numpy(lists[r, : counts[r]]).cuda()
            rng = rt.alloc_rng(mine.numel() * 256)
            rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
            scene.upload(rng.data_ptr())
            lm, nlong, _ = ST.lane_map(rt, scene, W, H, SPP, BOUNCES, mine, rng, (args.units, 1.0))
            saved = rng.clone()
            buf = torch.zeros((mine.numel() * 256, 4), dtype=torch.float32, device="cuda")
            waves = lm.numel() // 64 if lm is not None else mine.numel() * 4

            def frames(clock=True, **kw):
                """three consecutive frames of the RNG chain from the saved states: per-frame event
                time and per-frame wave clocks (frames differ -- each its own random paths -- and the
                same three frames are replayed for every occupancy)"""
                ms, per = [], []
                clk = torch.zeros(waves, dtype=torch.int64, device="cuda")
                if clock:
                    kw["wave_clock"] = clk
                for f in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, 0, 1, out_shard=buf, tile_list=mine, lane_slots=lm,
                              **kw)
                    e1.record()
                    torch.cuda.synchronize()
                    ms.append(e0.elapsed_time(e1))
                    per.append(bench.sanitize_wave_clocks(clk.cpu().numpy())[0] / CLOCK_HZ * 1e3)
                rng.copy_(saved)
                return np.array(ms), np.array(per)

            shard_ms = float(np.mean([frames(clock=False, waves_per_simd=args.wps)[0].mean() for _ in range(2)]))
            full_frames_ms, full_per = frames(waves_per_simd=args.wps)
            alone_frames_ms, alone_per = frames(waves_per_simd=1)
            full_ms, alone_shard_ms = float(full_frames_ms.mean()), float(alone_frames_ms.mean())
            t_full, t_alone = full_per.mean(0), alone_per.mean(0)
            out[f"n{n}_r{r}_frames_ms"] = full_frames_ms
            out[f"n{n}_r{r}_alone_per_frame"] = alone_per.astype(np.float32)
            out[f"n{n}_r{r}_full_per_frame"] = full_per.astype(np.float32)
            # one timing frame (RT_TUNE 256 + 2048) at the same occupancy: every wave's start and end on
            # the 100 MHz device clock, indexed by hardware workgroup (dispatch order)
            st = torch.zeros(rt.STAT_COUNT + 8 * waves, dtype=torch.int64, device="cuda")
            rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, 0, 1, out_shard=buf, tile_list=mine, lane_slots=lm,
                      stats=st, tune=256 | 2048, waves_per_simd=args.wps)
            torch.cuda.synchronize()
            rng.copy_(saved)
            rec = st[rt.STAT_COUNT:].view(-1, 8).cpu().numpy()
            t0 = rec[:, 0].min()
            out[f"n{n}_r{r}_start"] = (rec[:, 0] - t0) / CLOCK_HZ * 1e3
            out[f"n{n}_r{r}_end"] = (rec[:, 1] - t0) / CLOCK_HZ * 1e3
            pix = (lm.view(-1, 64) >= 0).sum(1).cpu().numpy() if lm is not None else np.full(waves, 64)
            key = f"n{n}_r{r}"
            out[key + "_full"], out[key + "_alone"], out[key + "_pixels"] = t_full, t_alone, pix
            out[key + "_meta"] = np.array([shard_ms, full_ms, alone_shard_ms, n, r, waves])
            se, ee = out[f"n{n}_r{r}_start"], out[f"n{n}_r{r}_end"]
            print(json.dumps({"n": n, "rank": r, "timing_frame": {"start_ms_p50_p99_max": [round(float(np.percentile(se, q)), 4) for q in (50, 99, 100)],
                                                                 "last_end_ms": round(float(ee.max()), 3),
                                                                 "longest_ms": round(float((ee - se).max()), 3),
                                                                 "end_of_longest_ms": round(float(ee[np.argmax(ee - se)]), 3)}}), flush=True)
            print(json.dumps({"n": n, "rank": r, "waves": int(waves), "shard_ms": round(shard_ms, 3),
                              "clocked_frame_ms": round(full_ms, 3), "capped1_frame_ms": round(alone_shard_ms, 3),
                              "wave_full_ms_max": round(float(t_full.max()), 3), "wave_alone_ms_max": round(float(t_alone.max()), 3),
                              "sum_alone_ms": round(float(t_alone.sum()), 1)}), flush=True)
    np.savez_compressed(args.out, **out)


def fit_k0(args):
    """The free constants -- k0, and the device-load term GDEV with --fit-dev -- fitted to the measured
    shard times of the N in --fit-ns only (least squares in log space over the slowest rank of each N),
    beside the microbenchmark's k0 = 8.2 / 1.8; the other N are then out of sample."""
    global GDEV
    fit_ns = {int(x) for x in args.fit_ns.split(",")}
    best = None
    for g in ((0.0, 0.25, 0.5, 1.0, 1.5, 2.0) if args.fit_dev else (GDEV,)):
        GDEV = g
        for k0 in np.arange(3.5, 7.01, 0.25):
            a = argparse.Namespace(**vars(args))
            a.k0 = float(k0)
            s = model(a, quiet=True, ns=fit_ns)
            err = sum(np.log(v["model_ms"] / v["measured_ms"]) ** 2 for v in s.values())
            if best is None or err < best[0]:
                best = (err, float(k0), g)
    GDEV = best[2]
    return best[1]


def model(args, quiet=False, ns=None):
    d = np.load(args.model)
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_meta")})
    rows = []
    for key in keys:
        meta = d[key + "_meta"]
        shard_ms, n, r, waves = float(meta[0]), int(meta[3]), int(meta[4]), int(meta[5])
        if ns is not None and n not in ns:
            continue
        alone, full, pix = d[key + "_alone"], d[key + "_full"], d[key + "_pixels"]
        lb = xcd_order(waves)  # hardware dispatch order g -> logical wave lb
        if key + "_alone_per_frame" in d.files:
            # frame by frame: each frame's own waves (the longest wave differs from frame to frame, and
            # a strong-scaled frame ends with its longest), against that frame's measured time
            per = d[key + "_alone_per_frame"].astype(np.float64)
            preds = [float(simulate_dt(a, args.k0, args.slots, order=lb).max()) for a in per[: (1 if quiet else len(per))]]
            shard_ms = float(d[key + "_frames_ms"][: len(preds)].mean())
            if quiet:
                rows.append({"n": n, "rank": r, "measured_ms": shard_ms, "model_ms": float(np.mean(preds))})
                continue
            fin, simd = simulate(per[int(np.argmax(preds))], args.k0, args.slots, order=lb)
            alone = per[int(np.argmax(preds))]
            pred = float(np.mean(preds))
        else:
            fin, simd = simulate(alone, args.k0, args.slots, order=lb)
            pred = float(simulate_dt(alone, args.k0, args.slots, order=lb).max())
            if quiet:
                rows.append({"n": n, "rank": r, "measured_ms": shard_ms, "model_ms": pred})
                continue
        crit = int(simd[int(np.argmax(fin))])
        on = np.flatnonzero(simd == crit)
        rows.append({"n": n, "rank": r, "waves": waves, "measured_ms": round(shard_ms, 3), "model_ms": round(pred, 3),
                     "err": round(pred / shard_ms - 1, 3),
                     "critical_simd": {"waves": int(on.size), "alone_ms": [round(float(x), 3) for x in np.sort(alone[on])[::-1]],
                                       "pixels": [int(pix[w]) for w in on[np.argsort(-alone[on])]]},
                     "longest_alone_ms": round(float(alone.max()), 3),
                     "mean_waves_per_simd": round(waves / SIMDS, 2),
                     "slowdown_measured_p50": round(float(np.median(full / np.maximum(alone, 1e-9))), 3)})
    by_n = {}
    for row in rows:
        by_n.setdefault(row["n"], []).append(row)
    summary = {str(n): {"measured_ms": max(x["measured_ms"] for x in v), "model_ms": max(x["model_ms"] for x in v)}
               for n, v in sorted(by_n.items())}
    for v in summary.values():
        v["err"] = round(v["model_ms"] / v["measured_ms"] - 1, 3)
    if quiet:
        return summary
    for row in rows:
        print(json.dumps(row))
    print(json.dumps({"k0": args.k0, "device_load_term": GDEV, "slots": args.slots,
                      "fitted_on_n": args.fit_ns if args.fit else None, "per_n_slowest_rank": summary}))
    return summary


def whatif(args):
    """The model's answer to the two levers, on the slowest rank of every N (its first measured frame, with
    the run's k0 and device-load term): every chain shorter by 10 / 20 / 30 % (a faster kernel), or the
    waves above a threshold split in two halves of 0.79x their alone time each (the measured cost of
    halving a wave's pixels), dispatched longest first."""
    d = np.load(args.model)
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_meta")})
    worst = {}
    for key in keys:
        meta = d[key + "_meta"]
        n = int(meta[3])
        if n not in worst or meta[0] > d[worst[n] + "_meta"][0]:
            worst[n] = key
    for n, key in sorted(worst.items()):
        per = key + "_alone_per_frame"
        a = d[per][0].astype(np.float64) if per in d.files else d[key + "_alone"].astype(np.float64)
        meas = float(d[key + "_frames_ms"][0]) if per in d.files else float(d[key + "_meta"][0])
        lb = xcd_order(len(a))
        sim = lambda x, o=lb: round(float(simulate_dt(x, args.k0, args.slots, order=o).max()), 3)
        out = {"n": n, "rank": int(d[key + "_meta"][4]), "measured_ms": round(meas, 3), "model_ms": sim(a)}
        for f in (0.9, 0.8, 0.7):
            out[f"chain_x{f}"] = sim(a * f)
        for thr in (3.0, 2.5, 2.0):
            big = a > thr
            b = np.concatenate([a[~big], np.repeat(a[big] * 0.79, 2)])
            b = b[np.argsort(-b)]
            out[f"split_above_{thr}ms"] = [sim(b, None), int(b.size)]
        print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--measure", action="store_true")
    ap.add_argument("--model", default=None)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--refine", type=int, default=5)
    ap.add_argument("--theta", type=float, default=0.85)
    ap.add_argument("--units", type=float, default=48000.0)
    ap.add_argument("--wps", type=int, default=7)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "wave_model.npz"))
    ap.add_argument("--k0", type=float, default=8.2 / 1.8)
    ap.add_argument("--slots", type=int, default=7)
    ap.add_argument("--fit", action="store_true", help="fit k0 (and the device-load term with --fit-dev) to the "
                    "measured shard times of --fit-ns instead; the other N are out of sample")
    ap.add_argument("--fit-ns", default="1,2,4")
    ap.add_argument("--fit-dev", action="store_true")
    ap.add_argument("--c-dev", type=float, default=0.0, help="device-load term (simulate_dt)")
    ap.add_argument("--dispatch", default="rr", choices=["rr", "fill", "xcd"], help="initial wave placement")
    ap.add_argument("--c0", type=float, default=0.0, help="CU-level saturation in waves per CU (0 = off)")
    ap.add_argument("--whatif", action="store_true", help="also price the two levers (shorter chains, split waves)")
    args = ap.parse_args()
    global DISPATCH, C0, GDEV
    DISPATCH = args.dispatch
    GDEV = args.c_dev
    C0 = args.c0 if args.c0 > 0 else 1e9
    if args.measure:
        measure(args)
    if args.model:
        if args.fit:
            args.k0 = fit_k0(args)
        model(args)
        if args.whatif:
            whatif(args)


if __name__ == "__main__":
    main()
