#!/usr/bin/env python3
"""Benchmark: WoS walk-steps/sec + pressure-projection wall-time per step,
2D karman 64k points x 128 walks (BASELINE.json configs[1] / metric).

One "step" = one pressure projection: the walk-on-stars solve over every query
point (inputs already resident in HBM) followed, for N>1 GPUs, by the single
RCCL all-gather of [p, grad] that hands every rank the full field.  Points are
sharded by stride across ranks (no data-path collective during the solve); the
RNG is keyed by the global point index so results do not depend on N.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (multi-GPU, RCCL)

Prints ONE JSON line on rank 0.  `value` counts the ball steps of recorded walks
(the first ball + every walk() iteration, walk_on_stars.h:523,182); steps of
dropped walks (escaped / over max length) are reported separately as wasted.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "neural-monte-carlo-fluid-simulation_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP64_VECTOR_PEAK_TFLOPS = 78.6  # dense FP64 vector peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--walks", type=int, default=128)
    ap.add_argument("--points", type=int, default=65536)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-budget-s", type=float, default=15.0)
    ap.add_argument("--no-projection-wall", action="store_true")
    ap.add_argument("--blocking", action="store_true",
                    help="wait for every solve before enqueueing the next (default: the next projection is "
                         "enqueued while the previous one runs; its stats are read after)")
    return ap.parse_args()


def algorithmic_bytes(n_points, dim, total_steps, grid_elems):
    """Bytes one projection must move at minimum: read the query
    points, write p and grad, read the source grid once, plus one 4-byte source
    texel per ball step (walk_on_stars.h:273 / :539).  Geometry (<4 KB,
    LDS-staged) is negligible."""
    return n_points * 4 * dim + n_points * 4 * (1 + dim) + 4 * grid_elems + 4 * total_steps


def walk_kernel_bytes(walk_kernel_steps, grid_elems):
    """Algorithmic bytes of the dominant kernel (wos_walk_kernel) per launch: one
    4-byte source texel per walk() step plus the source grid once.  The walk-task
    records it reads and writes are an artifact of the kernel split, not part of
    the algorithm, so they are not counted (they show up in `traffic`)."""
    return 4 * walk_kernel_steps + 4 * grid_elems


def measured_traffic(points, walks):
    """HBM bytes per walk-kernel launch from the committed rocprofv3 PMC passes
    (tools/collect_traffic.py -> profiles/*walk_traffic.json), if they were taken
    on this configuration; else None."""
    prof = os.path.join(REPO, "profiles")
    best = None
    if os.path.isdir(prof):
        for f in sorted(os.listdir(prof)):
            if f.endswith("walk_traffic.json"):
                try:
                    d = json.load(open(os.path.join(prof, f)))
                except (OSError, ValueError):
                    continue
                if d.get("points") == points and d.get("walks") == walks:
                    best = d
    return best


def measured_issue():
    """Vector-instruction issue of the walk kernel from the committed rocprofv3 SQ
    pass (tools/collect_sq.py -> profiles/*walk_sq.json), if any."""
    prof = os.path.join(REPO, "profiles")
    best = None
    if os.path.isdir(prof):
        for f in sorted(os.listdir(prof)):
            if f.endswith("walk_sq.json"):
                try:
                    best = json.load(open(os.path.join(prof, f)))
                except (OSError, ValueError):
                    continue
    return best


def cpu_baseline(cfg, n_threads, budget_s):
    """The CPU oracle restatement (oracle/, C + pthreads) timed on this host on a
    bounded, strided sample of the same workload -- a reported baseline only."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    import objparse
    v, ix = objparse.load(cfg["obj"], 2)
    osc = oracle_lib.OracleScene(v, ix, cfg["source"], float(cfg["scene"]["absorptionCoeff"]))
    prm = oracle_lib.make_params(cfg["solver"], cfg["output"], math_mode=0, n_threads=n_threads)
    pts = cfg["points"]
    # calibrate on a small slice, then size the sample to ~budget_s of wall time
    stride = max(1, pts.shape[0] // 512)
    t0 = time.perf_counter()
    _, _, _, _, st = oracle_lib.solve(osc, prm, pts[::stride], index_base=0, index_stride=stride)
    dt = time.perf_counter() - t0
    per_pt = dt / max(1, pts[::stride].shape[0])
    n_sample = int(min(pts.shape[0], max(512, budget_s / max(per_pt, 1e-9))))
    stride = max(1, pts.shape[0] // n_sample)
    sample = pts[::stride]
    t0 = time.perf_counter()
    _, _, _, _, st = oracle_lib.solve(osc, prm, sample, index_base=0, index_stride=stride)
    dt = time.perf_counter() - t0
    # one core on a smaller strided subset (BASELINE.md asks for both)
    prm1 = oracle_lib.make_params(cfg["solver"], cfg["output"], math_mode=0, n_threads=1)
    s1 = max(1, pts.shape[0] // 1024)
    t1 = time.perf_counter()
    _, _, _, _, st1 = oracle_lib.solve(osc, prm1, pts[::s1], index_base=0, index_stride=s1)
    dt1 = time.perf_counter() - t1
    return {
        "value_1core": st1["walk_steps"] / dt1,
        "value": st["walk_steps"] / dt,
        "unit": "walk-steps/s",
        "cores": n_threads,
        "kind": "port",
        "sample": f"{sample.shape[0]} of {pts.shape[0]} karman points (stride {stride}), {cfg['solver']['nWalks']} "
                  f"walks/pt, oracle/wos_oracle.c det math, {dt:.2f} s wall",
        "projection_s_extrapolated": dt * pts.shape[0] / sample.shape[0],
    }


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    from wos_amd import WosScene, solver_params, workloads
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    # weak scaling: every rank owns one 64k-point batch of a world*64k global projection
    cfg = workloads.karman_config(n_walks=a.walks, n_points=a.points * world)
    pts_all = cfg["points"]
    n_all = pts_all.shape[0]
    dim = 2
    scene = WosScene.from_obj(cfg["obj"], 2, torch.from_numpy(cfg["source"]).to(dev),
                              float(cfg["scene"]["absorptionCoeff"]), watertight=True, device=local_rank)
    params = solver_params(cfg["solver"], cfg["output"])

    # stride sharding keyed by global index (load balance: near-wall points are slower)
    local = np.ascontiguousarray(pts_all[rank::world])
    n_local = local.shape[0]
    n_pad = (n_all + world - 1) // world
    x = torch.from_numpy(local).to(dev)
    gather_buf = torch.empty(world, n_pad, 1 + dim, dtype=torch.float32, device=dev)
    send = torch.zeros(n_pad, 1 + dim, dtype=torch.float32, device=dev)

    def step():
        """Enqueue one projection (+ the all-gather); returns its stats ticket."""
        p, g, st = scene.solve(x, params, index_base=rank, index_stride=world, sync=a.blocking)
        if world > 1:
            send[:n_local, 0] = p
            send[:n_local, 1:] = g
            dist.all_gather_into_tensor(gather_buf, send)
        return st["ticket"]

    for _ in range(a.warmup):
        scene.solve_stats(step())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps_rec = steps_all = 0
    kernel_ms, walk_ms, fb_ms, fold_ms, walk_kernel_steps, launches = [], [], [], [], 0, 0
    # one projection in flight behind the one whose counters are read (device counters,
    # copied per solve; wos_solve_stats waits only for that solve)
    tickets = [step()]
    for k in range(a.steps):
        if k + 1 < a.steps:
            tickets.append(step())
        st = scene.solve_stats(tickets[k])
        steps_rec += st["walk_steps"]
        steps_all += st["walk_steps"] + st["wasted_steps"]
        kernel_ms.append(st["kernel_ms"])
        walk_ms.append(st["walk_ms"])
        fb_ms.append(st["first_ball_ms"])
        fold_ms.append(st["fold_ms"])
        launches += st["walk_launches"]
        # every walk has exactly one first-ball step (taken in wos_first_ball_kernel)
        n_walks_run = st["walks_recorded"] + st["walks_escaped"] + st["walks_max_length"]
        walk_kernel_steps += st["walk_steps"] + st["wasted_steps"] - n_walks_run
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    tot = torch.tensor([elapsed, float(steps_rec), float(steps_all)], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = tot[0:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        sums = tot[1:].clone()
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        elapsed = float(tmax.item())
        steps_rec, steps_all = float(sums[0].item()), float(sums[1].item())

    if rank == 0:
        kms = float(np.mean(kernel_ms))
        # dominant kernel: wos_walk_kernel, timed with HIP events on the solve's stream
        wms = float(np.sum(walk_ms) / max(1, launches))
        wbytes = walk_kernel_bytes(walk_kernel_steps / max(1, launches), cfg["source"].size)
        achieved = wbytes / (wms * 1e-3) / 1e9
        steps_per_launch = steps_all / a.steps / world
        pbytes = algorithmic_bytes(n_local, dim, steps_per_launch, cfg["source"].size)
        tr = measured_traffic(a.points, a.walks)
        line = {
            "metric": "WoS walk-steps/sec + pressure-projection wall-time per step, 2D karman 64k pts",
            "value": steps_rec / elapsed,
            "unit": "walk-steps/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": "karman2d: geometry_1cyl_long_open.obj, lambda=350, RR 0.99, "
                                   f"{n_all} random query pts ({world} x 256^2 minus cylinder), {a.walks} walks/pt",
                       "points": n_all, "walks_per_point": a.walks, "source_grid": list(cfg["source"].shape),
                       "parallelism": f"points sharded by stride over {world} GPU(s) + 1 RCCL all-gather"},
            "projection_ms": elapsed / a.steps * 1e3,
            "enqueue": "blocking" if a.blocking else "pipelined (next projection enqueued before the previous one's stats are read)",
            "kernel_ms": kms,
            "walk_steps_per_projection": steps_rec / a.steps,
            "wasted_steps_per_projection": (steps_all - steps_rec) / a.steps,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": tr["bytes_per_launch"] if tr else None,
                         "kernel": "wos_walk_kernel", "kernel_ms": wms,
                         "algorithmic_bytes_per_launch": wbytes,
                         "traffic_source": tr["source"] if tr else None,
                         "projection_achieved_GBps": pbytes / (kms * 1e-3) / 1e9},
            "valu_issue": None,
            "kernel_split_ms": {"first_ball": float(np.mean(fb_ms)), "walk": float(np.mean(walk_ms)),
                                "fold": float(np.mean(fold_ms)), "total": kms},
        }
        sq = measured_issue()
        if sq:
            line["valu_issue"] = {"kernel": sq["kernel"], "frac": sq["valu_issue_frac"],
                                  "wait_any_frac": sq["wait_any_frac"], "wait_inst_frac": sq["wait_inst_frac"],
                                  "source": sq["source"]}
        if world == 1 and not a.no_projection_wall:
            # the metric's second half: wall time of one whole projection call as the
            # time-stepper issues it (fresh Scene(sceneConfig, div) + wost, model_split.py:185-202)
            sys.path.insert(0, os.path.join(REPO, "tools"))
            from projection_timing import projection_timings
            pt = projection_timings(steps=3, n_walks=a.walks)
            line["projection_wall"] = {
                "device_handoff_ms": pt["device_fresh_scene_ms"],
                "reference_handoff_ms": pt["ref_style_ms"],
                "scene_create_ms": pt["scene_create_ms"],
                "note": "device: Scene(cfg, div CUDA tensor) + wost(CUDA points), outputs on device; reference: "
                        "div/points via .cpu().numpy(), nested-list outputs, grad p back to the device",
            }
        if world == 1 and not a.no_cpu_baseline:
            threads = a.cpu_threads or min(16, os.cpu_count() or 1)
            line["cpu_baseline"] = cpu_baseline(cfg, threads, a.cpu_budget_s)
        print(json.dumps(line), flush=True)
    scene.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
