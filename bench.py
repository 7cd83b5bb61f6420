#!/usr/bin/env python3
"""Benchmark: WoS walk-steps/sec + pressure-projection wall-time per step
(BASELINE.json metric), default workload config B: karman 2D, 64k points x 128 walks.

One "step" = one pressure projection: the walk-on-stars solve over every query
point (inputs already resident in HBM) followed, for N>1 GPUs, by the single
RCCL all-gather of [p, grad] that hands every rank the full field.  Points are
sharded by stride across ranks (no data-path collective during the solve); the
RNG is keyed by the global point index so results do not depend on N.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config B|B_grid|C|D|E|A]
                    [--scaling weak|strong]
    torchrun --nproc-per-node N bench.py --gpus N ...   (same ranks, external launcher)

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N ranks
itself (N child processes, rank r on GPU r, RCCL); under a launcher --gpus must equal
WORLD_SIZE or it exits non-zero.

Scaling: "weak" (default for B) gives every rank one 64k-point batch of an
N x 64k projection; "strong" (default for the grid configs C, D, E -- BASELINE's
8-GPU configs are fixed-size problems) shards the config's fixed point set.
Config B's line carries both views: `value` (weak) and a `strong` object (the fixed
65398-point projection stride-sharded over the N ranks + its all-gather); at N=1 it
also times `strong_shard_ms`, the 1/8 stride shard rank 0 of an 8-GPU strong run
solves, alone on this GPU (the per-rank latency that bounds 8-GPU strong scaling); the
strong-scaled configs (C, D, E) carry the same `strong_shard` for their own point sets.

Prints ONE JSON line on rank 0.  `value` counts the ball steps of recorded walks
(the first ball + every walk() iteration, walk_on_stars.h:523,182); steps of
dropped walks (escaped / over max length) are reported separately as wasted.
"""
import argparse
import hashlib
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "neural-monte-carlo-fluid-simulation_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402
from wos_amd import dist as wdist  # noqa: E402  (pure Python: no library load at import)

# MI355X_MICROARCH.md chip table (spec, dense)
HBM_PEAK_GBS = 8000.0
FP32_VECTOR_PEAK_TFLOPS = 157.3
FP64_VECTOR_PEAK_TFLOPS = 78.6
LIB = os.environ.get("WOS_LIB_PATH") or os.path.join(PKG, "lib", "libwos_hip.so")  # the library wos_amd loads


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment bench.py starts them "
                         "itself; under torchrun it must equal WORLD_SIZE (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="B", help="A, B, B_grid, C, D or E (SURVEY.md section 8(d))")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"])
    ap.add_argument("--points", type=int, default=65536, help="config B: random points per rank (weak)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-budget-s", type=float, default=15.0)
    ap.add_argument("--no-projection-wall", action="store_true")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the strong line (config B) and the stride-8 shard (profiling passes that must "
                         "see the main workload's launches only)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, the product path); gloo stages the all-gather through host "
                         "memory and lets N ranks share one GPU (tests/test_bench_dist.py)")
    ap.add_argument("--blocking", action="store_true",
                    help="wait for every solve before enqueueing the next (default: the next projection is "
                         "enqueued while the previous one runs; its stats are read after)")
    # test hook for the rank launcher (tests/test_bench_dist.py): a CPU stand-in whose
    # "solution" is the global point index -- no engine, no GPU, not a measurement
    ap.add_argument("--standin-scene", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, grace_s=30.0):
    """`bench.py --gpus N` without a launcher: start N fresh child processes of this
    script (never an exec of this one), rank r on GPU r, rendezvous on 127.0.0.1.  The
    parent touches no GPU; rank 0's JSON line goes straight to the shared stdout and
    is the only one.  When a rank fails the others are given `grace_s` to finish and
    are then terminated (a peer stuck in a collective would never return).  Returns
    the worst child exit status."""
    import signal
    import subprocess
    import threading
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE, text=True, bufsize=1))

    def relay(r, pipe):
        # stdout carries rank 0's JSON line only; anything else a rank prints there
        # (gloo / RCCL chatter) goes to stderr
        for ln in pipe:
            out = sys.stdout if (r == 0 and ln.startswith("{")) else sys.stderr
            out.write(ln)
            out.flush()
    relays = [threading.Thread(target=relay, args=(r, p.stdout), daemon=True) for r, p in enumerate(procs)]
    for t in relays:
        t.start()

    def forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)
    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        failed_at = None
        while any(p.poll() is None for p in procs):
            if failed_at is None and any(p.returncode not in (None, 0) for p in procs):
                failed_at = time.monotonic()
            if failed_at is not None and time.monotonic() - failed_at > grace_s:
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
                for p in procs:
                    try:
                        p.wait(timeout=10)
                    except subprocess.TimeoutExpired:
                        p.kill()
                break
            time.sleep(0.05)
        for p in procs:
            p.wait()
        for t in relays:
            t.join(timeout=10)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    rcs = [p.returncode for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        print(f"bench.py: rank exit codes {rcs}", file=sys.stderr, flush=True)
        # a signal death (negative) maps to 128 + signo, like a shell
        return max(rc if rc > 0 else 128 - rc for rc in bad)
    return 0


def world_from_env(gpus):
    """(world, rank, local_rank) of this process; raises SystemExit when --gpus and a
    launcher's WORLD_SIZE disagree (a mismatched scaling line must never be printed)."""
    env_world = os.environ.get("WORLD_SIZE")
    world = int(env_world) if env_world is not None else 1
    if gpus is not None and gpus != world:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: run 'bench.py --gpus {gpus}' "
                         f"without a launcher, or under torchrun with --nproc-per-node {gpus}")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


class StandInScene:
    """--standin-scene: p = global index, grad = (index, -index) [, 0]; three steps per
    point.  Exercises the launcher, sharding, gather and JSON line without an engine."""

    def __init__(self, dim):
        self.dim, self.pending, self.next = dim, {}, 0

    def info(self):
        return {"n_silhouettes": 0, "n_prims": 0}

    def solve(self, x, params, index_base=0, index_stride=1, sync=False):
        import torch
        n = int(x.shape[0])
        p = (index_base + index_stride * torch.arange(n, dtype=torch.float64)).float()
        g = torch.stack([p, -p] + [torch.zeros_like(p)] * (self.dim - 2), 1)
        t, self.next = self.next, self.next + 1
        self.pending[t] = {"walk_steps": 3 * n, "wasted_steps": 0, "rejection_iters": 0, "kernel_ms": 1.0,
                           "walk_ms": 1.0, "first_ball_ms": 0.0, "fold_ms": 0.0, "walk_launches": 1,
                           "walks_recorded": n, "walks_escaped": 0, "walks_max_length": 0}
        return p, g, {"ticket": t}

    def solve_stats(self, ticket):
        return self.pending.pop(ticket)

    def close(self):
        pass


def lib_sha16():
    try:
        return hashlib.sha256(open(LIB, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


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


def algorithmic_flops_per_step(n_sil, n_prims, rej_iters_per_step):
    """F ~ 20 S_sil + 15 N_prim + I_rej x 60 (FP64) + 250 (FP64 ball
    Bessels + Poisson kernel) per walk step, S_sil / N_prim the scene's silhouette
    candidates / Neumann primitives (the brute-force query cost of fcpw's Baseline,
    baseline.inl:60-260), I_rej the measured rejection iterations per step."""
    f32 = 20.0 * n_sil + 15.0 * n_prims
    f64 = 60.0 * rej_iters_per_step + 250.0
    return f32, f64


def committed_profile(suffix, cfg_name):
    """A committed rocprofv3 profile (profiles/*<suffix>) of THIS library build on this
    configuration: stamped with the sha of libwos_hip.so it was measured on; a stale
    profile (kernel changed since) is not reported."""
    prof = os.path.join(REPO, "profiles")
    sha = lib_sha16()
    best = None
    if os.path.isdir(prof) and sha:
        for f in sorted(os.listdir(prof)):
            if f.endswith(suffix):
                try:
                    d = json.load(open(os.path.join(prof, f)))
                except (OSError, ValueError):
                    continue
                if d.get("lib_sha16") == sha and d.get("config", "B") == cfg_name:
                    best = dict(d, file=f)
    return best


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or None


def cpu_baseline(cfg, n_threads, budget_s):
    """The CPU oracle restatement (oracle/, C + pthreads) timed on this host on a
    bounded, strided sample of the same workload -- a reported baseline only."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    osc = oracle_lib.OracleScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"],
                                 **cfg["scene_kw"])
    pts = cfg["points"]
    n = pts.shape[0]

    def run(sample_stride, threads, reps=1):
        sample = pts[::sample_stride]
        prm = oracle_lib.make_params(cfg["solver"], cfg["output"], math_mode=0, n_threads=threads)
        t0 = time.perf_counter()
        for _ in range(reps):
            _, _, _, _, st = oracle_lib.solve(osc, prm, sample, index_base=0, index_stride=sample_stride)
        dt = time.perf_counter() - t0
        # per-projection figures (each repetition solves the same sample, same walks)
        return dt / reps, st, sample.shape[0]

    # calibrate on a small slice, then size the sample to ~budget_s of wall time; when
    # the whole point set takes less, repeat it (up to 50 times) to fill the budget
    stride = max(1, n // 512)
    dt, st, m = run(stride, n_threads)
    per_pt = dt / max(1, m)
    n_sample = int(min(n, max(256, budget_s / max(per_pt, 1e-9))))
    stride = max(1, n // n_sample)
    reps = 1
    if stride == 1:
        reps = int(min(50, max(1, budget_s / max(per_pt * n, 1e-9))))
    dt, st, m = run(stride, n_threads, reps)
    # one core on a smaller strided subset (BASELINE.md asks for both), ~budget/4
    s1 = max(1, int(n / max(16, (budget_s / 4) / max(per_pt * n_threads, 1e-9))))
    dt1, st1, m1 = run(s1, 1)
    ncpu = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {
        "value": st["walk_steps"] / dt,
        "unit": "walk-steps/s",
        "cores": n_threads,
        "kind": "port",
        "sample": f"{m} of {n} points of config {cfg['config_name']} (stride {stride}), "
                  f"{cfg['solver']['nWalks']} walks/pt, oracle/wos_oracle.c det math, {dt:.2f} s wall per "
                  f"pass x {reps} pass(es) on {n_threads} threads",
        "passes": reps,
        "value_1core": st1["walk_steps"] / dt1,
        "sample_1core": f"{m1} points (stride {s1}), {dt1:.2f} s wall",
        "host_cpus_visible": ncpu,
        "cpu_share": os.environ.get("OMP_NUM_THREADS"),
        "cpu_model": cpu_model(),
        "projection_s_extrapolated": dt * n / m,
        "wasted_steps_per_s": st["wasted_steps"] / dt,
    }


def timed_projections(scene, x, params, base, stride, steps, warmup, blocking, world, dist, torch, gather=None):
    """Time `steps` projections of the points `x` (global indices base + i * stride),
    each followed by `gather(p, grad)` (the RCCL all-gather for N > 1), bracketed by a
    barrier + device sync on both sides; returns (max-over-ranks seconds, per-solve
    stats).  One projection stays in flight behind the one whose counters are read
    (device counters, copied per solve; wos_solve_stats waits only for that solve)."""
    sync = torch.cuda.synchronize if x.device.type == "cuda" else (lambda: None)

    def step():
        p, g, st = scene.solve(x, params, index_base=base, index_stride=stride, sync=blocking)
        if gather is not None:
            gather(p, g)
        return st["ticket"]

    for _ in range(warmup):
        scene.solve_stats(step())
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    tickets, stats = [step()], []
    for k in range(steps):
        if k + 1 < steps:
            tickets.append(step())
        stats.append(scene.solve_stats(tickets[k]))
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=x.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, stats


def reduce_steps(steps_rec, steps_all, world, dist, torch, dev):
    """Whole-job step counts (sum over ranks)."""
    if world == 1:
        return float(steps_rec), float(steps_all)
    t = torch.tensor([float(steps_rec), float(steps_all)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t[0].item()), float(t[1].item())


def strong_projection(a, scene, params, world, rank, dim, dist, torch, dev, workloads):
    """Config B's fixed 65398-point projection stride-sharded over the N ranks (rank r
    solves points r, r + N, ...) + the one all-gather of [p, grad]: the strong-scaling
    view of the same metric beside the weak `value` (at N = 1 it is the same workload
    as the weak line)."""
    pts = workloads.config_by_name("B")["points"]
    n_all = pts.shape[0]
    local = np.ascontiguousarray(pts[rank::world])
    n_local = local.shape[0]
    n_pad = (n_all + world - 1) // world
    x = torch.from_numpy(local).to(dev)
    gather = wdist.make_gather(world, dist, n_local, n_pad, dim, dev, torch)

    elapsed, stats = timed_projections(scene, x, params, rank, world, a.steps, a.warmup, a.blocking,
                                       world, dist, torch, gather)
    rec, _ = reduce_steps(sum(s["walk_steps"] for s in stats),
                              sum(s["walk_steps"] + s["wasted_steps"] for s in stats), world, dist, torch, dev)
    return {"points": n_all, "n_gpus": world, "value": rec / elapsed, "unit": "walk-steps/s",
            "ms_per_step": elapsed / a.steps * 1e3, "walk_steps_per_projection": rec / a.steps,
            "kernel_ms_rank0": float(np.mean([s["kernel_ms"] for s in stats])),
            "note": "fixed point set (total work fixed as N grows), stride-sharded, + 1 RCCL all-gather"}


def shard_projection(a, scene, params, pts, torch, dev, shards=8):
    """One GPU timing the 1/8 stride shard an 8-GPU strong-scaled projection of the config's
    fixed point set gives rank 0 (points 0, 8, 16, ... with their global RNG indices): the
    per-rank latency floor that bounds 8-GPU strong scaling."""
    x = torch.from_numpy(np.ascontiguousarray(pts[0::shards])).to(dev)
    elapsed, stats = timed_projections(scene, x, params, 0, shards, a.steps, a.warmup, a.blocking,
                                       1, None, torch)
    return {"shards": shards, "shard_points": int(x.shape[0]), "ms": elapsed / a.steps * 1e3,
            "kernel_ms": float(np.mean([s["kernel_ms"] for s in stats])),
            "walk_ms": float(np.mean([s["walk_ms"] for s in stats]))}


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:
        # no launcher: this process only starts and waits for the N ranks (no GPU call here)
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    world, rank, local_rank = world_from_env(a.gpus)
    scaling = a.scaling or ("weak" if a.config == "B" else "strong")
    if scaling == "weak" and a.config != "B":
        raise SystemExit("weak scaling is defined for config B (random points per rank); use --scaling strong")
    if a.standin_scene:
        a.no_cpu_baseline = a.no_projection_wall = True
    import torch
    import torch.distributed as dist
    from wos_amd import WosScene, solver_params, workloads
    if a.standin_scene:
        dev = torch.device("cpu")
    else:
        # one rank per GPU; more ranks than GPUs (the gloo rehearsal on a 1-GPU box) share them
        n_dev = torch.cuda.device_count()
        if world > 1 and a.dist_backend == "nccl" and n_dev < world:
            raise SystemExit(f"bench.py: {world} RCCL ranks need {world} GPUs, {n_dev} visible "
                             "(--dist-backend gloo lets ranks share a GPU)")
        dev = torch.device("cuda", local_rank % max(1, n_dev))
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)

    cfg = workloads.config_by_name(a.config, n_points=a.points * world if scaling == "weak" else None)
    pts_all = cfg["points"]
    n_all = pts_all.shape[0]
    dim = cfg["dim"]
    if a.standin_scene:
        scene = StandInScene(dim)
    else:
        scene = WosScene(cfg["vertices"], cfg["prims"], torch.from_numpy(cfg["source"]).to(dev),
                         cfg["absorption"], watertight=True, device=dev.index, **cfg["scene_kw"])
    info = scene.info()
    params = solver_params(cfg["solver"], cfg["output"])

    # stride sharding keyed by global index (load balance: near-wall points are slower)
    local = np.ascontiguousarray(pts_all[rank::world])
    n_local = local.shape[0]
    n_pad = (n_all + world - 1) // world
    x = torch.from_numpy(local).to(dev)
    gather = wdist.make_gather(world, dist, n_local, n_pad, dim, dev, torch)

    elapsed, stats = timed_projections(scene, x, params, rank, world, a.steps, a.warmup, a.blocking,
                                       world, dist, torch, gather)
    steps_rec = steps_all = rej_iters = 0
    kernel_ms, walk_ms, fb_ms, fold_ms, walk_kernel_steps, launches = [], [], [], [], 0, 0
    for st in stats:
        steps_rec += st["walk_steps"]
        steps_all += st["walk_steps"] + st["wasted_steps"]
        rej_iters += st["rejection_iters"]
        kernel_ms.append(st["kernel_ms"])
        walk_ms.append(st["walk_ms"])
        fb_ms.append(st["first_ball_ms"])
        fold_ms.append(st["fold_ms"])
        launches += st["walk_launches"]
        # every walk has exactly one first-ball step (taken in wos_first_ball_kernel)
        n_walks_run = st["walks_recorded"] + st["walks_escaped"] + st["walks_max_length"]
        walk_kernel_steps += st["walk_steps"] + st["wasted_steps"] - n_walks_run
    steps_rec, steps_all = reduce_steps(steps_rec, steps_all, world, dist, torch, dev)

    strong = shard = None
    if a.config == "B" and scaling == "weak" and not a.no_strong:
        strong = strong_projection(a, scene, params, world, rank, dim, dist, torch, dev, workloads)
        if world == 1:
            shard = shard_projection(a, scene, params, workloads.config_by_name("B")["points"], torch, dev)
    elif scaling == "strong" and world == 1 and not a.no_strong and a.config != "A":
        # the fixed-size configs BASELINE runs on 8 GPUs (D, E; C alike): rank 0's 1/8 shard
        shard = shard_projection(a, scene, params, pts_all, torch, dev)

    if rank == 0:
        kms = float(np.mean(kernel_ms))
        # dominant kernel: wos_walk_kernel, timed with HIP events on the solve's stream
        wms = float(np.sum(walk_ms) / max(1, launches))
        wk_steps_launch = walk_kernel_steps / max(1, launches)
        wbytes = walk_kernel_bytes(wk_steps_launch, cfg["source"].size)
        achieved = wbytes / (wms * 1e-3) / 1e9
        local_steps_all = steps_all / world  # rank 0's share (stride sharding: balanced)
        pbytes = algorithmic_bytes(n_local, dim, local_steps_all / a.steps, cfg["source"].size)
        tr = committed_profile("walk_traffic.json", a.config)
        sq = committed_profile("walk_sq.json", a.config)
        # FLOP roofline of the walk kernel (the meaningful one: SURVEY.md 8(d))
        f32, f64 = algorithmic_flops_per_step(info["n_silhouettes"], info["n_prims"],
                                              rej_iters / max(1.0, local_steps_all))
        wk_flops32, wk_flops64 = f32 * wk_steps_launch, f64 * wk_steps_launch
        t_need = wk_flops32 / (FP32_VECTOR_PEAK_TFLOPS * 1e12) + wk_flops64 / (FP64_VECTOR_PEAK_TFLOPS * 1e12)
        achieved_tf = (wk_flops32 + wk_flops64) / (wms * 1e-3) / 1e12
        mixed_peak = (wk_flops32 + wk_flops64) / max(t_need, 1e-30) / 1e12
        line = {
            "metric": "WoS walk-steps/sec + pressure-projection wall-time per step, 2D karman 64k pts",
            "value": steps_rec / elapsed,
            "unit": "walk-steps/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": cfg["desc"], "name": a.config, "points": n_all,
                       "walks_per_point": cfg["solver"]["nWalks"], "source_grid": list(cfg["source"].shape),
                       "parallelism": f"points sharded by stride over {world} GPU(s) + 1 RCCL all-gather"},
            "projection_ms": elapsed / a.steps * 1e3,
            "enqueue": "blocking" if a.blocking else "pipelined (next projection enqueued before the previous one's stats are read)",
            "kernel_ms": kms,
            "walk_steps_per_projection": steps_rec / a.steps,
            "wasted_steps_per_projection": (steps_all - steps_rec) / a.steps,
            "lib_sha16": lib_sha16(),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": tr["bytes_per_launch"] if tr else None,
                         "kernel": "wos_walk_kernel", "kernel_ms": wms,
                         "algorithmic_bytes_per_launch": wbytes,
                         "walk_kernel_steps_per_launch": wk_steps_launch,
                         "traffic_source": (f"{tr['file']}: {tr['source']}" if tr else
                                            "no committed PMC profile of this library build on this config"),
                         "projection_achieved_GBps": pbytes / (kms * 1e-3) / 1e9},
            "flop_roofline": {"bound": "valu", "achieved": achieved_tf, "peak": mixed_peak, "unit": "TFLOP/s",
                              "frac": t_need / (wms * 1e-3), "kernel": "wos_walk_kernel",
                              "flops_per_step_fp32": f32, "flops_per_step_fp64": f64,
                              "peaks": {"fp32": FP32_VECTOR_PEAK_TFLOPS, "fp64": FP64_VECTOR_PEAK_TFLOPS},
                              "model": "SURVEY.md 8(d): 20 S_sil + 15 N_prim (fp32) + 60 I_rej + 250 (fp64) per "
                                       "step; frac = (F32/P32 + F64/P64) / kernel time"},
            "valu_issue": None,
            "kernel_split_ms": {"first_ball": float(np.mean(fb_ms)), "walk": float(np.mean(walk_ms)),
                                "fold": float(np.mean(fold_ms)), "total": kms},
        }
        if a.standin_scene:
            line["engine"] = "stand-in scene (launcher test hook): not a measurement"
        if strong is not None:
            line["strong"] = strong
        if shard is not None:
            full_ms = elapsed / a.steps * 1e3
            line["strong_shard_ms"] = shard["ms"]
            line["strong_shard"] = dict(shard, full_ms=full_ms, implied_8gpu_speedup=full_ms / shard["ms"],
                                        note=f"rank 0's share of an 8-GPU strong-scaled config {a.config} "
                                             "projection, timed alone on this GPU (all-gather excluded)")
        if sq:
            # calibrated: each instruction type at its measured SIMD-cycles (tools/collect_sq.py combine);
            # older profiles carry only the 4-cycle CDNA3 rule of thumb
            cal = "valu_issue_frac" in sq and "issue_cycles" in sq
            line["valu_issue"] = {"kernel": sq["kernel"],
                                  "frac": sq["valu_issue_frac"] if cal else None,
                                  "frac_hi": sq.get("valu_issue_frac_hi") if cal else None,
                                  "frac_4cyc": sq.get("valu_issue_frac_4cyc", sq.get("valu_issue_frac")),
                                  "calibrated": cal,
                                  "parts": sq.get("valu_issue_parts"),
                                  "wait_any_frac": sq["wait_any_frac"], "wait_inst_frac": sq["wait_inst_frac"],
                                  "active_frac": sq.get("active_frac"),
                                  "source": f"{sq['file']}: {sq['source']}"}
        if world == 1 and a.config == "B" and not a.no_projection_wall:
            # the metric's second half: wall time of one whole projection call as the
            # time-stepper issues it (fresh Scene(sceneConfig, div) + wost, model_split.py:185-202)
            sys.path.insert(0, os.path.join(REPO, "tools"))
            from projection_timing import projection_timings
            pt = projection_timings(steps=3, n_walks=cfg["solver"]["nWalks"])
            line["projection_wall"] = {
                "device_handoff_ms": pt["device_fresh_scene_ms"],
                "reference_handoff_ms": pt["ref_style_ms"],
                "scene_create_ms": pt["scene_create_ms"],
                "device_scene_reuse_ms": pt["device_scene_reuse_ms"],
                "device_handoff_breakdown": pt["device_handoff_breakdown"],
                "note": "device: Scene(cfg, div CUDA tensor) + wost(CUDA points), outputs on device, synced per call; "
                        "reference: div/points via .cpu().numpy(), nested-list outputs, grad p back to the device; "
                        "scene_create_ms: Scene(cfg, div numpy); device_scene_reuse_ms: one Scene, set_source + wost",
            }
        if world == 1 and not a.no_cpu_baseline:
            sys.path.insert(0, os.path.join(REPO, "tests"))
            import oracle_lib
            threads = a.cpu_threads or oracle_lib.default_threads()
            line["cpu_baseline"] = cpu_baseline(cfg, threads, a.cpu_budget_s)
        print(json.dumps(line), flush=True)
    scene.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
