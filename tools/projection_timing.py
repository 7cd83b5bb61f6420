"""Wall time of one pressure projection the way the reference's time-stepper issues it
(src/2d/models/model_split.py:185-202): a fresh zombie_bindings.Scene(sceneConfig, div)
every step, then wost(scene, solver, output, pts) -> nested lists, then the gradient
back to the device (model_split.py:272).  Compared with the device-resident hand-off
(torch CUDA div + points, results stay on the GPU) and with one scene whose source is
replaced each step.  GPU box only.
    python3 tools/projection_timing.py [steps]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neural-monte-carlo-fluid-simulation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import zombie_bindings  # noqa: E402
from wos_amd import workloads  # noqa: E402


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(steps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(out))


def projection_timings(steps=10, n_walks=128):
    cfg = workloads.karman_config(n_walks=n_walks)
    scene_cfg = dict(cfg["scene"], boundary=cfg["obj"])
    solver, output = cfg["solver"], cfg["output"]
    div_np = np.ascontiguousarray(cfg["source"], np.float32)
    pts_np = np.ascontiguousarray(cfg["points"], np.float32)
    dev = torch.device("cuda", 0)
    div_t = torch.from_numpy(div_np).to(dev)
    pts_t = torch.from_numpy(pts_np).to(dev)
    res = {"points": int(pts_np.shape[0]), "source_grid": list(div_np.shape), "walks": solver["nWalks"]}

    # (a) the reference's call pattern: div / points on the host, a fresh Scene per
    # step, nested lists out, grad p copied back to the device
    def ref_style():
        sc = zombie_bindings.Scene(scene_cfg, div_t.cpu().numpy())
        s, p, g = zombie_bindings.wost(sc, solver, output, pts_t.detach().cpu().numpy())
        s, p, g = np.array(s), np.array(p), np.array(g)
        return torch.Tensor(g).to(dev)
    res["ref_style_ms"] = timed(ref_style, steps)

    def scene_only():
        return zombie_bindings.Scene(scene_cfg, div_np)
    res["scene_create_ms"] = timed(scene_only, steps)

    # (b) device hand-off: CUDA div + points, fresh Scene per step, outputs stay on device
    def dev_style():
        sc = zombie_bindings.Scene(scene_cfg, div_t)
        return zombie_bindings.wost(sc, solver, output, pts_t)
    res["device_fresh_scene_ms"] = timed(dev_style, steps)

    # (c) one scene for the whole run, the source replaced in place each step
    keep = zombie_bindings.Scene(scene_cfg, div_t)

    def dev_reuse():
        keep.set_source(div_t)
        return zombie_bindings.wost(keep, solver, output, pts_t)
    res["device_scene_reuse_ms"] = timed(dev_reuse, steps)
    st = keep.last_stats
    res["kernel_ms"] = st["kernel_ms"]
    res["walk_steps"] = st["walk_steps"]
    res["device_handoff_breakdown"] = handoff_breakdown(steps, scene_cfg, solver, output, div_t, pts_t)
    return res


def handoff_breakdown(steps, scene_cfg, solver, output, div_t, pts_t):
    """device_fresh_scene_ms itemised: the stages of one Scene(cfg, div CUDA) + wost(CUDA
    points) call, each bracketed by host clocks in one call (median over `steps` calls):
    OBJ parse (a fresh parse; Scene() itself takes the cached one), scene create (host prep
    from the geometry cache + source copy), solver-parameter parsing, the solve's enqueue,
    the wait for its completion, the statistics read-back and the scene's destruction;
    `gpu_kernel_ms` is the solve's first-to-last kernel time on the device clock."""
    from wos_amd import engine
    path = scene_cfg["boundary"]
    flip = bool(scene_cfg.get("flipOrientation", False))
    norm = bool(scene_cfg.get("normalizeDomain", False))
    keys = ["obj_parse_ms", "obj_cached_ms", "scene_create_ms", "params_ms", "enqueue_ms", "gpu_wait_ms",
            "stats_ms", "destroy_ms", "sum_ms", "gpu_kernel_ms"]
    rows = []
    for it in range(steps + 1):
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        engine.load_obj(path, 2, flip, norm)
        t.append(time.perf_counter())
        zombie_bindings._load_boundary(path, 2, flip, norm)
        t.append(time.perf_counter())
        sc = zombie_bindings.Scene(scene_cfg, div_t)
        t.append(time.perf_counter())
        prm = engine.solver_params(solver, output)
        t.append(time.perf_counter())
        _, _, st = sc._scene.solve(pts_t, prm, sync=False)
        t.append(time.perf_counter())
        torch.cuda.current_stream().synchronize()
        t.append(time.perf_counter())
        full = sc._scene.solve_stats(st["ticket"])
        t.append(time.perf_counter())
        sc._scene.close()
        t.append(time.perf_counter())
        if it:
            d = [(t[k + 1] - t[k]) * 1e3 for k in range(len(t) - 1)]
            rows.append(d + [sum(d) - d[0], full["kernel_ms"]])
    med = np.median(np.asarray(rows), 0)
    out = {k: float(v) for k, v in zip(keys, med)}
    out["note"] = ("sum_ms = obj_cached + scene_create + params + enqueue + gpu_wait + stats + destroy "
                   "(what one Scene + wost call costs; obj_parse_ms is the uncached parse, shown for reference)")
    return out


def pipeline_timings(steps=5, n_points=65536, n_walks=128, vis_resolution=1000):
    """The whole projection step of the karman example (examples/karman/run.sh:
    SIREN 2 x 128 sine, vis_resolution 1000, wost.json solver): SIREN divergence on
    the grid, the solve at the pressure samples, the projection loss + backward --
    (a) with the reference's host hand-offs, (b) device-resident (wos_amd.projection)."""
    from wos_amd import projection as pj
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = workloads.karman_config(n_walks=n_walks, n_points=n_points)
    size = workloads.scene_size(workloads.KARMAN_OBJ)
    scene_cfg = dict(cfg["scene"], boundary=cfg["obj"])
    u = pj.Siren(2, 2, 2, 128).to(dev)
    u_prev = pj.Siren(2, 2, 2, 128).to(dev)
    samples = torch.from_numpy(cfg["points"]).to(dev)
    proj = pj.PressureProjector(scene_cfg, cfg["solver"], cfg["output"], samples)
    n_loss = 128 * 128  # sample_resolution 128 (run.sh)
    res = {"points": int(samples.shape[0]), "walks": n_walks, "vis_resolution": vis_resolution}

    def host_step():
        div = proj.source_from_velocity(u_prev, vis_resolution, size).cpu().numpy()
        sc = zombie_bindings.Scene(scene_cfg, div)
        s, p, g = zombie_bindings.wost(sc, cfg["solver"], cfg["output"], samples.detach().cpu().numpy())
        grad_p = torch.Tensor(np.array(g)).to(dev)
        loss = proj.projection_loss(u, u_prev, grad_p, n_loss)
        loss.backward()

    def device_step():
        div = proj.source_from_velocity(u_prev, vis_resolution, size)
        p, g = proj.solve(div)
        loss = proj.projection_loss(u, u_prev, g, n_loss)
        loss.backward()

    def divergence_only():
        return proj.source_from_velocity(u_prev, vis_resolution, size)

    res["host_handoff_step_ms"] = timed(host_step, steps)
    res["device_step_ms"] = timed(device_step, steps)
    res["siren_divergence_ms"] = timed(divergence_only, steps)
    res["solve_kernel_ms"] = proj.last_stats["kernel_ms"]
    return res


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    print(json.dumps({"scene_handoff": projection_timings(steps),
                      "pipeline_64k": pipeline_timings(max(3, steps // 2)),
                      "pipeline_512sq": pipeline_timings(max(3, steps // 2), n_points=512 * 512)}), flush=True)
