"""Where does the walk kernel's latency floor come from?  (GPU box only.)

Karman 64k x 128 (config B) is solved once with per-point step counts; then
  * the stride-8 shard (8 175 points, index_base 0, stride 8: one rank of 8);
  * the K hardest points (most walk steps per point) for K = 1, 8, 64, 512, 4096,
    each point with its 128 walks;
are timed (kernel split, walk steps, walk-kernel iterations), so that the per-step
latency of a lone walk and the tail of the full solve can be compared.

    python3 tools/latency_probe.py [> gpurun_out/latency.jsonl]
With WOS_LIB_PATH pointing at a -DWOS_DIAG=1 build the per-section cycle counts are
printed on stderr for every solve.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neural-monte-carlo-fluid-simulation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from wos_amd import WosScene, solver_params, workloads  # noqa: E402


def timed(sc, x, prm, base=0, stride=1, reps=5):
    best = None
    for _ in range(reps):
        p, g, st, ne, sp = sc.solve(x, prm, index_base=base, index_stride=stride, counts=True)
        if best is None or st["kernel_ms"] < best[0]["kernel_ms"]:
            best = (st, sp)
    return best


def row(tag, n, st, sp):
    steps = st["walk_steps"] + st["wasted_steps"]
    return {"case": tag, "points": n, "kernel_ms": st["kernel_ms"], "first_ball_ms": st["first_ball_ms"],
            "walk_ms": st["walk_ms"], "fold_ms": st["fold_ms"], "steps": steps,
            "max_point_steps": int(sp.max()) if sp.size else 0,
            "walk_iters": st.get("rejection_iters", 0)}


def main():
    only = sys.argv[1] if len(sys.argv) > 1 else None  # e.g. "hardest1": that case alone (after the full solve)
    dev = torch.device("cuda", 0)
    cfg = workloads.karman_config(n_walks=128)
    sc = WosScene.from_obj(cfg["obj"], 2, cfg["source"], 350.0, watertight=True)
    prm = solver_params(cfg["solver"], cfg["output"])
    pts = np.ascontiguousarray(cfg["points"])
    x = torch.from_numpy(pts).to(dev)
    sc.solve(x, prm)
    st, sp = timed(sc, x, prm, reps=1 if only else 5)
    sp = sp.cpu().numpy()
    print(json.dumps(row("full", len(pts), st, sp)), flush=True)
    if only == "hardest1":
        idx = int(np.argmax(sp))
        xk = torch.from_numpy(np.ascontiguousarray(pts[idx:idx + 1])).to(dev)
        stk, spk = timed(sc, xk, prm, base=idx, stride=1)
        print(json.dumps(row("hardest1", 1, stk, spk.cpu().numpy())), flush=True)
        sc.close()
        return
    xs = torch.from_numpy(np.ascontiguousarray(pts[0::8])).to(dev)
    st8, sp8 = timed(sc, xs, prm, base=0, stride=8)
    print(json.dumps(row("shard8", xs.shape[0], st8, sp8.cpu().numpy())), flush=True)
    order = np.argsort(-sp, kind="stable")
    for k in (1, 8, 64, 512, 4096):
        idx = np.sort(order[:k])
        xk = torch.from_numpy(np.ascontiguousarray(pts[idx])).to(dev)
        # keep each point's RNG key: one solve per point would be slow, so the hardest
        # points are solved with their own indices only when K == 1 (index_base = idx)
        if k == 1:
            stk, spk = timed(sc, xk, prm, base=int(idx[0]), stride=1)
        else:
            stk, spk = timed(sc, xk, prm)
        r = row(f"hardest{k}", k, stk, spk.cpu().numpy())
        r["point_steps_in_full"] = int(sp[idx].max())
        print(json.dumps(r), flush=True)
    sc.close()


if __name__ == "__main__":
    main()
