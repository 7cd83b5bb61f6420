"""Runs the karman 64k x 128 projection a few times (for rocprofv3 --pmc / --kernel-trace passes).
    python3 tools/prof_solve.py [reps] [n_walks]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neural-monte-carlo-fluid-simulation_amd"))
import torch  # noqa: E402
from wos_amd import WosScene, solver_params, workloads  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
walks = int(sys.argv[2]) if len(sys.argv) > 2 else 128
cfg = workloads.karman_config(n_walks=walks)
dev = torch.device("cuda", 0)
sc = WosScene.from_obj(cfg["obj"], 2, cfg["source"], 350.0, watertight=True)
x = torch.from_numpy(cfg["points"]).to(dev)
prm = solver_params(cfg["solver"], cfg["output"])
for i in range(reps):
    p, g, st = sc.solve(x, prm)
    print(i, st["kernel_ms"], st["walk_steps"] + st["wasted_steps"], flush=True)
