"""Times alternative builds of libwos_hip.so on the karman 64k x 128 workload.
Each variant runs in its own subprocess (WOS_LIB_PATH selects the library).
    python tools/time_variants.py lib/abl/libwos_base.so lib/abl/libwos_nosil.so ...
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, time
sys.path.insert(0, "%s/neural-monte-carlo-fluid-simulation_amd")
import numpy as np, torch
from wos_amd import WosScene, solver_params, workloads
cfg = workloads.karman_config(n_walks=int(sys.argv[1]))
dev = torch.device("cuda", 0)
sc = WosScene.from_obj(cfg["obj"], 2, cfg["source"], 350.0, watertight=True)
x = torch.from_numpy(cfg["points"]).to(dev)
prm = solver_params(cfg["solver"], cfg["output"])
ms = []
for i in range(6):
    p, g, st = sc.solve(x, prm)
    ms.append(st["kernel_ms"])
print(json.dumps({"kernel_ms": sorted(ms[1:])[len(ms[1:])//2], "min_ms": min(ms[1:]), "steps": st["walk_steps"] + st["wasted_steps"], "iters": st["rejection_iters"], "p_sum": float(p.double().sum())}))
''' % REPO

if __name__ == "__main__":
    walks = os.environ.get("WALKS", "128")
    for rnd in range(2):
        for lib in sys.argv[1:]:
            env = dict(os.environ, WOS_LIB_PATH=os.path.abspath(lib))
            out = subprocess.run([sys.executable, "-c", CHILD, walks], env=env, capture_output=True, text=True)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            print(rnd, os.path.basename(lib), line[-1] if line else out.stderr[-500:], flush=True)
