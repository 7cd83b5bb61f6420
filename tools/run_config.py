"""Solves one tools/time_configs.py configuration a few times (a short program for
rocprofv3 --pmc / --kernel-trace passes).   python3 tools/run_config.py NAME [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from time_configs import scene_for  # noqa: E402
from wos_amd import solver_params  # noqa: E402

name = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cfg, sc = scene_for(name)
x = torch.from_numpy(np.ascontiguousarray(cfg["points"])).to(torch.device("cuda", 0))
prm = solver_params(cfg["solver"], cfg["output"])
for i in range(reps):
    p, g, st = sc.solve(x, prm)
    print(name, i, st["kernel_ms"], st["first_ball_ms"], st["walk_ms"], flush=True)
sc.close()
