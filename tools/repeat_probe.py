import sys, numpy as np
sys.path[:0]=["tests","neural-monte-carlo-fluid-simulation_amd"]
import kat_cases
from wos_amd import WosScene, solver_params
c = kat_cases.box2d(350.0, 1, 1, npts=400, n_walks=32, side=2 * np.pi, robust=True)
sc = WosScene(c["vertices"], c["prims"], c["source"], c["absorption"], watertight=True)
ref=None
for r in range(6):
    p, g, st, ne, sp = sc.solve(c["points"], solver_params(c["solver"], c["output"]), counts=True)
    if ref is None: ref=(p.view(np.uint32).copy(), sp.copy())
    print(r, "steps", int(sp.sum()), "p-diff", int((p.view(np.uint32)!=ref[0]).sum()), "sp-diff", int((sp!=ref[1]).sum()), flush=True)
