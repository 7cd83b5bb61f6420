"""Boundary value caching on the engine demo's own settings (bindings/zombie/demo/scenes/engine/
bvc.json: 6144 boundary + 6144 domain samples, 96 / 960 walks, 256^2 grid; the mixed Dirichlet /
Neumann scene rebuilt by tests/engine_pin.py) on the HIP engine, timed per call, beside the CPU
oracle (oracle/, one thread: oracle_bvc is sequential) on a bounded sample: the same settings
with the caches cut to 1/8 (its walks and splat scale with the cache size), extrapolated x8.
GPU box only.      python3 tools/bvc_timing.py [out.json]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neural-monte-carlo-fluid-simulation_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import engine_pin as ep  # noqa: E402
import oracle_lib as oracle  # noqa: E402
from wos_amd import WosScene, bvc_params, solver_params  # noqa: E402

SOLVER = {"boundaryCacheSize": 6144, "domainCacheSize": 6144, "nWalksForCachedSolutionEstimates": 96,
          "nWalksForCachedGradientEstimates": 960, "maxWalkLength": 1024, "epsilonShell": 1e-3,
          "minStarRadius": 1e-3, "radiusClampForKernels": 0, "ignoreDirichlet": False, "ignoreNeumann": True,
          "ignoreSource": True}
OUTPUT = {"gridRes": 256, "boundaryDistanceMask": 1e-2}


def main():
    from bench import lib_sha16
    U = ep.upstream_scene()
    (nv, nix), (dv, dix) = U["neumann"], U["dirichlet"]
    kw = dict(dvertices=dv, dprims=dix, dirichlet_image=U["dirichlet_image"], dirichlet_image_box=U["box"],
              watertight=True)
    sc = WosScene(nv, nix, np.zeros((4, 4), np.float32), 0.0, **kw)
    bp = bvc_params(SOLVER, OUTPUT, grid_box=U["box"])
    wall, kern = [], []
    info = None
    for s in range(6):
        t0 = time.perf_counter()
        _, _, info = sc.bvc(solver_params(SOLVER, OUTPUT, seed=0x5EED6000 + s), bp, samples=False)
        wall.append((time.perf_counter() - t0) * 1e3)
        kern.append(info["stats"]["kernel_ms"])
    sc.close()
    st = info["stats"]
    gpu = {"ms_per_call_median": float(np.median(wall[1:])), "ms_per_call_min": float(np.min(wall[1:])),
           "kernel_ms_median": float(np.median(kern[1:])), "walk_steps": int(st["walk_steps"]),
           "wasted_steps": int(st["wasted_steps"]), "counts": {k: int(v) for k, v in info["counts"].items()}}
    if os.environ.get("BVC_GPU_ONLY"):
        print(json.dumps(gpu))
        return
    # CPU oracle, 1/8 caches
    small = dict(SOLVER, boundaryCacheSize=SOLVER["boundaryCacheSize"] // 8,
                 domainCacheSize=SOLVER["domainCacheSize"] // 8)
    osc = oracle.OracleScene(nv, nix, np.zeros((4, 4), np.float32), 0.0, **kw)
    t0 = time.perf_counter()
    _, _, _, ocounts, ost = oracle.bvc(osc, oracle.make_params(small, OUTPUT), oracle.bvc_params(small, OUTPUT,
                                                                                             grid_box=U["box"]))
    cpu_s = time.perf_counter() - t0
    res = {"workload": "engine demo bvc.json (6144 + 6144 cached samples, 96 / 960 walks, 256^2 grid, mixed "
                       "Dirichlet / Neumann scene of tests/engine_pin.py)",
           "lib_sha16": lib_sha16(), "gpu": gpu,
           "cpu_oracle": {"threads": 1, "sample": "caches 768 + 768 (1/8), same walks and grid",
                          "seconds": cpu_s, "walk_steps": int(ost["walk_steps"]),
                          "extrapolated_full_s": cpu_s * 8.0},
           "gpu_vs_cpu_1thread": cpu_s * 8.0 / (gpu["ms_per_call_median"] * 1e-3)}
    txt = json.dumps(res, indent=1)
    print(txt)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(txt)


if __name__ == "__main__":
    main()
