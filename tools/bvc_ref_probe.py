"""The HIP BVC on the upstream engine scene (bvc.json settings) over K keys: per-pixel mean and
spread saved for the comparison with the reference's solutions/bvc.pfm (GPU box).
    python3 tools/bvc_ref_probe.py OUT.npz [K]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neural-monte-carlo-fluid-simulation_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402

import engine_pin as ep  # noqa: E402
from wos_amd import WosScene, bvc_params, solver_params  # noqa: E402


def main():
    out = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    U = ep.upstream_scene()
    (nv, nix), (dv, dix) = U["neumann"], U["dirichlet"]
    sc = WosScene(nv, nix, np.zeros((4, 4), np.float32), 0.0, dvertices=dv, dprims=dix,
                  dirichlet_image=U["dirichlet_image"], dirichlet_image_box=U["box"], watertight=True)
    solver = {"boundaryCacheSize": 6144, "domainCacheSize": 6144, "nWalksForCachedSolutionEstimates": 96,
              "nWalksForCachedGradientEstimates": 960, "maxWalkLength": 1024, "epsilonShell": 1e-3,
              "minStarRadius": 1e-3, "radiusClampForKernels": 0, "ignoreDirichlet": False, "ignoreNeumann": True,
              "ignoreSource": True}
    output = {"gridRes": 256, "boundaryDistanceMask": 1e-2}
    runs, ms = [], []
    for s in range(K):
        sol, _, info = sc.bvc(solver_params(solver, output, seed=0x5EED6000 + s),
                              bvc_params(solver, output, grid_box=U["box"]), samples=False)
        runs.append(sol.ravel())
        ms.append(info["stats"]["kernel_ms"])
    sc.close()
    R = np.asarray(runs, np.float32)
    np.savez_compressed(out, runs=R, kernel_ms=np.asarray(ms))
    print(f"{K} runs, kernel {np.median(ms):.1f} ms median")


if __name__ == "__main__":
    main()
