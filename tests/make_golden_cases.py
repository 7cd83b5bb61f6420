"""Golden-fixture cases: small, fixed-seed inputs for every scene family.

The fixtures in tests/golden/*.npz hold the oracle's (det math mode) outputs for
these inputs; tests compare the oracle (CPU) and the HIP kernel (GPU) to them.
Regenerate with:  python tests/golden/make_golden.py
"""
import numpy as np

import objparse
from wos_amd import workloads

SEED = 0x5EED0001


def case_inputs(name):
    """-> dict(vertices, prims, dvertices, dprims, dirichlet_value, absorption, source, solver, output, pts)"""
    if name == "karman_small":
        cfg = workloads.karman_config(n_walks=128)
        v, ix = objparse.load(cfg["obj"], 2)
        return dict(vertices=v, prims=ix, dvertices=None, dprims=None, dirichlet_value=0.0, absorption=350.0,
                    source=cfg["source"], solver=cfg["solver"], output=cfg["output"], pts=cfg["points"][:256])
    if name == "taylorgreen_small":
        cfg = workloads.taylorgreen_config(n_walks=32, res=8, flip=True)
        cfg["solver"]["maxWalkLength"] = 300
        v, ix = objparse.load(cfg["obj"], 2, flip=True)
        return dict(vertices=v, prims=ix, dvertices=None, dprims=None, dirichlet_value=0.0, absorption=350.0,
                    source=cfg["source"], solver=cfg["solver"], output=cfg["output"], pts=cfg["points"])
    if name == "box_dirichlet_small":
        cfg = workloads.dirichlet_obstacle_config(n_walks=64, res=12)
        return dict(vertices=cfg["vertices"], prims=cfg["prims"], dvertices=cfg["dvertices"], dprims=cfg["dprims"],
                    dirichlet_value=1.0, absorption=350.0, source=cfg["source"], solver=cfg["solver"],
                    output=cfg["output"], pts=cfg["points"])
    if name == "cube_small":
        cfg = workloads.cube_config(res=6, n_walks=64)
        v, ix = objparse.load(cfg["obj"], 3)
        return dict(vertices=v, prims=ix, dvertices=None, dprims=None, dirichlet_value=0.0, absorption=350.0,
                    source=cfg["source"], solver=cfg["solver"], output=cfg["output"], pts=cfg["points"])
    raise KeyError(name)


def run_case(name, oracle):
    c = case_inputs(name)
    sc = oracle.OracleScene(c["vertices"], c["prims"], c["source"], c["absorption"], dvertices=c["dvertices"],
                            dprims=c["dprims"], dirichlet_value=c["dirichlet_value"])
    prm = oracle.make_params(c["solver"], c["output"], seed=SEED, math_mode=0, n_threads=4)
    p, g, _, _, _ = oracle.solve(sc, prm, c["pts"])
    return p, g


def run_case_gpu(name):
    from wos_amd import WosScene, solver_params
    c = case_inputs(name)
    sc = WosScene(c["vertices"], c["prims"], c["source"], c["absorption"], dvertices=c["dvertices"],
                  dprims=c["dprims"], dirichlet_value=c["dirichlet_value"], watertight=True)
    p, g, _ = sc.solve(c["pts"], solver_params(c["solver"], c["output"], seed=SEED))
    sc.close()
    return p, g


CASES = ["karman_small", "taylorgreen_small", "box_dirichlet_small", "cube_small"]
