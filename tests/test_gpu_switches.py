"""The engine's scheduling switches change how a solve runs, never its result.

wos_solver_params.schedule (include/wos.h WOS_SCHED_*) selects, per solve:
* WOS_SCHED_GEOM_GLOBAL  geometry records read through L2 (the path of scenes too large
                         for LDS) instead of staged in LDS;
* WOS_SCHED_FULL_NEUMANN the walk kernel with the Neumann term's code even where the
                         term is provably +0 (the "Neumann-inert" instantiation is the
                         default for such scenes);
* WOS_SCHED_NO_STAR_GRID the cooperative silhouette-group scan alone, without the
                         star-radius cell grid;
* WOS_SCHED_NO_DIR_GRID  the culled Dirichlet-distance scans alone, without the
                         Dirichlet cell grid (2D scenes with Dirichlet segments);
* WOS_SCHED_NO_TAIL_SPREAD the walk kernel without the hand-over of walks to idle sibling
                         waves (2D scenes with LDS geometry use it by default).
(WOS_SCHED_NO_GRID_SPREAD is reserved and has no effect: the grid-wide hand-over was removed.)
One process solves the same points under all 32 combinations of the five bits and compares p, grad p,
the per-point walk counts and step counts bit for bit with the default (schedule 0), which
itself is compared with the CPU oracle.
Karman (2D, no Dirichlet geometry: the walk kernel recomputes the start distance), the
Dirichlet obstacle (stored distance) and the cube (3D)."""
import numpy as np
import pytest

import objparse
from wos_amd import WosScene, solver_params, workloads
from wos_amd._lib import (SCHED_FULL_NEUMANN, SCHED_GEOM_GLOBAL, SCHED_NO_DIR_GRID, SCHED_NO_STAR_GRID,
                          SCHED_NO_TAIL_SPREAD)

pytestmark = pytest.mark.gpu

SETTINGS = list(range(32))  # every combination of the five bits
assert (SCHED_GEOM_GLOBAL | SCHED_FULL_NEUMANN | SCHED_NO_STAR_GRID | SCHED_NO_DIR_GRID | SCHED_NO_TAIL_SPREAD) == 31


def _scenes():
    out = []
    cfg = workloads.karman_config(n_walks=32)
    v, ix = objparse.load(cfg["obj"], 2)
    out.append(("karman", cfg, lambda: WosScene(v, ix, cfg["source"], 350.0, watertight=True), cfg["points"][:2048],
                lambda o: o.OracleScene(v, ix, cfg["source"], 350.0)))
    c = workloads.dirichlet_obstacle_config(n_walks=32, res=48)
    out.append(("dirichlet", c, lambda: WosScene(c["vertices"], c["prims"], c["source"], c["absorption"],
                                                 dvertices=c["dvertices"], dprims=c["dprims"], dirichlet_value=1.0,
                                                 watertight=True), c["points"][:2048],
                lambda o: o.OracleScene(c["vertices"], c["prims"], c["source"], c["absorption"], dvertices=c["dvertices"],
                                        dprims=c["dprims"], dirichlet_value=1.0)))
    k = workloads.cube_config(res=12, n_walks=16)
    kv, kix = objparse.load(k["obj"], 3)
    out.append(("cube", k, lambda: WosScene(kv, kix, k["source"], 350.0, watertight=True), k["points"],
                lambda o: o.OracleScene(kv, kix, k["source"], 350.0)))
    return out


@pytest.mark.parametrize("name,cfg,make,pts,make_oracle", _scenes(), ids=["karman", "dirichlet", "cube"])
def test_switches_are_bit_identical(gpu, oracle, name, cfg, make, pts, make_oracle):
    sc = make()
    ref = None
    for sched in SETTINGS:
        prm = solver_params(cfg["solver"], cfg["output"], schedule=sched)
        p, g, st, n_est, steps = sc.solve(np.ascontiguousarray(pts, np.float32), prm, counts=True)
        assert st["geom_global"] == (1 if sched & SCHED_GEOM_GLOBAL else 0)
        if sched & SCHED_NO_STAR_GRID:
            assert st["star_grid"] == 0
        if name == "dirichlet":
            assert st["dir_grid"] == (0 if sched & SCHED_NO_DIR_GRID else 1)
        out = [np.asarray(p).view(np.uint32), np.asarray(g).view(np.uint32), np.asarray(n_est), np.asarray(steps)]
        if ref is None:
            ref = out
            assert np.isfinite(np.asarray(p)).all()
            po, go, no, so, _ = oracle.solve(make_oracle(oracle), oracle.make_params(cfg["solver"], cfg["output"]),
                                             np.ascontiguousarray(pts, np.float32))
            for a, b in zip(ref, [po.view(np.uint32), go.view(np.uint32), no, so]):
                assert np.array_equal(a, b), "default schedule vs oracle"
            continue
        for a, b in zip(ref, out):
            assert np.array_equal(a, b), sched
    sc.close()
