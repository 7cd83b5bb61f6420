"""The engine's performance switches change the schedule, never the result.

Each switch below is read by wos_solve at every call (csrc/wos_capi.hip), so one
process can solve the same points under every setting and compare p, grad p, the
per-point walk counts and step counts bit for bit:
* WOS_FB_SORT      presorted first balls (point-setup kernel + queue order first) vs
                   the setup inside the first-ball kernel;
* WOS_FB_ORDER     the presorted first-ball queue order (point / walk-queue / reversed);
* WOS_NEUMANN_INERT the walk kernel without the Neumann term's code for scenes that
                   cannot reach the float-overflow regime vs the full kernel;
* WOS_TAIL_FOLD    the statistics folded inside the walk kernel by its idle waves vs
                   the separate fold kernel.
Karman (2D, no Dirichlet geometry: the walk kernel recomputes the start distance),
the Dirichlet obstacle (stored distance) and the cube (3D)."""
import os

import numpy as np
import pytest

import objparse
from wos_amd import WosScene, solver_params, workloads

pytestmark = pytest.mark.gpu

SETTINGS = [
    {},
    {"WOS_FB_SORT": "0"},
    {"WOS_FB_ORDER": "1"},
    {"WOS_FB_ORDER": "2"},
    {"WOS_NEUMANN_INERT": "0"},
    {"WOS_FB_SORT": "0", "WOS_NEUMANN_INERT": "0"},
    {"WOS_TAIL_FOLD": "0"},
]


def _scenes():
    out = []
    cfg = workloads.karman_config(n_walks=32)
    v, ix = objparse.load(cfg["obj"], 2)
    out.append(("karman", cfg, lambda: WosScene(v, ix, cfg["source"], 350.0, watertight=True), cfg["points"][:2048]))
    c = workloads.dirichlet_obstacle_config(n_walks=32, res=48)
    out.append(("dirichlet", c, lambda: WosScene(c["vertices"], c["prims"], c["source"], c["absorption"],
                                                 dvertices=c["dvertices"], dprims=c["dprims"], dirichlet_value=1.0,
                                                 watertight=True), c["points"][:2048]))
    k = workloads.cube_config(res=12, n_walks=16)
    kv, kix = objparse.load(k["obj"], 3)
    out.append(("cube", k, lambda: WosScene(kv, kix, k["source"], 350.0, watertight=True), k["points"]))
    return out


@pytest.mark.parametrize("name,cfg,make,pts", _scenes(), ids=["karman", "dirichlet", "cube"])
def test_switches_are_bit_identical(gpu, name, cfg, make, pts):
    sc = make()
    prm = solver_params(cfg["solver"], cfg["output"])
    ref = None
    saved = {k: os.environ.get(k) for s in SETTINGS for k in s}
    try:
        for setting in SETTINGS:
            for k in saved:
                os.environ.pop(k, None)
            os.environ.update(setting)
            p, g, _, n_est, steps = sc.solve(np.ascontiguousarray(pts, np.float32), prm, counts=True)
            out = [np.asarray(p).view(np.uint32), np.asarray(g).view(np.uint32), np.asarray(n_est),
                   np.asarray(steps)]
            if ref is None:
                ref = out
                assert np.isfinite(np.asarray(p)).all()
                continue
            for a, b in zip(ref, out):
                assert np.array_equal(a, b), setting
    finally:
        for k, v in saved.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v
        sc.close()
