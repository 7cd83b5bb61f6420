"""Two-phase walks (WOS_PHASES=2: wos_walk_first_kernel runs the first walk-kernel step
of every task, the walk kernel resumes the survivors) against the one-pass persistent
walk kernel: identical p, grad p, per-point walk and step counts and statistics on
every scene family -- the split changes the schedule, not the arithmetic."""
import numpy as np
import pytest

import kat_cases
import objparse
from wos_amd import WosScene, solver_params, workloads

pytestmark = pytest.mark.gpu

STATS = ("walk_steps", "wasted_steps", "walks_recorded", "walks_escaped", "walks_max_length", "walks_rr",
         "walks_dirichlet", "points_estimated", "rejection_iters")


def _cases():
    out = []
    cfg = workloads.karman_config(n_walks=64, n_points=8192)
    v, ix = objparse.load(cfg["obj"], 2)
    out.append(("karman", v, ix, cfg["source"], 350.0, {}, cfg["solver"], cfg["output"], cfg["points"]))
    cfg = workloads.dirichlet_obstacle_config(n_walks=32, res=48)
    kw = dict(dvertices=cfg["dvertices"], dprims=cfg["dprims"], dirichlet_value=1.0)
    out.append(("dirichlet", cfg["vertices"], cfg["prims"], cfg["source"], 350.0, kw, cfg["solver"], cfg["output"],
                cfg["points"]))
    cfg = workloads.cube_config(res=16, n_walks=32)
    v, ix = objparse.load(cfg["obj"], 3)
    out.append(("cube", v, ix, cfg["source"], 350.0, {}, cfg["solver"], cfg["output"], cfg["points"]))
    cfg = workloads.gear_config(n_walks=32)
    out.append(("gear", cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], {}, cfg["solver"],
                cfg["output"], cfg["points"]))
    cfg = workloads.taylorgreen_config(n_walks=8, res=12, flip=True)
    v, ix = objparse.load(cfg["obj"], 2, flip=True)
    out.append(("taylorgreen_flipped_robust", v, ix, cfg["source"], 350.0, {},
                dict(cfg["solver"], robustFloatSemantics=True), cfg["output"], cfg["points"]))
    c = kat_cases.box2d(50.0, 1, 2, npts=800, n_walks=32)
    out.append(("box_lambda50", c["vertices"], c["prims"], c["source"], 50.0, {}, c["solver"], c["output"],
                c["points"]))
    return out


CASES = _cases()


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_two_phase_matches_one_pass(gpu, monkeypatch, case):
    name, v, ix, src, lam, kw, solver, output, pts = case
    sc = WosScene(v, ix, src, lam, watertight=True, **kw)
    prm = solver_params(solver, output)
    monkeypatch.setenv("WOS_PHASES", "1")
    p1, g1, s1, n1, st1 = sc.solve(pts, prm, counts=True)
    monkeypatch.setenv("WOS_PHASES", "2")
    p2, g2, s2, n2, st2 = sc.solve(pts, prm, counts=True)
    sc.close()
    np.testing.assert_array_equal(n1, n2)
    np.testing.assert_array_equal(st1, st2)
    for a, b in ((p1, p2), (g1, g2)):
        a, b = np.asarray(a), np.asarray(b)
        np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
        np.testing.assert_array_equal(a[~np.isnan(a)].view(np.uint32), b[~np.isnan(b)].view(np.uint32))
    assert s1["walk_steps"] > 0 and s1["walks_recorded"] > 0
    for k in STATS:
        assert s1[k] == s2[k], (name, k)
