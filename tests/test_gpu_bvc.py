"""Boundary value caching on the GPU (wos_bvc: boundary-start walks on the persistent
walk kernel, LDS-tiled splat) against the CPU restatement (oracle_bvc), bit for bit:
the cached samples, their estimated boundary values, the splatted evaluation grid
(solution and gradient), and the walk counters.  Plus the drop-in bvc(scene, solver,
output) writing its solution image like saveEvaluationGrid (grid.h:370-414)."""
import numpy as np
import pytest

import bvc_cases
from wos_amd import WosScene, bvc_params, solver_params

pytestmark = pytest.mark.gpu


def _bits(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    np.testing.assert_array_equal(na, nb)
    np.testing.assert_array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


@pytest.mark.parametrize("name", bvc_cases.NAMES)
def test_bvc_bit_exact(gpu, oracle, name):
    c = bvc_cases.case(name)
    sc = WosScene(c["vertices"], c["prims"], c["source"], c["absorption"], watertight=True,
                  double_sided=c["double_sided"])
    sol, grad, info = sc.bvc(solver_params(c["solver"], c["output"]), bvc_params(c["solver"], c["output"]))
    sc.close()
    osc = oracle.OracleScene(c["vertices"], c["prims"], c["source"], c["absorption"], double_sided=c["double_sided"])
    osol, ograd, osmp, ocounts, ost = oracle.bvc(osc, oracle.make_params(c["solver"], c["output"]),
                                                 oracle.bvc_params(c["solver"], c["output"]))
    assert [info["counts"][k] for k in ("boundary", "boundary_aligned", "domain", "total")] == [int(v) for v in ocounts]
    _bits(info["samples"], osmp)
    _bits(sol, osol)
    _bits(grad, ograd)
    for k in ("walk_steps", "wasted_steps", "walks_recorded", "walks_escaped", "walks_max_length",
              "rejection_iters"):
        assert info["stats"][k] == ost[k], k


def test_bvc_drop_in_writes_solution(gpu, tmp_path):
    import zombie_bindings
    c = bvc_cases.case("karman")
    from wos_amd import workloads
    scene_cfg = dict(workloads.SCENE_BASE, boundary=workloads.KARMAN_OBJ)
    scene = zombie_bindings.Scene(scene_cfg, c["source"])
    out = dict(c["output"], solutionFile=str(tmp_path / "solutions" / "bvc.pfm"))
    assert zombie_bindings.bvc(scene, c["solver"], out) is None
    raw = (tmp_path / "solutions" / "bvc.pfm").read_bytes()
    g = c["output"]["gridRes"]
    assert raw.startswith(b"PF\n%d %d\n-1\n" % (g, g))
    img = np.frombuffer(raw[len(b"PF\n%d %d\n-1\n" % (g, g)):], "<f4").reshape(g, g, 3)[::-1, :, 0]
    sol, _, _ = zombie_bindings.bvc(scene, c["solver"], out, return_arrays=True)
    np.testing.assert_array_equal(img, sol.T)
    assert np.isfinite(sol).all() and np.abs(sol).max() > 0
