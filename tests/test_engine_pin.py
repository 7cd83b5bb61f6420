"""The oracle and the HIP path against the reference's own engine-scene outputs
(bindings/zombie/demo/scenes/engine/solutions/wost.pfm, bvc.pfm; fixture:
tests/golden/engine_solution_masks.npz).  See tests/engine_pin.py for what the
zero pattern pins and how "masked" is read off a solve.

Measured (DESIGN.md "What pins the oracle"): of 65 536 grid points, 33 165 are
masked (32 371 unmasked); the reference image is non-zero at 28 871.  89 non-zero
reference pixels are masked here, every one within 1.17 grid spacings of the
boundary (they run along three straight stretches of the outline, one pixel
outside it); 3 589 unmasked points are zero in the reference image, which its
Dirichlet-only Laplace run produces wherever every walk ends on zero boundary data.
"""
import numpy as np
import pytest

import engine_pin as ep


def _oracle_masked(oracle, v, ix, pts, closed=True):
    osc = oracle.OracleScene(v, ix, ep.source_grid(), ep.ABSORPTION, watertight=True)
    p, g, n_est, _, st = oracle.solve(osc, oracle.make_params(ep.SOLVER, ep.OUTPUT), pts)
    if closed:  # every estimated point keeps at least one recorded walk
        assert st["walks_escaped"] == 0 and st["walks_max_length"] == 0
    assert not np.isnan(g).any()
    return (g[:, 0] == 0) & (g[:, 1] == 0), n_est


def _check(report):
    assert report["masked_but_nonzero"] <= ep.MAX_RESIDUAL, report
    assert report.get("residual_max_dist_spacings", 0.0) <= ep.RESIDUAL_BAND, report


def test_oracle_mask_matches_reference_engine_images(oracle):
    fx, g = ep.fixture()
    v, ix = ep.load_geometry()
    pts, ext = ep.grid_points(v, g)
    masked, n_est = _oracle_masked(oracle, v, ix, pts)
    # a point is masked because it is outside or within the mask distance of the wall
    assert np.all(masked[n_est == 0])
    for name in ("wost", "bvc"):
        rep = ep.compare(masked, fx[name], v, ix, pts, ext, g)
        print(name, rep)
        _check(rep)
        assert rep["masked"] == 33165 and rep["unmasked_zero"] == 3589
    # the pin discriminates: the writer's row order or the OBJ winding, got wrong, fail it
    mirrored = ep.compare(masked, fx["wost"][:, ::-1], v, ix, pts, ext, g)
    assert mirrored["masked_but_nonzero"] > 50 * ep.MAX_RESIDUAL
    from wos_amd import engine
    v2, ix2 = engine.load_obj(ep.ENGINE_OBJ, 2, False, False)
    masked2, _ = _oracle_masked(oracle, v2, ix2, pts, closed=False)
    unflipped = ep.compare(masked2, fx["wost"], v2, ix2, pts, ext, g)
    assert unflipped["masked_but_nonzero"] > 0.9 * unflipped["fixture_nonzero"]


@pytest.mark.gpu
def test_hip_mask_matches_reference_engine_images(gpu, oracle):
    """The HIP path's setup (closest point, inside test, masks) on the reference's own
    engine grid: equal to the oracle's mask everywhere, so the same residual against
    the reference images."""
    from wos_amd import WosScene, solver_params
    fx, g = ep.fixture()
    v, ix = ep.load_geometry()
    pts, ext = ep.grid_points(v, g)
    sc = WosScene(v, ix, ep.source_grid(), ep.ABSORPTION, watertight=True)
    p, grad, st, n_est, _ = sc.solve(pts, solver_params(ep.SOLVER, ep.OUTPUT), counts=True)
    sc.close()
    assert st["walks_escaped"] == 0 and st["walks_max_length"] == 0
    masked = (grad[:, 0] == 0) & (grad[:, 1] == 0)
    masked_o, n_est_o = _oracle_masked(oracle, v, ix, pts)
    np.testing.assert_array_equal(n_est, n_est_o)
    np.testing.assert_array_equal(masked, masked_o)
    for name in ("wost", "bvc"):
        rep = ep.compare(masked, fx[name], v, ix, pts, ext, g)
        print(name, rep)
        _check(rep)
