"""Robust float semantics on the HIP path (solver key robustFloatSemantics, C ABI
wos_solver_params.robust_float; SURVEY.md section 7.2 hard part 4).

The reference stores the 2D Yukawa ball members K0(mu R), I0(mu R), ... as floats
(distributions.h:585-587,695), which overflow for mu R > ~92 and poison walks with NaN;
the 3D exp/sinh members under/overflow alike.  The robust kernels (Gfn<DIM, true>,
csrc/wos_robust.hip) evaluate balls with mu R > 80 with exponentially scaled Bessels;
below that they are the reference arithmetic.  Checks:
  * bit-exact against the oracle's robust mode (2D Taylor-Green-size square, the flipped
    Taylor-Green config A, a 3D cube scaled to [-3, 3]^3);
  * bit-identical to the reference semantics where no ball exceeds mu R = 80 (karman);
  * the analytic solution on the 2 pi square, per point over 16 RNG keys.
"""
import numpy as np
import pytest

import kat_cases
import objparse
from wos_amd import WosScene, solver_params, workloads

pytestmark = pytest.mark.gpu


def _bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    np.testing.assert_array_equal(a[~np.isnan(a)].view(np.uint32), b[~np.isnan(b)].view(np.uint32))


def _gpu_vs_oracle(oracle, v, ix, src, lam, solver, output, pts):
    sc = WosScene(v, ix, src, lam, watertight=True)
    p, g, st, ne, sp = sc.solve(pts, solver_params(solver, output), counts=True)
    sc.close()
    osc = oracle.OracleScene(v, ix, src, lam)
    po, go, neo, spo, ost = oracle.solve(osc, oracle.make_params(solver, output), pts)
    np.testing.assert_array_equal(ne, neo)
    np.testing.assert_array_equal(sp, spo)
    _bits_equal(p, po)
    _bits_equal(g, go)
    return p, g, st


@pytest.mark.parametrize("case", ["square2pi", "cube_x3"])
def test_robust_bit_exact_vs_oracle(gpu, oracle, case):
    if case == "square2pi":
        c = kat_cases.box2d(350.0, 1, 1, npts=400, n_walks=32, side=2 * np.pi, robust=True)
    else:
        c = kat_cases.cube3d(350.0, 1, 1, 1, npts=150, n_walks=16, scale=3.0, robust=True)
    p, g, st = _gpu_vs_oracle(oracle, c["vertices"], c["prims"], c["source"], c["absorption"], c["solver"],
                              c["output"], c["points"])
    assert np.isfinite(p).all() and np.isfinite(g).all()
    assert st["points_estimated"] == c["points"].shape[0]


def test_robust_config_a_flipped(gpu, oracle):
    """Config A flipped (the meaningful Taylor-Green problem): NaN under the reference
    semantics (test_gpu_configs), finite and bit-exact vs the oracle in robust mode."""
    cfg = workloads.taylorgreen_config(n_walks=8, res=16, flip=True)
    v, ix = objparse.load(cfg["obj"], 2, flip=True)
    solver = dict(cfg["solver"], robustFloatSemantics=True)
    p, g, st = _gpu_vs_oracle(oracle, v, ix, cfg["source"], 350.0, solver, cfg["output"], cfg["points"])
    assert np.isfinite(p).all() and np.isfinite(g).all()
    assert st["walks_max_length"] == 0 and st["wasted_steps"] == 0


def test_robust_identical_below_threshold(gpu):
    """karman (mu R <= 60): the robust kernels reproduce the reference-semantics kernels
    bit for bit."""
    cfg = workloads.karman_config(n_points=4096, n_walks=32)
    v, ix = objparse.load(cfg["obj"], 2)
    sc = WosScene(v, ix, cfg["source"], 350.0, watertight=True)
    p0, g0, _ = sc.solve(cfg["points"], solver_params(cfg["solver"], cfg["output"]))
    p1, g1, _ = sc.solve(cfg["points"], solver_params(dict(cfg["solver"], robustFloatSemantics=True), cfg["output"]))
    sc.close()
    _bits_equal(p0, p1)
    _bits_equal(g0, g1)


def test_robust_kat_square2pi(gpu):
    c = kat_cases.box2d(350.0, 1, 1, npts=600, n_walks=32, side=2 * np.pi, robust=True)
    sc = WosScene(c["vertices"], c["prims"], c["source"], c["absorption"], watertight=True)
    P, G = [], []
    for k in range(16):
        p, g, st = sc.solve(c["points"], solver_params(c["solver"], c["output"], seed=0x524F0000 + k))
        assert st["points_estimated"] == c["points"].shape[0]
        P.append(p)
        G.append(g)
    sc.close()
    kat_cases.check_z(*kat_cases.z_with_bias_floor(P, G, c))
