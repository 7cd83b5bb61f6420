"""HIP-path known-answer tests: the engine (through the C ABI) against the exact
solution of the screened Poisson problem, with no oracle in the loop.

These pin the GPU path independently of the CPU restatement ("give the
HIP path pins that do not go through the oracle").  The cases are those of
tests/kat_cases.py: Neumann box (2D) and the reference's cube.obj (3D) with a cosine
source mode, and a Dirichlet disk.  Tolerance, per point: 16 solves with independent
RNG keys give each point's standard error sigma_hat / sqrt(16); the seed-averaged
estimate must sit within 4 such errors (plus the source-lookup bias bound) for all
but 1 % of the points, mean z^2 < 1.5 (Student-t(15): 1.15), no point beyond 8
(kat_cases.check_z).  One solve at a time must also pass the aggregate unbiasedness
check the oracle KATs use (kat_cases.check_unbiased).
"""
import numpy as np
import pytest

import kat_cases
from wos_amd import WosScene, solver_params

pytestmark = pytest.mark.gpu

CASES = {
    "box2d_l350_m1n1": lambda: kat_cases.box2d(350.0, 1, 1),
    "box2d_l350_m2n1": lambda: kat_cases.box2d(350.0, 2, 1),
    "box2d_l50_m1n2": lambda: kat_cases.box2d(50.0, 1, 2),
    "disk2d_dirichlet": lambda: kat_cases.disk2d_dirichlet(),
    "cube3d_l350_m111": lambda: kat_cases.cube3d(350.0, 1, 1, 1),
    "cube3d_l50_m111": lambda: kat_cases.cube3d(50.0, 1, 1, 1),
    "cube3d_l350_m210": lambda: kat_cases.cube3d(350.0, 2, 1, 0),
    # non-convex: the reflex vertex / edge is a silhouette candidate (star-radius path)
    "lshape2d_l50_m1n1": lambda: kat_cases.lshape2d(50.0, 1, 1),
    "lshape2d_l10_m2n1": lambda: kat_cases.lshape2d(10.0, 2, 1),
    "lshape2d_l350_m1n2": lambda: kat_cases.lshape2d(350.0, 1, 2),
    "lprism3d_l50_m111": lambda: kat_cases.lprism3d(50.0, 1, 1, 1),
    "lprism3d_l350_m210": lambda: kat_cases.lprism3d(350.0, 2, 1, 0),
    # non-zero Neumann data h (image-valued, ABI 9): the solution comes from the Neumann term
    "disk2d_neumann_l10_mode0": lambda: kat_cases.disk2d_neumann_flux(10.0, 0),
    "disk2d_neumann_l10_mode1": lambda: kat_cases.disk2d_neumann_flux(10.0, 1),
}


@pytest.mark.parametrize("name", list(CASES))
def test_gpu_kat(gpu, name):
    c = CASES[name]()
    sc = WosScene(c["vertices"], c["prims"], c["source"], c["absorption"], watertight=True, **c["kw"])
    P, G = [], []
    for k in range(16):
        p, g, st = sc.solve(c["points"], solver_params(c["solver"], c["output"], seed=0x4B410000 + k))
        assert st["points_estimated"] == c["points"].shape[0]
        # convex cases: no escapes; the L's reflex vertex leaks a rare walk (test_oracle.py)
        assert st["walks_escaped"] <= (1e-4 * st["walks_recorded"] if "shape" in name or "prism" in name else 0)
        P.append(p)
        G.append(g)
    sc.close()
    kat_cases.check_unbiased(P[0], G[0], c, 0.1 if c["absorption"] > 100 else (0.3 if c["absorption"] >= 50 else 0.6))
    zp, zg = kat_cases.per_point_z(P, G, c)
    kat_cases.check_z(zp, zg)
