"""Boundary-value-caching cases shared by the oracle test (test_bvc.py) and the GPU
parity test (test_gpu_bvc.py): the reference's bvc (demo.cpp:265-363) on 2D
all-Neumann scenes."""
import numpy as np

import kat_cases
from wos_amd import workloads


def case(name):
    """-> dict(vertices, prims, source, absorption, double_sided, solver, output)"""
    if name.startswith("karman"):
        cfg = workloads.config_by_name("B")
        solver = dict(cfg["solver"], boundaryCacheSize=256, domainCacheSize=256, nWalksForCachedSolutionEstimates=32)
        out = dict(cfg["output"], gridRes=32)
        c = {"vertices": cfg["vertices"], "prims": cfg["prims"], "source": cfg["source"], "absorption": 350.0,
             "double_sided": name == "karman_double_sided", "solver": solver, "output": out}
    elif name.startswith("box"):
        lam = 0.0 if name == "box_harmonic" else 50.0
        k = kat_cases.box2d(50.0, 1, 1, res=256)
        solver = dict(k["solver"], boundaryCacheSize=384, domainCacheSize=512, nWalksForCachedSolutionEstimates=32)
        if name == "box_regularized":
            solver["regularizationForKernels"] = 0.05
        if lam == 0.0:
            # no absorption: Neumann-only walks never end (throughput 1 >= the 0.99 roulette
            # threshold) -- they all run into maxWalkLength and are dropped, so the cached
            # boundary values are 0; the case exercises the harmonic free-space kernels
            solver["setpsBeforeApplyingTikhonov"] = 10000
            solver["maxWalkLength"] = 20
        c = {"vertices": k["vertices"], "prims": k["prims"], "source": k["source"], "absorption": lam,
             "double_sided": False, "solver": solver, "output": {"gridRes": 24, "boundaryDistanceMask": 1e-3}}
    else:
        raise KeyError(name)
    return c


NAMES = ["karman", "karman_double_sided", "box", "box_harmonic", "box_regularized"]


def box_kat_reference(grid_res, lam, bbox_min, bbox_max):
    """p = cos(pi x) cos(pi y) / (lam + 2 pi^2) at the evaluation grid points
    (createEvaluationGrid, grid.h:352-368)."""
    i, j = np.meshgrid(np.arange(grid_res), np.arange(grid_res), indexing="ij")
    ext = np.asarray(bbox_max, np.float32) - np.asarray(bbox_min, np.float32)
    x = (i.astype(np.float32) / np.float32(grid_res)) * ext[0] + np.float32(bbox_min[0])
    y = (j.astype(np.float32) / np.float32(grid_res)) * ext[1] + np.float32(bbox_min[1])
    x, y = x.astype(np.float64), y.astype(np.float64)
    return x, y, np.cos(np.pi * x) * np.cos(np.pi * y) / (lam + 2 * np.pi ** 2)


def junction_square(lam=4.0):
    """Unit square: the bottom side Dirichlet (g = 1, one segment), the other three Neumann,
    two Neumann/Dirichlet junctions at (0, 0) and (1, 0), f = 0 -> u = cosh(mu (1 - y)) / cosh(mu).
    The sampler's vertex normals come from the scene's one mesh (boundary_sampler.h:193-236 over
    scene.vertices / scene.segments, demo.cpp:316): at a junction the Neumann side's normal is
    summed in, so the Dirichlet segment displaced by normalOffset runs from (d, d) to (1 - d, d),
    d = normalOffset / sqrt(2) (a Dirichlet-only normal would put it at y = normalOffset)."""
    v = np.array([[1, 0], [1, 1], [0, 1], [0, 0]], np.float32)
    ix = np.array([[0, 1], [1, 2], [2, 3]], np.int32)  # right, top, left (counter-clockwise)
    dv = np.array([[0, 0], [1, 0]], np.float32)
    dix = np.array([[0, 1]], np.int32)                  # bottom
    solver = {"nWalks": 64, "maxWalkLength": 10000, "setpsBeforeApplyingTikhonov": 0,
              "setpsBeforeUsingMaximalSpheres": 0, "epsilonShell": 1e-3, "minStarRadius": 1e-3,
              "silhouettePrecision": 1e-3, "russianRouletteThreshold": 0.0, "ignoreDirichlet": False,
              "ignoreNeumann": False, "ignoreSource": True, "boundaryCacheSize": 512,
              "nWalksForCachedGradientEstimates": 128, "nWalksForCachedSolutionEstimates": 64}
    return {"vertices": v, "prims": ix, "source": np.zeros((2, 2), np.float32), "absorption": lam,
            "kw": {"dvertices": dv, "dprims": dix, "dirichlet_value": 1.0}, "solver": solver,
            "output": {"gridRes": 32, "boundaryDistanceMask": 1e-3}}


def junction_reference(grid_res, lam, pmin, pmax):
    """u = cosh(mu (1 - y)) / cosh(mu) at the evaluation grid (createEvaluationGrid, grid.h:352-368)."""
    t = np.arange(grid_res, dtype=np.float32) / np.float32(grid_res)
    X, Y = np.meshgrid(t * (pmax[0] - pmin[0]) + pmin[0], t * (pmax[1] - pmin[1]) + pmin[1], indexing="ij")
    mu = np.sqrt(lam)
    return X.astype(np.float64), Y.astype(np.float64), np.cosh(mu * (1.0 - Y.astype(np.float64))) / np.cosh(mu)
