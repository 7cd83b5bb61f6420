"""Helpers for the pin against the reference's own engine-scene outputs
(tests/golden/engine_solution_masks.npz, made by tests/golden/make_engine_mask.py
from bindings/zombie/demo/scenes/engine/solutions/{wost,bvc}.pfm).

The reference ran its grid demo on scenes/engine/data/geometry.obj (byte-identical to
scenes/engine_geometry.obj here) with Scene(json)'s defaults flipOrientation = true,
isWatertight = true (scene.h:22-33) and output.boundaryDistanceMask = 1e-2
(scenes/engine/wost.json, bvc.json).  Its writer zeroes a grid point when
    (!insideDomain(pt) && !isDoubleSided) || min(|dDist|, |nDist|) < boundaryDistanceMask
(grid.h:316-319, 407-409).  Which pixels that rule zeroes depends only on the geometry
conventions (OBJ winding + flip, FLT_EPSILON-padded bbox, segment / vertex normals,
the inside test, closest distances) and on the writer's orientation -- not on the
estimator.  The solution values themselves need the upstream mixed-boundary scene,
which this fork no longer builds (scene.h:28-30,43-45), so they are not compared.

A point is "masked" here when the solve returns grad == (0, 0): getGradient zeroes
exactly (!inside && !doubleSided) || |nDist| < mask (grid.h:227-228), and with no
Dirichlet geometry dDist is the bbox far-corner distance (fcpw_scene_loader.h:312-314),
far above the mask, so the two rules coincide.
"""
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENGINE_OBJ = os.path.join(REPO, "scenes", "engine_geometry.obj")
FIXTURE = os.path.join(REPO, "tests", "golden", "engine_solution_masks.npz")
MASK = 1e-2
# the solver settings only have to produce a non-zero gradient wherever the writer
# keeps a value: a tiny absorption (mu R <= 14 on this 1000-unit scene) and roulette
# end every walk after a few steps; a positive random source without antithetic or
# control variates makes every estimated gradient non-zero
SOLVER = {"nWalks": 2, "maxWalkLength": 1024, "russianRouletteThreshold": 0.99,
          "setpsBeforeApplyingTikhonov": 0, "ignoreDirichlet": True, "ignoreNeumann": True,
          "ignoreSource": False, "disableGradientAntitheticVariates": True,
          "disableGradientControlVariates": True}
OUTPUT = {"gridRes": 256, "boundaryDistanceMask": MASK}
ABSORPTION = 1e-4
# residual allowed against the reference's images (see DESIGN.md "What pins the oracle")
MAX_RESIDUAL = 89
RESIDUAL_BAND = 1.25  # grid spacings


def source_grid():
    return np.random.default_rng(11).uniform(0.5, 1.5, (64, 64)).astype(np.float32)


def fixture():
    d = np.load(FIXTURE)
    g = int(d["grid_res"])
    return {k: np.unpackbits(d[k + "_nonzero_bits"])[:g * g].reshape(g, g).astype(bool)
            for k in ("wost", "bvc")}, g


def load_geometry():
    """Scene(json) defaults: flipOrientation = true (scene.h:33, loadOBJ :123-124)."""
    from wos_amd import engine
    return engine.load_obj(ENGINE_OBJ, 2, True, False)


def bbox(v):
    """computeBoundingBox(vertices, false, 1.0) with fcpw's FLT_EPSILON padding
    (fcpw_scene_loader.h:76-93, bounding_volumes.h:43-47)."""
    eps = np.float32(np.finfo(np.float32).eps)
    return (v - eps).min(0).astype(np.float32), (v + eps).max(0).astype(np.float32)


def grid_points(v, g):
    """createSolutionGrid (grid.h:35-52): point idx = i*g + j at
    ((i / float(g)) * extent.x + bMin.x, (j / float(g)) * extent.y + bMin.y), in float."""
    lo, hi = bbox(v)
    ext = (hi - lo).astype(np.float32)
    t = (np.arange(g, dtype=np.float32) / np.float32(g)).astype(np.float32)
    x = (t * ext[0]).astype(np.float32) + lo[0]
    y = (t * ext[1]).astype(np.float32) + lo[1]
    X, Y = np.meshgrid(x, y, indexing="ij")
    return np.stack([X.ravel(), Y.ravel()], 1).astype(np.float32), ext


def boundary_distance(v, ix, pts):
    """Unsigned distance to the polyline (float64; zero-length segments are points)."""
    v = v.astype(np.float64)
    a, b = v[ix[:, 0]], v[ix[:, 1]]
    d = b - a
    dd = (d * d).sum(1)
    deg = dd == 0
    dd[deg] = 1.0
    out = np.empty(len(pts))
    for s in range(0, len(pts), 2048):
        p = pts[s:s + 2048, None, :].astype(np.float64)
        t = np.clip(((p - a) * d).sum(2) / dd, 0.0, 1.0)
        c = a + t[..., None] * d
        out[s:s + 2048] = np.linalg.norm(p - c, axis=2).min(1)
    return out


def compare(masked, nonzero, v, ix, pts, ext, g):
    """Pass rule: every pixel the engine masks is zero in the reference image, except
    a residual of at most MAX_RESIDUAL pixels, each within RESIDUAL_BAND grid spacings
    of the boundary.  Returns a report dict."""
    masked = masked.reshape(g, g)
    bad = masked & nonzero
    report = {"masked": int(masked.sum()), "fixture_nonzero": int(nonzero.sum()),
              "masked_but_nonzero": int(bad.sum()),
              "unmasked_zero": int((~masked & ~nonzero).sum())}
    if bad.any():
        dist = boundary_distance(v, ix, pts.reshape(g, g, 2)[bad])
        report["residual_max_dist_spacings"] = float(dist.max() / float(max(ext) / g))
    return report
