"""Helpers for the pin against the reference's own engine-demo outputs
(bindings/zombie/demo/scenes/engine/solutions/{wost,bvc}.pfm, stored with the demo's boundary
images in tests/golden/engine_scene.npz by tests/golden/make_engine_scene.py).

The upstream demo solved scenes/engine/wost.json on data/geometry.obj (byte-identical to
scenes/engine_geometry.obj here) with a Scene that the fork has since changed: its boundary was
split into Dirichlet and Neumann parts by data/is_neumann.png, g came from
data/dirichlet_boundary_value.pfm, the domain was normalised (normalizeDomain, scene.h:132-142)
and its bounding box was square (computeBoundingBox(..., makeSquare = true, ...)).  Rebuilt with
those conventions (upstream_scene below; DESIGN.md "What pins the oracle" 4), the writer's zeroing
rule (grid.h:316-319: outside, or within boundaryDistanceMask = 1e-2 of either boundary) reproduces
the zero pattern of both images pixel for pixel, and the estimator's values agree with wost.pfm
within its own Monte-Carlo error (96 walks).
"""
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENGINE_OBJ = os.path.join(REPO, "scenes", "engine_geometry.obj")
SCENE_FIXTURE = os.path.join(REPO, "tests", "golden", "engine_scene.npz")
MASK = 1e-2  # scenes/engine/wost.json output.boundaryDistanceMask


def bbox(v):
    """computeBoundingBox(vertices, false, 1.0) with fcpw's FLT_EPSILON padding
    (fcpw_scene_loader.h:76-93, bounding_volumes.h:43-47)."""
    eps = np.float32(np.finfo(np.float32).eps)
    return (v - eps).min(0).astype(np.float32), (v + eps).max(0).astype(np.float32)


def grid_points(lo, hi, g):
    """createSolutionGrid (grid.h:35-52): point idx = i*g + j at
    ((i / float(g)) * extent.x + bMin.x, (j / float(g)) * extent.y + bMin.y), in float."""
    ext = (hi - lo).astype(np.float32)
    t = (np.arange(g, dtype=np.float32) / np.float32(g)).astype(np.float32)
    X, Y = np.meshgrid((t * ext[0]).astype(np.float32) + lo[0], (t * ext[1]).astype(np.float32) + lo[1],
                       indexing="ij")
    return np.stack([X.ravel(), Y.ravel()], 1).astype(np.float32)


def boundary_distance(v, ix, pts):
    """Unsigned distance to the polyline (float64; zero-length segments are points)."""
    v = v.astype(np.float64)
    a, b = v[ix[:, 0]], v[ix[:, 1]]
    d = b - a
    dd = (d * d).sum(1)
    dd[dd == 0] = 1.0
    out = np.empty(len(pts))
    for s in range(0, len(pts), 2048):
        p = pts[s:s + 2048, None, :].astype(np.float64)
        t = np.clip(((p - a) * d).sum(2) / dd, 0.0, 1.0)
        c = a + t[..., None] * d
        out[s:s + 2048] = np.linalg.norm(p - c, axis=2).min(1)
    return out


# ---------------------------------------------------------------------------------------------
# The value-level pin: the upstream engine demo's own scene (tests/golden/make_engine_scene.py)
# ---------------------------------------------------------------------------------------------
# scenes/engine/wost.json:3-11 as the solver reads it (demo.cpp:121-137): 96 walks,
# maxWalkLength 1024, epsilonShell 1e-3, harmonic (no absorptionCoeff), Dirichlet on, Neumann and
# source terms off; "minStarShapedRadius" is not a key the solver reads (minStarRadius keeps 1e-3)
WOST_SOLVER = {"nWalks": 96, "maxWalkLength": 1024, "epsilonShell": 1e-3, "minStarShapedRadius": 1e-3,
               "ignoreDirichlet": False, "ignoreNeumann": True, "ignoreSource": True}
WOST_OUTPUT = {"gridRes": 256, "boundaryDistanceMask": MASK}
WOST_WALKS = 96


def scene_fixture():
    d = np.load(SCENE_FIXTURE)
    n = int(d["is_neumann_shape"][0]) * int(d["is_neumann_shape"][1])
    out = {k: d[k] for k in ("dirichlet_image", "wost_values", "bvc_values")}
    out["is_neumann"] = np.unpackbits(d["is_neumann_bits"])[:n].reshape(d["is_neumann_shape"]).astype(bool)
    return out


def _subset(v, ix, sel):
    """separateBoundaries (upstream, restated): the selected segments in order, their vertices
    renumbered in order of first use -- each boundary type gets its own mesh and therefore its
    own vertex normals and silhouettes (scene.h:151-153)."""
    remap, vv, out = {}, [], []
    for a, b in ix[sel]:
        for q in (a, b):
            if q not in remap:
                remap[q] = len(vv)
                vv.append(v[q])
        out.append((remap[a], remap[b]))
    return np.asarray(vv, np.float32).reshape(-1, 2), np.asarray(out, np.int32).reshape(-1, 2)


def square_bbox(v):
    """computeBoundingBox(vertices, makeSquare = true, 1.0) (fcpw_scene_loader.h:75-93) in float:
    the FLT_EPSILON-padded box, then centre +- 0.5 * extent.maxCoeff() (centroid() =
    (pMin + pMax) * 0.5f, bounding_volumes.h:130-132)."""
    lo, hi = bbox(v)
    c = ((lo + hi) * np.float32(0.5)).astype(np.float32)
    half = np.float32(np.float32(0.5) * (hi - lo).astype(np.float32).max())
    return (c - half).astype(np.float32), (c + half).astype(np.float32)


def image_lookup(img, pts, origin, extent):
    """Image::get(uv) (image.h:53-58) at uv = (x - origin) / extent, in float."""
    uv = ((np.asarray(pts, np.float32) - origin) / extent).astype(np.float32)
    h, w = img.shape
    i = np.clip((uv[:, 1] * np.float32(h)).astype(np.int64), 0, h - 1)
    j = np.clip((uv[:, 0] * np.float32(w)).astype(np.int64), 0, w - 1)
    return img[i, j]


def upstream_scene(load_obj=None, normalize=True, square=True, flip=True):
    """The scene the upstream engine demo solved (DESIGN.md "What pins the oracle" 4): the OBJ
    loaded as the upstream Scene(json) did -- flipOrientation and normalizeDomain on (the OBJ
    recentred and scaled to unit radius, scene.h:132-142) and a SQUARE bounding box
    (computeBoundingBox(vertices, true, 1.0); the fork passes false, scene.h:144) -- split by
    onNeumannBoundary at the segment midpoints (scene.h:79-82 with that box), and g from the
    Dirichlet image over the same box (uv = (x - pMin) / maxLength, scene.h:202-207).
    normalize / square / flip = False give the fork's conventions instead (negative controls).
    Returns a dict: neumann / dirichlet meshes (v, ix), dirichlet_image, box (x0, y0, ex, ey),
    pts (the 256^2 createSolutionGrid points over the square box, point i*256 + j),
    values (the reference's wost.pfm, flattened the same way)."""
    if load_obj is None:
        from wos_amd import engine
        load_obj = engine.load_obj
    fx = scene_fixture()
    v, ix = load_obj(ENGINE_OBJ, 2, flip, normalize)
    lo, hi = square_bbox(v) if square else bbox(v)
    ext = (hi - lo).astype(np.float32)
    max_len = np.float32(ext.max())
    mid = (np.float32(0.5) * (v[ix[:, 0]] + v[ix[:, 1]])).astype(np.float32)
    neu = image_lookup(fx["is_neumann"].astype(np.float32), mid, lo, max_len) > 0
    g = int(fx["wost_values"].shape[0])
    pts = grid_points(lo, hi, g)
    return {"neumann": _subset(v, ix, neu), "dirichlet": _subset(v, ix, ~neu),
            "n_neumann": int(neu.sum()), "dirichlet_image": fx["dirichlet_image"],
            "box": np.array([lo[0], lo[1], max_len, max_len], np.float32), "pts": pts,
            "values": fx["wost_values"].ravel(), "bvc_values": fx["bvc_values"].ravel(), "grid_res": g,
            "v": v, "ix": ix}


def near_boundary(v, ix, pts, r):
    """dist(pt, polyline) < r for every point (float64 distances): candidate pairs from a k-d
    tree over the points, around each segment's midpoint, then the exact segment distance."""
    from scipy.spatial import cKDTree
    v = v.astype(np.float64)
    P = np.asarray(pts, np.float64)
    a, b = v[ix[:, 0]], v[ix[:, 1]]
    half = 0.5 * np.linalg.norm(b - a, axis=1)
    tree = cKDTree(P)
    out = np.zeros(len(P), bool)
    for s, cands in enumerate(tree.query_ball_point(0.5 * (a + b), half + r)):
        if not cands:
            continue
        q = P[cands]
        d = b[s] - a[s]
        dd = float(d @ d)
        t = np.clip(((q - a[s]) @ d) / dd, 0.0, 1.0) if dd > 0 else np.zeros(len(q))
        out[np.asarray(cands)[np.linalg.norm(q - (a[s] + t[:, None] * d), axis=1) < r]] = True
    return out


def writer_mask(inside, near_dirichlet, near_neumann):
    """saveSolutionGrid's zeroing rule (grid.h:316-319): outside, or within the mask distance
    (output.boundaryDistanceMask) of either boundary."""
    return ~inside | near_dirichlet | near_neumann
