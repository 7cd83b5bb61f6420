"""Synthetic workloads of BASELINE.json's configs.

Inputs mirror what the reference's caller hands to zombie_bindings:
  * query points: src/2d/models/base.py:226-251 (sample_random_2D(res^2) over the
    OBJ's vertex bbox, karman points inside the cylinder removed, base.py:239-241)
    or cell-centred grids (src/2d/utils/model_utils.py:3-20);
  * source grid: -div(u) sampled on sample_uniform_2D(1000, with_boundary=True)
    (model_split.py:230-243): shape (res_y+2, res_x+2), rows ~ y ('xy' meshgrid).
    The SIREN divergence is replaced by a smooth analytic field (no checkpoints).
"""
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SCENES = os.path.join(REPO, "scenes")

KARMAN_OBJ = os.path.join(SCENES, "geometry_1cyl_long_open.obj")
SQUARE_OBJ = os.path.join(SCENES, "square.obj")
CUBE_OBJ = os.path.join(SCENES, "cube.obj")

# examples/*/wost.json "solver" section (shared by all examples) with the
# BASELINE walk counts substituted per config.
SOLVER_BASE = {
    "maxWalkLength": 10000, "epsilonShell": 1e-3, "minStarShapedRadius": 1e-3,
    "ignoreDirichlet": True, "ignoreNeumann": False, "ignoreSource": False,
    "russianRouletteThreshold": 0.99, "setpsBeforeApplyingTikhonov": 0,
}
OUTPUT_BASE = {"gridRes": 300, "boundaryDistanceMask": 1e-3}
SCENE_BASE = {"absorptionCoeff": 350, "normalizeDomain": False, "flipOrientation": False,
              "isDoubleSided": False, "isWatertight": True}


def read_obj_vertices(path, dim):
    vs = []
    with open(path) as f:
        for line in f:
            t = line.split()
            if t and t[0] == "v":
                vs.append([float(c) for c in t[1:1 + dim]])
    return np.asarray(vs, np.float64)


def scene_size(path, dim=2):
    """[min_x, max_x, min_y, max_y(, min_z, max_z)] as src/2d/main.py:36-44 computes it."""
    v = read_obj_vertices(path, dim)
    out = []
    for k in range(dim):
        out += [float(v[:, k].min()), float(v[:, k].max())]
    return out


def uniform_grid_2d(resolution, size, with_boundary=True):
    """sample_uniform_2D (src/2d/utils/model_utils.py:3-20), meshgrid 'xy' -> [res_y(+2), res_x(+2), 2]."""
    if (size[1] - size[0]) > (size[3] - size[2]):
        res_x, res_y = resolution, int(resolution * (size[3] - size[2]) / (size[1] - size[0]))
    else:
        res_x, res_y = int(resolution * (size[1] - size[0]) / (size[3] - size[2])), resolution
    x = np.linspace(0.5, res_x - 0.5, res_x, dtype=np.float32)
    y = np.linspace(0.5, res_y - 0.5, res_y, dtype=np.float32)
    if with_boundary:
        x = np.concatenate([[0.0], x, [res_x * 1.0]]).astype(np.float32)
        y = np.concatenate([[0.0], y, [res_y * 1.0]]).astype(np.float32)
    X, Y = np.meshgrid(x, y, indexing="xy")
    X = X / res_x * (size[1] - size[0]) + size[0]
    Y = Y / res_y * (size[3] - size[2]) + size[2]
    return np.stack([X, Y], -1).astype(np.float32)


def karman_source(grid):
    x, y = grid[..., 0].astype(np.float64), grid[..., 1].astype(np.float64)
    return (np.sin(3 * x) * np.cos(2 * y) + 0.5 * np.cos(5 * x + 1)).astype(np.float32)


def karman_obstacle(size):
    """Cylinder centre/radius as src/2d/main.py:94-96 derives them (vertices strictly inside the bbox)."""
    v = read_obj_vertices(KARMAN_OBJ, 2)
    inside = (v[:, 0] > size[0]) & (v[:, 0] < size[1]) & (v[:, 1] > size[2]) & (v[:, 1] < size[3])
    ov = v[inside]
    c = ov.mean(0)
    r = np.mean(np.linalg.norm(ov - c, axis=1)) + OUTPUT_BASE["boundaryDistanceMask"]
    return c, r


def karman_points(n=65536, seed=1234):
    """sample_random_2D(256^2) over the scene bbox minus points in the cylinder (base.py:230-241)."""
    size = scene_size(KARMAN_OBJ)
    rng = np.random.default_rng(seed)
    u = rng.random((n, 2), dtype=np.float32)
    pts = np.empty_like(u)
    pts[:, 0] = u[:, 0] * (size[1] - size[0]) + size[0]
    pts[:, 1] = u[:, 1] * (size[3] - size[2]) + size[2]
    c, r = karman_obstacle(size)
    d = np.sqrt((pts[:, 0] - c[0]) ** 2 + (pts[:, 1] - c[1]) ** 2) - r
    return np.ascontiguousarray(pts[d > 0], dtype=np.float32)


def karman_grid_points(nx=256, ny=128):
    size = scene_size(KARMAN_OBJ)
    x = (np.arange(nx, dtype=np.float64) + 0.5) / nx * (size[1] - size[0]) + size[0]
    y = (np.arange(ny, dtype=np.float64) + 0.5) / ny * (size[3] - size[2]) + size[2]
    X, Y = np.meshgrid(x, y, indexing="xy")
    return np.stack([X.ravel(), Y.ravel()], -1).astype(np.float32)


def karman_config(n_walks=128, n_points=65536, seed=1234, grid_points=False):
    """Config B: karman 2D (geometry_1cyl_long_open.obj, lambda=350, 128 walks)."""
    size = scene_size(KARMAN_OBJ)
    grid = uniform_grid_2d(1000, size, with_boundary=True)
    src = karman_source(grid)
    pts = karman_grid_points() if grid_points else karman_points(n_points, seed)
    solver = dict(SOLVER_BASE, nWalks=n_walks)
    scene = dict(SCENE_BASE, boundary=KARMAN_OBJ)
    return {"name": "karman2d", "dim": 2, "scene": scene, "solver": solver, "output": dict(OUTPUT_BASE),
            "source": src, "points": pts, "obj": KARMAN_OBJ}


def taylorgreen_config(n_walks=32, res=32, flip=False):
    """Config A: taylorgreen 2D on square.obj, 32x32 cell-centred points, 32 walks.

    As shipped (flipOrientation false) square.obj's segments run clockwise, so their
    normals (s.y,-s.x) point INTO the square and the reference's insideDomain
    (fcpw_scene_loader.h:642-648) classifies every interior point as outside: the
    reference returns p = grad p = 0 there.  flip=True gives the meaningful problem."""
    size = scene_size(SQUARE_OBJ)
    L = size[1] - size[0]
    grid = uniform_grid_2d(1000, size, with_boundary=True)
    x, y = grid[..., 0].astype(np.float64), grid[..., 1].astype(np.float64)
    src = (np.cos(2 * np.pi * (x - size[0]) / L) * np.cos(np.pi * (y - size[2]) / L)).astype(np.float32)
    xs = (np.arange(res) + 0.5) / res * (size[1] - size[0]) + size[0]
    ys = (np.arange(res) + 0.5) / res * (size[3] - size[2]) + size[2]
    X, Y = np.meshgrid(xs, ys, indexing="xy")
    pts = np.stack([X.ravel(), Y.ravel()], -1).astype(np.float32)
    solver = dict(SOLVER_BASE, nWalks=n_walks)
    return {"name": "taylorgreen2d", "dim": 2, "scene": dict(SCENE_BASE, boundary=SQUARE_OBJ, flipOrientation=flip),
            "solver": solver, "output": dict(OUTPUT_BASE), "source": src, "points": pts, "obj": SQUARE_OBJ,
            "flip": flip}


def box_2d(L=1.0):
    """Unit box, counter-clockwise so segment normals (s.y,-s.x) point outward."""
    v = np.array([[0, 0], [L, 0], [L, L], [0, L]], np.float32)
    ix = np.array([[0, 1], [1, 2], [2, 3], [3, 0]], np.int32)
    return v, ix


def subdivided_cube(k=12, half=1.0):
    """[-half, half]^3 with every face split into k x k quads (2 k^2 triangles per face),
    shared vertices, wound like scenes/cube.obj (positive signed volume): a 3D mesh far
    beyond the LDS budget for the global-memory geometry path and its group hierarchy
    (no reference analogue: the reference's 3D meshes have 12 triangles)."""
    axes = {0: np.eye(3)[0], 1: np.eye(3)[1], 2: np.eye(3)[2]}
    faces = [(0, 1, 2, 1), (0, 2, 1, -1), (1, 2, 0, 1), (1, 0, 2, -1), (2, 0, 1, 1), (2, 1, 0, -1)]
    index, verts, tris = {}, [], []

    def vid(p):
        key = tuple(int(round(c * k / half)) for c in p)
        if key not in index:
            index[key] = len(verts)
            verts.append(p)
        return index[key]

    for n_ax, u_ax, v_ax, sgn in faces:
        n, u, v = axes[n_ax] * sgn, axes[u_ax], axes[v_ax]
        g = np.linspace(-half, half, k + 1)
        for a in range(k):
            for b in range(k):
                p00 = n * half + g[a] * u + g[b] * v
                p10 = n * half + g[a + 1] * u + g[b] * v
                p11 = n * half + g[a + 1] * u + g[b + 1] * v
                p01 = n * half + g[a] * u + g[b + 1] * v
                i00, i10, i11, i01 = vid(p00), vid(p10), vid(p11), vid(p01)
                tris.append((i00, i10, i11))
                tris.append((i00, i11, i01))
    return np.array(verts, np.float32), np.array(tris, np.int32)


def circle_2d(c, r, n=64, clockwise=True):
    """Polygonal circle.  Clockwise: normals (s.y,-s.x) point into the disk, i.e. out of
    a fluid that surrounds it (obstacle); counter-clockwise: fluid inside the disk."""
    t = (-1.0 if clockwise else 1.0) * np.arange(n) / n * 2 * np.pi
    v = np.stack([c[0] + r * np.cos(t), c[1] + r * np.sin(t)], -1).astype(np.float32)
    ix = np.stack([np.arange(n), (np.arange(n) + 1) % n], -1).astype(np.int32)
    return v, ix


def dirichlet_obstacle_config(n_walks=256, res=512, src_res=514):
    """Config C (synthetic, no reference analogue): unit-square Neumann box with an
    interior Dirichlet disk g=0 at (0.5,0.35), r=0.1; 512^2 cell-centred points."""
    v, ix = box_2d(1.0)
    dv, dix = circle_2d((0.5, 0.35), 0.1, 64)
    xs = (np.arange(src_res) + 0.5) / src_res
    X, Y = np.meshgrid(xs, xs, indexing="xy")
    src = (np.cos(np.pi * X) * np.cos(np.pi * Y)).astype(np.float32)
    g = (np.arange(res) + 0.5) / res
    PX, PY = np.meshgrid(g, g, indexing="xy")
    pts = np.stack([PX.ravel(), PY.ravel()], -1).astype(np.float32)
    solver = dict(SOLVER_BASE, nWalks=n_walks, ignoreDirichlet=False)
    return {"name": "box_dirichlet2d", "dim": 2, "vertices": v, "prims": ix, "dvertices": dv, "dprims": dix,
            "dirichlet_value": 0.0, "absorption": 350.0, "solver": solver, "output": dict(OUTPUT_BASE),
            "source": src, "points": pts}


def cube_config(res=128, n_walks=64, src_res=82):
    """Config D/E: cube.obj ([-1,1]^3), res^3 cell-centred points, 82^3 source grid."""
    xs = (np.arange(src_res) + 0.5) / src_res * 2 - 1
    X, Y, Z = np.meshgrid(xs, xs, xs, indexing="ij")
    src = (np.cos(np.pi * X / 2) * np.cos(np.pi * Y / 2) * np.cos(np.pi * Z / 2)).astype(np.float32)
    g = ((np.arange(res) + 0.5) / res * 2 - 1).astype(np.float32)
    PX, PY, PZ = np.meshgrid(g, g, g, indexing="ij")
    pts = np.stack([PX.ravel(), PY.ravel(), PZ.ravel()], -1).astype(np.float32)
    solver = dict(SOLVER_BASE, nWalks=n_walks)
    return {"name": f"cube3d_{res}", "dim": 3, "scene": dict(SCENE_BASE, boundary=CUBE_OBJ), "solver": solver,
            "output": dict(OUTPUT_BASE, gridRes=100), "source": src, "points": pts, "obj": CUBE_OBJ}


ENGINE_OBJ = os.path.join(SCENES, "engine_geometry.obj")


def engine_config(n_walks=64, n_points=4096, flip=False, seed=3):
    """The largest mesh the reference ships: the zombie demo's engine outline
    (bindings/zombie/demo/scenes/engine/data/geometry.obj, 647 segments in several
    loops), loaded with normalizeDomain (scene.h:104-145) and used here as an
    all-Neumann karman-style problem (lambda = 350, the wost.json solver) -- the
    capacity case for the LDS-staged kernels (beyond the star-grid limit of 255
    silhouette candidates).  Uniform random points over the bounding box; about
    half lie inside the fluid region (either orientation)."""
    from .engine import load_obj
    v, ix = load_obj(ENGINE_OBJ, 2, flip, True)
    lo, hi = v.min(0), v.max(0)
    rng = np.random.default_rng(seed)
    pts = rng.uniform(lo, hi, (n_points, 2)).astype(np.float32)
    X, Y = np.meshgrid(np.linspace(lo[0], hi[0], 203), np.linspace(lo[1], hi[1], 203), indexing="xy")
    src = (np.sin(3 * X) * np.cos(2 * Y) + 0.5 * np.cos(5 * X + 1)).astype(np.float32)
    solver = dict(SOLVER_BASE, nWalks=n_walks)
    scene = dict(SCENE_BASE, boundary=ENGINE_OBJ, normalizeDomain=True, flipOrientation=flip)
    return {"name": "engine2d", "dim": 2, "scene": scene, "solver": solver, "output": dict(OUTPUT_BASE),
            "source": src, "points": pts, "vertices": v, "prims": ix, "absorption": 350.0, "flip": flip}


def gear_config(n_teeth=160, n_walks=64, res=24, holes=3, seed=7):
    """Stress scene for the culling / compaction paths (no reference analogue):
    fluid inside a counter-clockwise gear (2*n_teeth segments alternating between
    radii 1.0 and 0.93 -> n_teeth reflex silhouette vertices) around `holes`
    clockwise polygonal obstacles.  With the defaults there are >128 silhouette
    candidates and >128 segments, i.e. more than one 16-group compaction chunk."""
    t = np.arange(2 * n_teeth) / (2 * n_teeth) * 2 * np.pi
    r = np.where(np.arange(2 * n_teeth) % 2 == 0, 1.0, 0.93)
    v = [np.stack([r * np.cos(t), r * np.sin(t)], -1).astype(np.float32)]
    ix = [np.stack([np.arange(2 * n_teeth), (np.arange(2 * n_teeth) + 1) % (2 * n_teeth)], -1).astype(np.int32)]
    base = 2 * n_teeth
    centres = [(0.35 * np.cos(a), 0.35 * np.sin(a)) for a in np.arange(holes) / max(1, holes) * 2 * np.pi + 0.3]
    for c in centres:
        hv, hix = circle_2d(c, 0.12, n=24, clockwise=True)
        v.append(hv)
        ix.append(hix + base)
        base += hv.shape[0]
    v = np.concatenate(v)
    ix = np.concatenate(ix)
    size = (np.array([-1.0, -1.0], np.float32) - 1e-3, np.array([1.0, 1.0], np.float32) + 1e-3)
    gy = np.linspace(size[0][1], size[1][1], 203)
    gx = np.linspace(size[0][0], size[1][0], 203)
    X, Y = np.meshgrid(gx, gy, indexing="xy")
    src = (np.sin(3 * X) * np.cos(2 * Y) + 0.5 * np.cos(5 * X + 1)).astype(np.float32)
    rng = np.random.default_rng(seed)
    ang = rng.uniform(0, 2 * np.pi, res * res)
    rad = 0.95 * np.sqrt(rng.uniform(0, 1, res * res))
    pts = np.stack([rad * np.cos(ang), rad * np.sin(ang)], -1).astype(np.float32)
    for c in centres:  # drop points inside the obstacles
        pts = pts[np.linalg.norm(pts - np.asarray(c, np.float32), axis=1) > 0.125]
    solver = dict(SOLVER_BASE, nWalks=n_walks)
    return {"name": "gear2d", "dim": 2, "vertices": v, "prims": ix, "source": src, "points": pts,
            "solver": solver, "output": dict(OUTPUT_BASE), "absorption": 350.0}



def _with_geometry(cfg, dim, flip=False):
    """Adds vertices / prims (the reference's OBJ parsing rules, engine.load_obj) to a
    config that names an OBJ, so every config has the same keys."""
    if "vertices" not in cfg:
        from .engine import load_obj
        cfg["vertices"], cfg["prims"] = load_obj(cfg["obj"], dim, flip, False)
    cfg.setdefault("absorption", float(cfg.get("scene", {}).get("absorptionCoeff", 350.0)))
    kw = {}
    if cfg.get("dprims") is not None:
        kw = {"dvertices": cfg["dvertices"], "dprims": cfg["dprims"], "dirichlet_value": 1.0}
    cfg["scene_kw"] = kw
    return cfg


# BASELINE.json configs by short name:
#   A  taylorgreen 2D, 32x32 points, 32 walks (maxWalkLength 10000; flipped to make
#      the points inside -- as shipped every point is outside and the solve is empty)
#   B  karman 2D, 64k random points (256^2 minus the cylinder), 128 walks (the metric)
#   B_grid  karman 2D, 256x128 grid, 128 walks
#   C  unit box + Dirichlet disk (synthetic), 512^2 points, 256 walks
#   D  cube 3D, 128^3 points, 64 walks
#   E  cube 3D, 256^3 points, 128 walks
CONFIG_NAMES = ("A", "A_robust", "B", "B_grid", "C", "D", "E")


def config_by_name(name, n_points=None):
    if name in ("A", "A_robust"):
        cfg = _with_geometry(taylorgreen_config(n_walks=32, res=32, flip=True), 2, flip=True)
        desc = "taylorgreen2d (flipped square.obj), 32x32 cell-centred points, 32 walks, maxWalkLength 10000"
        if name == "A_robust":
            # the same config with robust float semantics (solver extension key): finite
            # Yukawa members where the reference's overflow to NaN (SURVEY.md 7.2 part 4)
            cfg["solver"] = dict(cfg["solver"], robustFloatSemantics=True)
            desc += ", robust float semantics"
    elif name == "B":
        cfg = _with_geometry(karman_config(n_walks=128, n_points=n_points or 65536), 2)
        desc = (f"karman2d: geometry_1cyl_long_open.obj, lambda=350, RR 0.99, {cfg['points'].shape[0]} random "
                f"query pts ({n_points or 65536} minus cylinder), 128 walks/pt")
    elif name == "B_grid":
        cfg = _with_geometry(karman_config(n_walks=128, grid_points=True), 2)
        desc = "karman2d, 256x128 cell-centred grid, 128 walks/pt"
    elif name == "C":
        cfg = _with_geometry(dirichlet_obstacle_config(n_walks=256, res=512), 2)
        desc = "unit box (Neumann) + Dirichlet disk r=0.1 (synthetic), 512^2 points, 256 walks/pt"
    elif name in ("D", "E"):
        res, walks = (128, 64) if name == "D" else (256, 128)
        cfg = _with_geometry(cube_config(res=res, n_walks=walks), 3)
        desc = f"cube3d (cube.obj), {res}^3 cell-centred points, {walks} walks/pt, 82^3 source grid"
    else:
        raise KeyError(f"unknown config {name!r} (one of {CONFIG_NAMES})")
    cfg["config_name"] = name
    cfg["desc"] = desc
    cfg["dim"] = int(cfg["vertices"].shape[1])
    return cfg
