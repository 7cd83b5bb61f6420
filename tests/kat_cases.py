"""Analytic known-answer cases of the screened Poisson problem the WoSt estimator
solves, shared by the oracle KATs (tests/test_oracle.py) and the HIP-path KATs
(tests/test_gpu_kat.py).

The estimator integrates +G f (walk_on_stars.h:262-276) with the Yukawa Green's
function of -lap + lambda (distributions.h:573-832), so with zero-flux Neumann
walls it solves  -lap p + lambda p = f.  On an axis-aligned box a cosine mode
f = prod_k cos(m_k pi (x_k - a_k) / L_k) has zero normal derivative on every wall
and p = f / (lambda + sum_k (m_k pi / L_k)^2) exactly.
The source grid is sampled at cell centres of the FLT_EPSILON-padded bbox, the
layout the engine's nearest-texel lookup reads (scene.h:194-198, image.h:53-58;
scene_3d.h:120-126).  That lookup is piecewise constant on cells of width h centred
on the samples; the first-order error f(x) - f(centre) averages out over each cell,
so for balls spanning many cells the estimator's mean differs from the smooth
solution by O(h^2): `bias` below bounds it by (h^2 / 8) k^2 max|f| / lambda (three
times the cell-average estimate h^2 k^2 / 24), and the tolerances carry it.

Each case returns a dict: scene geometry, source grid, solver/output sections,
query points, the exact p and grad p at them, and the bias bound.
"""
import numpy as np
from scipy import special

from wos_amd import workloads

EPS32 = float(np.finfo(np.float32).eps)


def _solver(n_walks, **kw):
    return dict(workloads.SOLVER_BASE, nWalks=n_walks, **kw)


def box2d(lam=350.0, m=1, n=1, n_walks=128, npts=1500, res=1000, seed=0, side=1.0, robust=False):
    """Square [0, side]^2, Neumann walls, f = cos(m pi x / side) cos(n pi y / side).
    side = 2 pi is the Taylor-Green square's size: there balls reach mu R ~ 166 and the
    reference's float Bessel members overflow (SURVEY.md section 7.2 hard part 4) unless
    `robust` (solver key robustFloatSemantics) is set."""
    L = float(side)
    v, ix = workloads.box_2d(L)
    pmin, pmax = v.min(0) - EPS32, v.max(0) + EPS32
    ys = (np.arange(res) + 0.5) / res * (pmax[1] - pmin[1]) + pmin[1]
    xs = (np.arange(res) + 0.5) / res * (pmax[0] - pmin[0]) + pmin[0]
    X, Y = np.meshgrid(xs, ys)   # rows ~ y
    km, kn = m * np.pi / L, n * np.pi / L
    f = (np.cos(km * X) * np.cos(kn * Y)).astype(np.float32)
    pts = (np.random.default_rng(seed).uniform(0.05, 0.95, (npts, 2)) * L).astype(np.float32)
    k2 = km ** 2 + kn ** 2
    x, y = pts[:, 0].astype(np.float64), pts[:, 1].astype(np.float64)
    pe = np.cos(km * x) * np.cos(kn * y) / (lam + k2)
    gx = -km * np.sin(km * x) * np.cos(kn * y) / (lam + k2)
    gy = -kn * np.cos(km * x) * np.sin(kn * y) / (lam + k2)
    h = (pmax - pmin).max() / res
    bias = h * h / 8 * k2 / lam
    solver = _solver(n_walks, robustFloatSemantics=True) if robust else _solver(n_walks)
    tag = f"_side{L:.3g}" if L != 1.0 else ""
    return {"name": f"box2d_l{lam:g}_m{m}n{n}{tag}{'_robust' if robust else ''}", "dim": 2, "vertices": v,
            "prims": ix, "source": f, "absorption": lam, "solver": solver,
            "output": {"boundaryDistanceMask": 1e-3}, "points": pts, "p": pe, "grad": np.stack([gx, gy], -1),
            "bias": bias, "kw": {}}


def disk2d_dirichlet(lam=4.0, n_walks=256, npts=800, seed=3):
    """Disk of radius 1, Dirichlet g = 1, f = 0: p = I0(mu r)/I0(mu)."""
    mu = np.sqrt(lam)
    dv, dix = workloads.circle_2d((0.0, 0.0), 1.0, 256, clockwise=False)
    rng = np.random.default_rng(seed)
    r = np.sqrt(rng.uniform(0.0, 0.7 ** 2, npts))
    t = rng.uniform(0, 2 * np.pi, npts)
    pts = np.stack([r * np.cos(t), r * np.sin(t)], -1).astype(np.float32)
    pe = special.i0(mu * r) / special.i0(mu)
    gm = mu * special.i1(mu * r) / special.i0(mu)
    # walks stop in the epsilon shell (1e-3) and take g there (walk_on_stars.h:145,334-341),
    # and the 256-gon's inscribed circle differs from the unit circle by 1 - cos(pi/256)
    # ~ 7.5e-5: both shift p by at most |dp/dn| times that distance
    bias = mu * special.i1(mu) / special.i0(mu) * (1e-3 + 1e-4)
    return {"name": "disk2d_dirichlet", "dim": 2, "vertices": np.zeros((0, 2), np.float32),
            "prims": np.zeros((0, 2), np.int32), "source": np.zeros((2, 2), np.float32), "absorption": lam,
            "solver": _solver(n_walks, ignoreDirichlet=False, russianRouletteThreshold=0.0, maxWalkLength=10000),
            "output": {"boundaryDistanceMask": 1e-3}, "points": pts, "p": pe,
            "grad": np.stack([gm * np.cos(t), gm * np.sin(t)], -1), "bias": bias,
            "kw": {"dvertices": dv, "dprims": dix, "dirichlet_value": 1.0}}


def disk2d_neumann_flux(lam=10.0, mode=0, n_walks=128, npts=600, seed=4, n_seg=256, img_res=2048):
    """Unit disk (counter-clockwise polygon, n_seg sides), NON-ZERO Neumann data h, f = 0:
    the walks' Neumann term throughput * alpha * G * h / pdf (walk_on_stars.h:212-260) carries
    the whole solution.  mode 0: u = I0(mu r), h = mu I1(mu) (constant flux, a 1 x 1 image);
    mode 1: u = I1(mu r) cos(theta), h = mu I1'(mu) cos(theta) = mu (I0(mu) - I1(mu)/mu) x on the
    unit circle (a 1 x img_res image varying with x: the nearest-texel lookup is within half a
    texel of x).  The polygon's inscribed circle lies d = 1 - cos(pi/n_seg) inside the unit
    circle, and on a side the exact flux of u differs from the
    segment's h by a factor within [cos(pi/n_seg), 1/cos(pi/n_seg)] (second order in pi/n_seg,
    ~d); the texel offset (mode 1) adds |h'| ex / 2 img_res to the boundary data.  Bias bound:
    max|grad u| (= max h) times 3 d, plus that texel term."""
    mu = np.sqrt(lam)
    v, ix = workloads.circle_2d((0.0, 0.0), 1.0, n_seg, clockwise=False)
    rng = np.random.default_rng(seed)
    r = np.sqrt(rng.uniform(0.0, 0.85 ** 2, npts))
    t = rng.uniform(0, 2 * np.pi, npts)
    pts = np.stack([r * np.cos(t), r * np.sin(t)], -1).astype(np.float32)
    pmin = v.min(0) - EPS32
    ext = (v.max(0) + EPS32) - pmin
    box = (float(pmin[0]), float(pmin[1]), float(ext[0]), float(ext[1]))
    i1p = special.i0(mu) - special.i1(mu) / mu
    if mode == 0:
        pe = special.i0(mu * r)
        gr = mu * special.i1(mu * r)
        grad = np.stack([gr * np.cos(t), gr * np.sin(t)], -1)
        img = np.full((1, 1), mu * special.i1(mu), np.float32)
        hmax, texel = mu * special.i1(mu), 0.0
    else:
        # u = I1(mu r) x / r: grad = (I1'(mu r) mu - I1(mu r)/r) cos t r_hat - I1(mu r)/r sin t t_hat
        i1 = special.i1(mu * r)
        d1 = mu * (special.i0(mu * r) - special.i1(mu * r) / np.maximum(mu * r, 1e-12))
        pe = i1 * np.cos(t)
        ur, ut = d1 * np.cos(t), -i1 / np.maximum(r, 1e-12) * np.sin(t)
        grad = np.stack([ur * np.cos(t) - ut * np.sin(t), ur * np.sin(t) + ut * np.cos(t)], -1)
        xs = pmin[0] + (np.arange(img_res) + 0.5) / img_res * ext[0]
        img = (mu * i1p * xs).astype(np.float32)[None, :]
        hmax, texel = mu * i1p, mu * i1p * ext[0] / (2 * img_res)
    bias = hmax * 3.0 * (1.0 - np.cos(np.pi / n_seg)) + texel
    solver = _solver(n_walks, ignoreSource=True, ignoreNeumann=False)
    return {"name": f"disk2d_neumann_l{lam:g}_mode{mode}", "dim": 2, "vertices": v, "prims": ix,
            "source": np.zeros((2, 2), np.float32), "absorption": lam, "solver": solver,
            "output": {"boundaryDistanceMask": 1e-3}, "points": pts, "p": pe, "grad": grad, "bias": bias,
            "kw": {"neumann_image": img, "neumann_image_box": box}}


def cube3d(lam=350.0, m=1, n=1, l=1, n_walks=128, npts=600, res=82, seed=5, scale=1.0, robust=False):
    """scenes/cube.obj (the reference's examples/*/cube.obj, [-1,1]^3 up to 1e-6), scaled
    by `scale`, Neumann walls, f = cos(m pi (x+s)/2s) cos(n pi (y+s)/2s) cos(l pi (z+s)/2s):
    the 3D analogue of the box KAT.  res^3 source grid, [X][Y][Z].
    scale 3 puts balls at mu R ~ 194 (lambda 350): the reference's float members
    (expmuR, sinhmuR) under/overflow there unless `robust`."""
    import objparse
    v, ix = objparse.load(workloads.CUBE_OBJ, 3)
    S = float(scale)
    v = (v * np.float32(S)).astype(np.float32)
    pmin, pmax = v.min(0) - EPS32, v.max(0) + EPS32
    axes = [(np.arange(res) + 0.5) / res * (pmax[k] - pmin[k]) + pmin[k] for k in range(3)]
    X, Y, Z = np.meshgrid(*axes, indexing="ij")
    kx, ky, kz = m * np.pi / (2 * S), n * np.pi / (2 * S), l * np.pi / (2 * S)
    f = (np.cos(kx * (X + S)) * np.cos(ky * (Y + S)) * np.cos(kz * (Z + S))).astype(np.float32)
    pts = (np.random.default_rng(seed).uniform(-0.9, 0.9, (npts, 3)) * S).astype(np.float32)
    x, y, z = (pts[:, k].astype(np.float64) for k in range(3))
    k2 = kx ** 2 + ky ** 2 + kz ** 2
    cx, cy, cz = np.cos(kx * (x + S)), np.cos(ky * (y + S)), np.cos(kz * (z + S))
    sx, sy, sz = np.sin(kx * (x + S)), np.sin(ky * (y + S)), np.sin(kz * (z + S))
    pe = cx * cy * cz / (lam + k2)
    ge = np.stack([-kx * sx * cy * cz, -ky * cx * sy * cz, -kz * cx * cy * sz], -1) / (lam + k2)
    h = (pmax - pmin).max() / res
    bias = h * h / 8 * k2 / lam
    solver = _solver(n_walks, robustFloatSemantics=True) if robust else _solver(n_walks)
    tag = f"_x{S:g}" if S != 1.0 else ""
    return {"name": f"cube3d_l{lam:g}_m{m}{n}{l}{tag}{'_robust' if robust else ''}", "dim": 3, "vertices": v,
            "prims": ix, "source": f, "absorption": lam, "solver": solver,
            "output": {"boundaryDistanceMask": 1e-3}, "points": pts, "p": pe, "grad": ge, "bias": bias, "kw": {}}


def check_unbiased(p, g, case, rel_tol, n_sigma=4.0):
    """Aggregate checks of one solve against the exact field (independent points):
    the mean error is within n_sigma standard errors (+ the lookup bias), and the
    RMS error is a small fraction of the field."""
    pe, ge, bias = case["p"], case["grad"], case["bias"]
    err = p - pe
    assert abs(err.mean()) < n_sigma * err.std() / np.sqrt(err.size) + bias, (err.mean(), err.std(), bias)
    assert np.sqrt(np.mean(err ** 2)) < rel_tol * np.sqrt(np.mean(pe ** 2))
    gerr = g - ge
    assert np.abs(gerr.mean(0)).max() < n_sigma * gerr.std(0).max() / np.sqrt(err.size) + 5 * bias, gerr.mean(0)
    assert np.sqrt(np.mean(gerr ** 2)) < 2.5 * rel_tol * np.sqrt(np.mean(ge ** 2))


def per_point_z(runs_p, runs_g, case):
    """Per-point z-scores of the seed-averaged estimate against the exact field: K
    independent solves (different RNG keys) give the per-point standard error
    sigma_hat / sqrt(K); the lookup bias bound is added in quadrature."""
    P = np.asarray(runs_p, np.float64)
    G = np.asarray(runs_g, np.float64)
    K = P.shape[0]
    se_p = P.std(0, ddof=1) / np.sqrt(K)
    se_g = G.std(0, ddof=1) / np.sqrt(K)
    zp = (P.mean(0) - case["p"]) / np.sqrt(se_p ** 2 + case["bias"] ** 2 + 1e-30)
    zg = (G.mean(0) - case["grad"]) / np.sqrt(se_g ** 2 + (5 * case["bias"]) ** 2 + 1e-30)
    return zp, zg


def check_z(zp, zg, n_sigma=4.0):
    """Per-point acceptance: with K seeds the z-scores follow ~Student-t(K-1)
    (E z^2 = 1.15 for K = 16).  Bar: mean z^2 < 1.5, at most 1 % of the points beyond
    n_sigma, no point beyond 8, and no systematic shift of the mean z."""
    for z in (zp, zg.ravel()):
        assert np.mean(z ** 2) < 1.5, np.mean(z ** 2)
        assert np.mean(np.abs(z) > n_sigma) <= 0.01, np.mean(np.abs(z) > n_sigma)
        assert np.abs(z).max() < 8.0, np.abs(z).max()
        assert abs(z.mean()) < 4.5 / np.sqrt(z.size) + 0.05, z.mean()


def z_with_bias_floor(runs_p, runs_g, case, rel_floor=5e-4):
    """per_point_z with the bias term raised to rel_floor * rms(p).  Used where the
    seed-averaged per-point standard error (~1e-4 of p on the 2 pi square at lambda
    350) falls below the estimator's own near-wall bias (~2e-4 of p on average within
    one unit of a wall -- present alike in the reference semantics at lambda 80, where
    the reference and robust modes are bit-identical, tests/test_oracle.py)."""
    c = dict(case, bias=max(case["bias"], rel_floor * float(np.sqrt(np.mean(case["p"] ** 2)))))
    return per_point_z(runs_p, runs_g, c)


def _l_points(rng, npts, margin, near_corner):
    """Uniform points of the L-shape [0,2]x[0,1] U [0,1]x[1,2] at least `margin` from its
    walls, plus `near_corner` points within 0.3 of the reflex vertex (1, 1)."""
    pts = []
    while len(pts) < npts:
        q = rng.uniform(margin, 2 - margin, 2)
        if q[0] <= 1 - margin or q[1] <= 1 - margin:
            pts.append(q)
    k = 0
    while k < near_corner:
        q = 1.0 + rng.uniform(-0.3, 0.3, 2)
        if (q[0] <= 1 - margin or q[1] <= 1 - margin) and np.all(q >= margin) and np.hypot(*(q - 1)) > margin:
            pts.append(q)
            k += 1
    return np.asarray(pts)


def lshape2d(lam=50.0, m=1, n=1, n_walks=128, npts=1200, near_corner=300, res=800, seed=7):
    """Non-convex Neumann KAT: the L-shape [0,2]x[0,1] U [0,1]x[1,2]
    (three unit squares, counter-clockwise so normals (s.y,-s.x) point out), zero-flux
    walls, f = cos(m pi x) cos(n pi y).  Every wall lies on an integer line, where f's
    normal derivative vanishes, so p = f / (lambda + pi^2 (m^2 + n^2)) exactly on the
    L.  The reflex vertex (1, 1) is the scene's one silhouette candidate (its dihedral
    angle is not below 1e-3, scene.h:84-90), so the star radius of every point that
    sees both of its segments from opposite sides is set by it
    (computeStarRadius, fcpw_scene_loader.h:621-641) -- the path no convex KAT reaches."""
    v = np.array([[0, 0], [2, 0], [2, 1], [1, 1], [1, 2], [0, 2]], np.float32)
    ix = np.array([[0, 1], [1, 2], [2, 3], [3, 4], [4, 5], [5, 0]], np.int32)
    pmin, pmax = v.min(0) - EPS32, v.max(0) + EPS32
    ys = (np.arange(res) + 0.5) / res * (pmax[1] - pmin[1]) + pmin[1]
    xs = (np.arange(res) + 0.5) / res * (pmax[0] - pmin[0]) + pmin[0]
    X, Y = np.meshgrid(xs, ys)   # rows ~ y
    km, kn = m * np.pi, n * np.pi
    f = (np.cos(km * X) * np.cos(kn * Y)).astype(np.float32)
    pts = _l_points(np.random.default_rng(seed), npts, 0.03, near_corner).astype(np.float32)
    k2 = km ** 2 + kn ** 2
    x, y = pts[:, 0].astype(np.float64), pts[:, 1].astype(np.float64)
    pe = np.cos(km * x) * np.cos(kn * y) / (lam + k2)
    gx = -km * np.sin(km * x) * np.cos(kn * y) / (lam + k2)
    gy = -kn * np.cos(km * x) * np.sin(kn * y) / (lam + k2)
    h = (pmax - pmin).max() / res
    return {"name": f"lshape2d_l{lam:g}_m{m}n{n}", "dim": 2, "vertices": v, "prims": ix, "source": f,
            "absorption": lam, "solver": _solver(n_walks), "output": {"boundaryDistanceMask": 1e-3},
            "points": pts, "p": pe, "grad": np.stack([gx, gy], -1), "bias": h * h / 8 * k2 / lam, "kw": {}}


def lprism3d(lam=50.0, m=1, n=1, l=1, n_walks=128, npts=600, near_corner=150, res=96, seed=9):
    """3D analogue: the L-shape extruded over z in [0, 1] (12 vertices, 20 triangles wound
    like scenes/cube.obj: (b-a)x(c-a) points out), f = cos(m pi x) cos(n pi y) cos(l pi z),
    p = f / (lambda + pi^2 (m^2 + n^2 + l^2)).  The reflex edge x = y = 1 is the one
    silhouette edge candidate (edge_silhouettes.inl:83-111, sbvh.inl:405-421); the
    triangulation's flat diagonals are ignored (dihedral angle 0)."""
    poly = np.array([[0, 0], [2, 0], [2, 1], [1, 1], [1, 2], [0, 2]], np.float64)
    v = np.concatenate([np.c_[poly, np.zeros(6)], np.c_[poly, np.ones(6)]]).astype(np.float32)
    tris = []
    for a in range(6):  # side walls: quad (a, b, b+6, a+6), outward for a CCW polygon
        b = (a + 1) % 6
        tris += [(a, b, b + 6), (a, b + 6, a + 6)]
    fan = [(0, 1, 2), (0, 2, 3), (0, 3, 4), (0, 4, 5)]   # star-shaped from vertex 0
    tris += [(a, c, b) for a, b, c in fan]                # bottom (z = 0): facing -z
    tris += [(a + 6, b + 6, c + 6) for a, b, c in fan]    # top (z = 1): facing +z
    ix = np.array(tris, np.int32)
    pmin, pmax = v.min(0) - EPS32, v.max(0) + EPS32
    axes = [(np.arange(res) + 0.5) / res * (pmax[k] - pmin[k]) + pmin[k] for k in range(3)]
    X, Y, Z = np.meshgrid(*axes, indexing="ij")
    kx, ky, kz = m * np.pi, n * np.pi, l * np.pi
    f = (np.cos(kx * X) * np.cos(ky * Y) * np.cos(kz * Z)).astype(np.float32)
    rng = np.random.default_rng(seed)
    xy = _l_points(rng, npts, 0.04, near_corner)
    pts = np.c_[xy, rng.uniform(0.04, 0.96, len(xy))].astype(np.float32)
    x, y, z = (pts[:, k].astype(np.float64) for k in range(3))
    k2 = kx ** 2 + ky ** 2 + kz ** 2
    cx, cy, cz = np.cos(kx * x), np.cos(ky * y), np.cos(kz * z)
    sx, sy, sz = np.sin(kx * x), np.sin(ky * y), np.sin(kz * z)
    pe = cx * cy * cz / (lam + k2)
    ge = np.stack([-kx * sx * cy * cz, -ky * cx * sy * cz, -kz * cx * cy * sz], -1) / (lam + k2)
    h = (pmax - pmin).max() / res
    return {"name": f"lprism3d_l{lam:g}_m{m}{n}{l}", "dim": 3, "vertices": v, "prims": ix, "source": f,
            "absorption": lam, "solver": _solver(n_walks), "output": {"boundaryDistanceMask": 1e-3},
            "points": pts, "p": pe, "grad": ge, "bias": h * h / 8 * k2 / lam, "kw": {}}
