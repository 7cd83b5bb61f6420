"""GPU parity: the HIP kernel (through the C ABI) vs the CPU oracle restatement.

Bar: bit-exact on fixed seeds.  Both sides run the same counter-based RNG layout
and the same deterministic math (det mode), with -ffp-contract=off on both, so
every rejection / roulette decision, every walk and every Welford update must
agree exactly.  Full-size (64k point) runs are checked through properties that
do not need the oracle (determinism, shard invariance, finiteness, agreement of
aggregate statistics with an oracle subset).
"""
import numpy as np
import torch
import pytest

import objparse
from wos_amd import WosScene, selftest_math, solver_params, workloads
from wos_amd._lib import SCHED_GEOM_GLOBAL

pytestmark = pytest.mark.gpu


def _oracle_math_mode_det(oracle, which, x):
    return np.array([oracle.lib().oracle_math(which if which < 5 else which, float(v), 0) for v in x])


@pytest.mark.parametrize("which,lo,hi", [(0, -745, 709), (1, 1e-300, 1e300), (2, -20, 20), (3, -20, 20),
                                         (4, -50, 50), (5, 0, 1e6)])
def test_math_double_bit_exact(gpu, oracle, which, lo, hi):
    rng = np.random.default_rng(which)
    if which == 1 or which == 5:
        x = np.exp(rng.uniform(np.log(max(lo, 1e-300)), np.log(hi), 20000))
    else:
        x = rng.uniform(lo, hi, 20000)
    got = selftest_math(which, x)
    if which == 5:
        ref = np.sqrt(x)
    else:
        ref = np.array([oracle.lib().oracle_math(which, float(v), 0) for v in x])
    np.testing.assert_array_equal(got.view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("which", [6, 7, 8, 9])
def test_bessel_bit_exact(gpu, oracle, which):
    rng = np.random.default_rng(which)
    x = np.concatenate([rng.uniform(1e-4, 4.0, 5000), rng.uniform(3.7, 120.0, 5000), [2.0, 3.75, 1e-3]])
    got = selftest_math(which, x)
    ref = np.array([oracle.lib().oracle_bessel(which - 6, float(v), 0) for v in x])
    np.testing.assert_array_equal(got.view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("which,ref", [(18, 0), (19, 1), (20, 2), (21, 3), (22, 2), (23, 3)])
def test_fused_bessel_bit_exact(gpu, oracle, which, ref):
    """bessel_ik (one evaluation of the shared exp/log/sqrt pieces for I0, I1, K0, K1,
    as the ball update and the Green's function use it) == the separate A&S functions"""
    rng = np.random.default_rng(which)
    x = np.concatenate([rng.uniform(1e-4, 4.0, 5000), rng.uniform(3.7, 120.0, 5000), [2.0, 3.75, 1e-3, 1.9999999]])
    got = selftest_math(which, x)
    want = np.array([oracle.lib().oracle_bessel(ref, float(v), 0) for v in x])
    np.testing.assert_array_equal(got.view(np.uint64), want.view(np.uint64))


@pytest.mark.parametrize("which", [10, 11, 12, 13, 14])
def test_math_float_bit_exact(gpu, oracle, which):
    rng = np.random.default_rng(which)
    if which == 11:
        x = np.exp(rng.uniform(-80, 80, 20000)).astype(np.float32).astype(np.float64)
    elif which == 14:
        x = rng.uniform(0, 1, 20000).astype(np.float32).astype(np.float64)
    else:
        x = rng.uniform(-20, 20, 20000).astype(np.float32).astype(np.float64)
    got = selftest_math(which, x)
    ref = np.array([oracle.lib().oracle_math(which, float(v), 0) for v in x])
    np.testing.assert_array_equal(got, ref)


def assert_bits_equal(a, b):
    """Bitwise equality; NaNs must sit at the same places (their payload/sign bits are
    platform-defined: x86 default NaN is negative, the GPU's positive)."""
    na, nb = np.isnan(a), np.isnan(b)
    np.testing.assert_array_equal(na, nb)
    np.testing.assert_array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def _pair(cfg, oracle, dim=2):
    v, ix = objparse.load(cfg["obj"], dim, flip=cfg.get("flip", False))
    lam = float(cfg["scene"]["absorptionCoeff"])
    osc = oracle.OracleScene(v, ix, cfg["source"], lam, watertight=True)
    sc = WosScene(v, ix, cfg["source"], lam, watertight=True)
    return osc, sc


def _compare(oracle, osc, sc, cfg, pts, seed=0x5EED0001, schedule=0):
    prm_o = oracle.make_params(cfg["solver"], cfg["output"], seed=seed, math_mode=0)
    p0, g0, ne0, st0, s0 = oracle.solve(osc, prm_o, pts)
    prm = solver_params(cfg["solver"], cfg["output"], seed=seed, schedule=schedule)
    p1, g1, s1, ne1, st1 = sc.solve(pts, prm, counts=True)
    np.testing.assert_array_equal(ne1, ne0)
    np.testing.assert_array_equal(st1, st0)
    assert_bits_equal(p1, p0)
    assert_bits_equal(g1, g0)
    for k in ("walk_steps", "wasted_steps", "walks_recorded", "walks_escaped", "walks_rr",
              "points_estimated", "rejection_iters"):
        assert s1[k] == s0[k], k
    return p1, g1, s1


def test_karman_bit_exact(gpu, oracle):
    cfg = workloads.karman_config(n_walks=128)
    osc, sc = _pair(cfg, oracle)
    pts = cfg["points"][:2048]
    _compare(oracle, osc, sc, cfg, pts)


def test_karman_grid_and_edges_bit_exact(gpu, oracle):
    """256x128 grid subset + points outside the domain / on the open ends / near walls."""
    cfg = workloads.karman_config(n_walks=128, grid_points=True)
    osc, sc = _pair(cfg, oracle)
    pts = cfg["points"][::16]
    c, r = workloads.karman_obstacle(workloads.scene_size(workloads.KARMAN_OBJ))
    extra = np.array([[c[0], c[1]], [c[0] + r * 0.5, c[1]], [-1.2, 0.0], [2.0, 0.0], [0.0, 0.5995],
                      [0.0, -0.5980], [-1.1032, 0.1], [1.9067, -0.2], [0.0, 0.0]], np.float32)
    _compare(oracle, osc, sc, cfg, np.concatenate([pts, extra]))


@pytest.mark.parametrize("nw", [1, 2, 5, 32, 200])
def test_walk_counts_bit_exact(gpu, oracle, nw):
    """odd / tiny / >64-pair walk counts (multiple statistics chunks)."""
    cfg = workloads.karman_config(n_walks=nw)
    osc, sc = _pair(cfg, oracle)
    _compare(oracle, osc, sc, cfg, cfg["points"][:256])


@pytest.mark.parametrize("flag", ["disableGradientControlVariates", "disableGradientAntitheticVariates",
                                  "useCosineSamplingForDirectionalDerivatives", "ignoreSource",
                                  "ignoreNeumann"])
def test_solver_flags_bit_exact(gpu, oracle, flag):
    cfg = workloads.karman_config(n_walks=64)
    cfg["solver"][flag] = True
    osc, sc = _pair(cfg, oracle)
    _compare(oracle, osc, sc, cfg, cfg["points"][:256])


def test_harmonic_then_tikhonov_bit_exact(gpu, oracle):
    cfg = workloads.karman_config(n_walks=64)
    cfg["solver"]["setpsBeforeApplyingTikhonov"] = 2
    cfg["solver"]["russianRouletteThreshold"] = 0.5
    cfg["solver"]["maxWalkLength"] = 64
    osc, sc = _pair(cfg, oracle)
    _compare(oracle, osc, sc, cfg, cfg["points"][:256])


@pytest.mark.parametrize("flip", [False, True])
def test_taylorgreen_bit_exact(gpu, oracle, flip):
    """Config A (square of side 2*pi).  As shipped every point is classified outside
    (zero output, like the reference); flipped, it exercises the float-overflow (NaN)
    regime of the 2D Yukawa kernel for large balls (SURVEY.md §7.2 hard part 4)."""
    cfg = workloads.taylorgreen_config(n_walks=32, res=16, flip=flip)
    cfg["solver"]["maxWalkLength"] = 200
    osc, sc = _pair(cfg, oracle)
    _compare(oracle, osc, sc, cfg, cfg["points"])


def test_dirichlet_obstacle_bit_exact(gpu, oracle):
    cfg = workloads.dirichlet_obstacle_config(n_walks=64, res=24)
    osc = oracle.OracleScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"],
                             dvertices=cfg["dvertices"], dprims=cfg["dprims"],
                             dirichlet_value=1.0, watertight=True)
    sc = WosScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], dvertices=cfg["dvertices"],
                  dprims=cfg["dprims"], dirichlet_value=1.0, watertight=True)
    _compare(oracle, osc, sc, cfg, cfg["points"])


def test_gear_many_groups_bit_exact(gpu, oracle):
    """>16 silhouette groups and >16 segment groups: the multi-chunk compaction
    rounds of the wave-cooperative star-radius and ray queries."""
    cfg = workloads.gear_config()
    osc = oracle.OracleScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], watertight=True)
    sc = WosScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], watertight=True)
    info = sc.info()
    assert info["n_silhouettes"] > 8 * 16 and info["n_prims"] > 8 * 16, info
    _compare(oracle, osc, sc, cfg, cfg["points"])


@pytest.mark.parametrize("flip", [False, True])
def test_engine_mesh_bit_exact(gpu, oracle, flip):
    """the reference's largest mesh (647 segments, zombie engine demo), normalized:
    more silhouette candidates than the star grid takes, several loops"""
    cfg = workloads.engine_config(n_walks=64, n_points=2048, flip=flip)
    osc = oracle.OracleScene(cfg["vertices"], cfg["prims"], cfg["source"], 350.0, watertight=True)
    sc = WosScene(cfg["vertices"], cfg["prims"], cfg["source"], 350.0, watertight=True)
    _, _, s1 = _compare(oracle, osc, sc, cfg, cfg["points"])
    assert s1["points_estimated"] > 600
    sc.close()


def test_open_box3d_silhouette_edges_bit_exact(gpu, oracle):
    """3D with silhouette edges (one face of the cube removed -> open edges, like the
    karman3d cube): edge silhouette candidates, 3D cone culling, the cooperative
    star-radius and rejection paths in 3D."""
    cfg = workloads.cube_config(res=10, n_walks=64)
    v, ix = objparse.load(cfg["obj"], 3)
    ix = ix[2:]
    lam = float(cfg["scene"]["absorptionCoeff"])
    osc = oracle.OracleScene(v, ix, cfg["source"], lam, watertight=False)
    sc = WosScene(v, ix, cfg["source"], lam, watertight=False)
    assert sc.info()["n_silhouettes"] > 0
    _compare(oracle, osc, sc, cfg, cfg["points"])


@pytest.mark.parametrize("dim", [2, 3])
def test_double_sided_bit_exact(gpu, oracle, dim):
    """isDoubleSided: every point is estimated, normals flip toward the walk's side
    (walk_on_stars.h:150-160), silhouettes use both orientations."""
    if dim == 2:
        cfg = workloads.karman_config(n_walks=32)
        v, ix = objparse.load(cfg["obj"], 2)
        pts = cfg["points"][:512]
    else:
        cfg = workloads.cube_config(res=8, n_walks=32)
        v, ix = objparse.load(cfg["obj"], 3)
        ix = ix[2:]
        pts = cfg["points"]
    lam = float(cfg["scene"]["absorptionCoeff"])
    osc = oracle.OracleScene(v, ix, cfg["source"], lam, watertight=True, double_sided=True)
    sc = WosScene(v, ix, cfg["source"], lam, watertight=True, double_sided=True)
    _compare(oracle, osc, sc, cfg, pts)


def _h_image(v, res=(37, 53)):
    """A smooth, sign-changing Neumann image over the padded bbox of `v` (rows ~ y)."""
    eps = np.float32(np.finfo(np.float32).eps)
    pmin = v.min(0) - eps
    ext = (v.max(0) + eps) - pmin
    y, x = np.meshgrid(np.linspace(0, 1, res[0]), np.linspace(0, 1, res[1]), indexing="ij")
    img = (np.sin(5 * x + 1) * np.cos(3 * y) + 0.3).astype(np.float32)
    return img, (float(pmin[0]), float(pmin[1]), float(ext[0]), float(ext[1]))


@pytest.mark.parametrize("case", ["disk", "karman", "karman_double_sided", "lshape"])
def test_neumann_data_bit_exact(gpu, oracle, case):
    """Image-valued Neumann data h (ABI 9): the walks' Neumann term at every step -- fcpw's
    stochastic boundary sample, the line-of-sight test, G, h at the sample
    (walk_on_stars.h:212-260), and in double-sided scenes the sample normal's flips
    (:219-247) -- GPU == oracle bit for bit: the flux disk KAT scene, karman (Yukawa
    lambda 350, the walk kernel with the Neumann term on), karman double-sided, the L."""
    import kat_cases
    if case == "disk":
        c = kat_cases.disk2d_neumann_flux(10.0, 1, npts=300, n_walks=32)
        v, ix, src, lam, kw = c["vertices"], c["prims"], c["source"], c["absorption"], dict(c["kw"])
        cfg, pts, ds = {"solver": c["solver"], "output": c["output"]}, c["points"], False
    elif case == "lshape":
        c = kat_cases.lshape2d(10.0, 2, 1)
        v, ix, src, lam = c["vertices"], c["prims"], c["source"], c["absorption"]
        img, box = _h_image(v)
        kw = {"neumann_image": img, "neumann_image_box": box}
        cfg, pts, ds = {"solver": c["solver"], "output": c["output"]}, c["points"][:400], False
    else:
        cfg = workloads.karman_config(n_walks=32)
        v, ix = objparse.load(cfg["obj"], 2)
        src, lam = cfg["source"], float(cfg["scene"]["absorptionCoeff"])
        img, box = _h_image(v)
        kw = {"neumann_image": img, "neumann_image_box": box}
        pts, ds = cfg["points"][:1024], case == "karman_double_sided"
    osc = oracle.OracleScene(v, ix, src, lam, watertight=True, double_sided=ds, **kw)
    sc = WosScene(v, ix, src, lam, watertight=True, double_sided=ds, **kw)
    p1, g1, _ = _compare(oracle, osc, sc, cfg, pts)
    # the term is live: h = 0 gives a different field
    sc0 = WosScene(v, ix, src, lam, watertight=True, double_sided=ds)
    p0, _, _ = sc0.solve(pts, solver_params(cfg["solver"], cfg["output"], seed=0x5EED0001))
    assert np.abs(p1 - p0).max() > 0
    sc.close()
    sc0.close()


@pytest.mark.parametrize("which", ["lshape2d", "lprism3d"])
def test_nonconvex_l_bit_exact(gpu, oracle, which):
    """The non-convex KAT scenes (kat_cases.lshape2d / lprism3d): the reflex vertex /
    edge is the star radius's only silhouette candidate, including the walks that leak
    through it and escape (dropped, walk_on_stars.h:280-286)."""
    import kat_cases
    c = kat_cases.lshape2d(10.0, 2, 1) if which == "lshape2d" else kat_cases.lprism3d(50.0, 1, 1, 1)
    cfg = {"solver": c["solver"], "output": c["output"]}
    osc = oracle.OracleScene(c["vertices"], c["prims"], c["source"], c["absorption"], watertight=True)
    sc = WosScene(c["vertices"], c["prims"], c["source"], c["absorption"], watertight=True)
    for seed in (0x5EED0001, 0x4C000003):
        _compare(oracle, osc, sc, cfg, c["points"], seed=seed)
    sc.close()


def test_cube3d_bit_exact(gpu, oracle):
    cfg = workloads.cube_config(res=10, n_walks=64)
    osc, sc = _pair(cfg, oracle, dim=3)
    _compare(oracle, osc, sc, cfg, cfg["points"])


@pytest.mark.parametrize("dim,npts", [(2, 1), (2, 3), (3, 1), (3, 3)])
def test_lone_walks_bit_exact(gpu, oracle, dim, npts):
    """Solves of one to three near-wall points: the long walks of such points leave the
    walk kernel's waves with one live walk for most iterations, where the register-only
    solo forms of the sampler, star-radius and ray queries run (round 3); the oracle must
    still agree bit for bit."""
    if dim == 2:
        cfg = workloads.karman_config(n_walks=128)
        osc, sc = _pair(cfg, oracle)
        pts = cfg["points"]
        # the points nearest the channel walls (y = +-0.6035) but not on them
        d = 0.6035 - np.abs(pts[:, 1])
        order = np.argsort(np.where(d > 2e-3, d, np.inf), kind="stable")
    else:
        cfg = workloads.cube_config(res=16, n_walks=128)
        osc, sc = _pair(cfg, oracle, dim=3)
        pts = cfg["points"]
        order = np.argsort(1.0 - np.abs(pts).max(axis=1), kind="stable")  # nearest a face
    sel = np.ascontiguousarray(pts[order[:npts]])
    _, _, st = _compare(oracle, osc, sc, cfg, sel)
    assert st["walk_steps"] > 0


def test_karman_full_size_properties(gpu, oracle):
    """64k points x 128 walks (BASELINE config B): determinism, shard invariance,
    finiteness, and the oracle on a strided subset matches bit for bit."""
    cfg = workloads.karman_config(n_walks=128)
    osc, sc = _pair(cfg, oracle)
    pts = cfg["points"]
    prm = solver_params(cfg["solver"], cfg["output"])
    p1, g1, s1 = sc.solve(pts, prm)
    p2, g2, s2 = sc.solve(pts, prm)
    np.testing.assert_array_equal(p1, p2)
    np.testing.assert_array_equal(g1, g2)
    assert np.isfinite(p1).all() and np.isfinite(g1).all()
    # shard invariance: odd-indexed points solved alone with their global indices
    pe, ge, _ = sc.solve(pts[1::2], prm, index_base=1, index_stride=2)
    np.testing.assert_array_equal(pe, p1[1::2])
    np.testing.assert_array_equal(ge, g1[1::2])
    # oracle subset at global indices
    sub = np.arange(0, pts.shape[0], 97)
    prm_o = oracle.make_params(cfg["solver"], cfg["output"], math_mode=0)
    po, go, _, _, _ = oracle.solve(osc, prm_o, pts[sub], index_base=0, index_stride=97)
    np.testing.assert_array_equal(po, p1[sub])
    np.testing.assert_array_equal(go, g1[sub])
    assert s1["walks_recorded"] > 0.9 * 128 * pts.shape[0]


@pytest.mark.parametrize("scene", ["karman", "gear", "cube", "dirichlet"])
def test_geometry_from_global_memory_bit_exact(gpu, oracle, scene):
    """WOS_SCHED_GEOM_GLOBAL: the kernels read the geometry records through L2 instead of
    staging them in LDS (the path of scenes too large for LDS) -- same results."""
    if scene == "karman":
        cfg = workloads.karman_config(n_walks=64)
        osc, sc = _pair(cfg, oracle)
        pts = cfg["points"][:512]
    elif scene == "gear":
        cfg = workloads.gear_config(n_walks=32, res=16)
        osc = oracle.OracleScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], watertight=True)
        sc = WosScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], watertight=True)
        pts = cfg["points"]
    elif scene == "cube":
        cfg = workloads.cube_config(res=8, n_walks=32)
        osc, sc = _pair(cfg, oracle, dim=3)
        pts = cfg["points"]
    else:
        cfg = workloads.dirichlet_obstacle_config(n_walks=64, res=16)
        kw = dict(dvertices=cfg["dvertices"], dprims=cfg["dprims"], dirichlet_value=1.0, watertight=True)
        osc = oracle.OracleScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], **kw)
        sc = WosScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], **kw)
        pts = cfg["points"]
    _, _, st = _compare(oracle, osc, sc, cfg, pts, schedule=SCHED_GEOM_GLOBAL)
    assert st["geom_global"] == 1
    sc.close()


def test_mesh_beyond_lds_bit_exact(gpu, oracle):
    """a 12 000-segment boundary (192 KB of records: more than a CU's LDS) runs with
    the geometry in global memory and matches the oracle"""
    cfg = workloads.gear_config(n_teeth=6000, n_walks=16, res=6)
    osc = oracle.OracleScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], watertight=True)
    sc = WosScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], watertight=True)
    _, _, st = _compare(oracle, osc, sc, cfg, cfg["points"])
    assert st["geom_global"] == 1 and st["points_estimated"] > 0
    sc.close()


def test_mesh3d_beyond_lds_tree_bit_exact(gpu, oracle):
    """a 6912-triangle cube (subdivided faces; records far beyond the LDS budget): the
    global-memory geometry path with the group hierarchy (ray, star radius, closest
    point by group bounds) matches the oracle's brute-force scans"""
    v, ix = workloads.subdivided_cube(24)
    cfg = workloads.cube_config(res=6, n_walks=16)
    osc = oracle.OracleScene(v, ix, cfg["source"], 350.0, watertight=True)
    sc = WosScene(v, ix, cfg["source"], 350.0, watertight=True)
    _, _, st = _compare(oracle, osc, sc, cfg, cfg["points"])
    assert st["geom_global"] == 1 and st["points_estimated"] == cfg["points"].shape[0]
    sc.close()


def test_dirichlet_many_segments_tree_bit_exact(gpu, oracle):
    """a 4096-segment Dirichlet obstacle: the Dirichlet distance through the group
    hierarchy (nearest-bound descent + pruned depth-first walk) and the grouped closest
    point match the oracle's sequential scans"""
    cfg = workloads.dirichlet_obstacle_config(n_walks=16, res=16)
    dv, dix = workloads.circle_2d((0.5, 0.35), 0.1, 4096)
    kw = dict(dvertices=dv, dprims=dix, dirichlet_value=1.0, watertight=True)
    osc = oracle.OracleScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], **kw)
    sc = WosScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], **kw)
    _, _, st = _compare(oracle, osc, sc, cfg, cfg["points"])
    assert st["walks_dirichlet"] > 0
    sc.close()


@pytest.mark.parametrize("which", ["C_dirichlet512", "D_cube128"])
def test_full_size_configs_properties(gpu, oracle, which):
    """BASELINE configs C (Dirichlet obstacle, 512^2 points x 256 walks) and D (cube,
    128^3 points x 64 walks) at full size: determinism, shard invariance (the strided
    half solved alone), finiteness, the Dirichlet maximum principle bound, and the
    oracle on a sparse strided subset, bit for bit."""
    if which == "C_dirichlet512":
        cfg = workloads.dirichlet_obstacle_config(n_walks=256, res=512)
        kw = dict(dvertices=cfg["dvertices"], dprims=cfg["dprims"], dirichlet_value=1.0, watertight=True)
        osc = oracle.OracleScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], **kw)
        sc = WosScene(cfg["vertices"], cfg["prims"], cfg["source"], cfg["absorption"], **kw)
        stride = 4099
    else:
        cfg = workloads.cube_config(res=128, n_walks=64)
        osc, sc = _pair(cfg, oracle, dim=3)
        stride = 32771
    pts = np.ascontiguousarray(cfg["points"])
    prm = solver_params(cfg["solver"], cfg["output"])
    x = torch.from_numpy(pts).to(torch.device("cuda", 0))
    p1, g1, s1 = sc.solve(x, prm)
    p2, g2, _ = sc.solve(x, prm)
    p1, g1, p2, g2 = (t.cpu().numpy() for t in (p1, g1, p2, g2))
    np.testing.assert_array_equal(p1.view(np.uint32), p2.view(np.uint32))
    np.testing.assert_array_equal(g1.view(np.uint32), g2.view(np.uint32))
    assert np.isfinite(p1).all() and np.isfinite(g1).all()
    pe, ge, _ = sc.solve(x[1::2].contiguous(), prm, index_base=1, index_stride=2)
    np.testing.assert_array_equal(pe.cpu().numpy().view(np.uint32), p1[1::2].view(np.uint32))
    np.testing.assert_array_equal(ge.cpu().numpy().view(np.uint32), g1[1::2].view(np.uint32))
    sub = np.arange(0, pts.shape[0], stride)
    prm_o = oracle.make_params(cfg["solver"], cfg["output"], math_mode=0)
    po, go, _, _, _ = oracle.solve(osc, prm_o, pts[sub], index_base=0, index_stride=stride)
    assert_bits_equal(p1[sub], po)
    assert_bits_equal(g1[sub], go)
    assert s1["walk_steps"] > 0 and s1["points_estimated"] > 0.5 * pts.shape[0]
    sc.close()


@pytest.mark.parametrize("name", ["karman_small", "taylorgreen_small", "box_dirichlet_small", "cube_small"])
def test_gpu_matches_golden_fixture(gpu, name):
    import os
    import make_golden_cases as cases
    ref = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"{name}.npz"))
    p, g = cases.run_case_gpu(name)
    assert_bits_equal(p, ref["p"])
    assert_bits_equal(g, ref["grad"])


@pytest.mark.parametrize("which,ref_which", [(16, 0), (17, 2), (24, 0), (25, 2)])
def test_fast_bessel_error_within_certified_band(gpu, oracle, which, ref_which):
    """The float Bessel approximations of the rejection fast path must stay well inside
    the 8e-6 relative band the kernel certifies its decisions with."""
    x = np.concatenate([np.geomspace(1e-4, 2.0, 4000), np.linspace(2.0, 80.0, 8000)])
    x = x.astype(np.float32).astype(np.float64)
    got = selftest_math(which, x)
    ref = np.array([oracle.lib().oracle_bessel(ref_which, float(v), 0) for v in x])
    rel = np.abs(got - ref) / np.abs(ref)
    assert rel.max() < 2e-6, rel.max()


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [2, 3])
def test_empty_single_and_outside_batches(gpu, oracle, dim):
    """Degenerate batches the time-stepper can hand over: no points (empty outputs, zero
    counters), one point, and points that all lie outside the domain (p = grad p = 0, no
    walks) -- host and device inputs alike; the single point equals the oracle bit for bit."""
    import torch
    if dim == 2:
        cfg = workloads.karman_config(n_walks=32)
        v, ix = objparse.load(cfg["obj"], 2)
        outside = np.array([[-100.0, -100.0], [100.0, 50.0]], np.float32)
    else:
        cfg = workloads.cube_config(res=8, n_walks=16)
        v, ix = objparse.load(cfg["obj"], 3)
        outside = np.array([[2.0, 0.0, 0.0], [0.0, -3.0, 0.5]], np.float32)
    prm = solver_params(cfg["solver"], cfg["output"])
    sc = WosScene(v, ix, cfg["source"], 350.0, watertight=True)
    try:
        p, g, st = sc.solve(np.zeros((0, dim), np.float32), prm)
        assert p.shape == (0,) and g.shape == (0, dim) and st["walk_steps"] == 0 and st["walks_recorded"] == 0
        pd, gd, _ = sc.solve(torch.zeros((0, dim), device="cuda"), prm)
        assert pd.shape == (0,) and gd.shape == (0, dim)
        one = np.ascontiguousarray(cfg["points"][3:4])
        p1, g1, st1 = sc.solve(one, prm)
        po, go, _, _, _ = oracle.solve(oracle.OracleScene(v, ix, cfg["source"], 350.0),
                                       oracle.make_params(cfg["solver"], cfg["output"]), one, index_base=3)
        assert st1["walks_recorded"] > 0
        p1b, g1b, _ = sc.solve(one, prm, index_base=3)
        assert_bits_equal(p1b, po)
        assert_bits_equal(g1b, go)
        p0, g0, st0 = sc.solve(outside, prm)
        assert np.array_equal(p0, np.zeros(2, np.float32)) and np.array_equal(g0, np.zeros((2, dim), np.float32))
        assert st0["walk_steps"] == 0 and st0["points_estimated"] == 0
    finally:
        sc.close()
