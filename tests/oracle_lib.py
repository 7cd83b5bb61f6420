"""ctypes bindings to the CPU oracle (oracle/build/libwos_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product path never loads this library.
"""
import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "libwos_oracle.so")


class SceneDesc(C.Structure):
    _fields_ = [
        ("dim", C.c_int32), ("n_vertices", C.c_int32), ("n_prims", C.c_int32),
        ("vertices", C.POINTER(C.c_float)), ("prims", C.POINTER(C.c_int32)),
        ("n_dvertices", C.c_int32), ("n_dprims", C.c_int32),
        ("dvertices", C.POINTER(C.c_float)), ("dprims", C.POINTER(C.c_int32)),
        ("dirichlet_value", C.c_float), ("absorption", C.c_float),
        ("is_watertight", C.c_int32), ("is_double_sided", C.c_int32),
        ("source", C.POINTER(C.c_float)), ("source_dims", C.c_int32 * 3),
        ("dirichlet_image", C.POINTER(C.c_float)), ("dirichlet_image_dims", C.c_int32 * 2),
        ("dirichlet_image_box", C.c_float * 4),
        ("neumann_image", C.POINTER(C.c_float)), ("neumann_image_dims", C.c_int32 * 2),
        ("neumann_image_box", C.c_float * 4),
    ]


class Params(C.Structure):
    _fields_ = [
        ("n_walks", C.c_int32), ("max_walk_length", C.c_int32),
        ("steps_before_tikhonov", C.c_int32), ("steps_before_maximal_spheres", C.c_int32),
        ("epsilon_shell", C.c_float), ("min_star_radius", C.c_float),
        ("silhouette_precision", C.c_float), ("russian_roulette_threshold", C.c_float),
        ("boundary_distance_mask", C.c_float),
        ("disable_gradient_control_variates", C.c_int32),
        ("disable_gradient_antithetic_variates", C.c_int32),
        ("use_cosine_sampling", C.c_int32), ("ignore_dirichlet", C.c_int32),
        ("ignore_neumann", C.c_int32), ("ignore_source", C.c_int32),
        ("seed", C.c_uint64), ("math_mode", C.c_int32), ("n_threads", C.c_int32),
        ("robust_float", C.c_int32),
    ]


class BvcParams(C.Structure):
    _fields_ = [("n_walks_solution", C.c_int32), ("n_walks_gradient", C.c_int32),
                ("boundary_cache_size", C.c_int32), ("domain_cache_size", C.c_int32),
                ("grid_res", C.c_int32), ("use_finite_differences", C.c_int32),
                ("normal_offset", C.c_float), ("radius_clamp", C.c_float),
                ("kernel_regularization", C.c_float), ("grid_box", C.c_float * 4)]


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "walk_steps", "wasted_steps", "walks_recorded", "walks_escaped",
        "walks_max_length", "walks_rr", "walks_dirichlet", "points_estimated",
        "rejection_iters")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = C.CDLL(ORACLE_SO)
        L.oracle_solve.restype = C.c_int
        L.oracle_solve.argtypes = [C.POINTER(SceneDesc), C.POINTER(Params), C.c_void_p, C.c_int64,
                                   C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.POINTER(Stats)]
        L.oracle_solve_m2.restype = C.c_int
        L.oracle_solve_m2.argtypes = [C.POINTER(SceneDesc), C.POINTER(Params), C.c_void_p, C.c_int64,
                                      C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.POINTER(Stats)]
        L.oracle_point_info.restype = C.c_int
        L.oracle_point_info.argtypes = [C.POINTER(SceneDesc), C.c_void_p] + [C.c_void_p] * 6
        L.oracle_bessel.restype = C.c_double
        L.oracle_bessel.argtypes = [C.c_int, C.c_double, C.c_int]
        L.oracle_math.restype = C.c_double
        L.oracle_math.argtypes = [C.c_int, C.c_double, C.c_int]
        L.oracle_seed32.restype = C.c_uint32
        L.oracle_seed32.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32]
        L.oracle_bvc.restype = C.c_int
        L.oracle_bvc.argtypes = [C.POINTER(SceneDesc), C.POINTER(Params), C.POINTER(BvcParams), C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.POINTER(Stats)]
        L.oracle_lhs.restype = C.c_int
        L.oracle_lhs.argtypes = [C.c_uint32, C.c_int, C.c_int, C.c_void_p]
        L.oracle_fcpw_pick.restype = C.c_int
        L.oracle_fcpw_pick.argtypes = [C.POINTER(SceneDesc), C.c_void_p, C.c_float, C.c_int, C.c_void_p, C.c_void_p,
                                       C.c_void_p]
        L.oracle_fcpw_bvh.restype = C.c_int
        L.oracle_fcpw_bvh.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        _lib = L
    return _lib


def _fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float)) if a is not None else None


def _iptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32)) if a is not None else None


class OracleScene:
    """Keeps numpy buffers alive for the SceneDesc pointers."""

    def __init__(self, vertices, prims, source, absorption, *, dvertices=None, dprims=None,
                 dirichlet_value=0.0, dirichlet_image=None, dirichlet_image_box=None, neumann_image=None,
                 neumann_image_box=None, watertight=True, double_sided=False):
        self.v = np.ascontiguousarray(vertices, dtype=np.float32)
        self.ix = np.ascontiguousarray(prims, dtype=np.int32)
        self.dim = int(self.v.shape[1])
        self.dv = None if dvertices is None else np.ascontiguousarray(dvertices, dtype=np.float32)
        self.dix = None if dprims is None else np.ascontiguousarray(dprims, dtype=np.int32)
        self.src = np.ascontiguousarray(source, dtype=np.float32)
        d = SceneDesc()
        d.dim = self.dim
        d.n_vertices, d.n_prims = self.v.shape[0], self.ix.shape[0]
        d.vertices, d.prims = _fptr(self.v), _iptr(self.ix)
        if self.dv is not None:
            d.n_dvertices, d.n_dprims = self.dv.shape[0], self.dix.shape[0]
            d.dvertices, d.dprims = _fptr(self.dv), _iptr(self.dix)
        d.dirichlet_value = dirichlet_value
        d.absorption = absorption
        d.is_watertight = int(watertight)
        d.is_double_sided = int(double_sided)
        d.source = _fptr(self.src)
        dims = list(self.src.shape) + [0] * (3 - self.src.ndim)
        for k in range(3):
            d.source_dims[k] = dims[k]
        self.dimg = None if dirichlet_image is None else np.ascontiguousarray(dirichlet_image, dtype=np.float32)
        if self.dimg is not None:
            d.dirichlet_image = _fptr(self.dimg)
            d.dirichlet_image_dims[0], d.dirichlet_image_dims[1] = self.dimg.shape
            for k in range(4):
                d.dirichlet_image_box[k] = float(dirichlet_image_box[k])
        self.nimg = None if neumann_image is None else np.ascontiguousarray(neumann_image, dtype=np.float32)
        if self.nimg is not None:
            d.neumann_image = _fptr(self.nimg)
            d.neumann_image_dims[0], d.neumann_image_dims[1] = self.nimg.shape
            for k in range(4):
                d.neumann_image_box[k] = float(neumann_image_box[k])
        self.desc = d


def make_params(solver=None, output=None, *, seed=0x5EED0001, math_mode=0, n_threads=None):
    """Build oracle params from the reference's JSON dicts (demo.cpp:121-137, grid.h:159)."""
    s = dict(solver or {})
    o = dict(output or {})
    p = Params()
    p.n_walks = int(s.get("nWalks", 128))
    p.max_walk_length = int(s.get("maxWalkLength", 1024))
    p.steps_before_tikhonov = int(s.get("setpsBeforeApplyingTikhonov", p.max_walk_length))
    p.steps_before_maximal_spheres = int(s.get("setpsBeforeUsingMaximalSpheres", p.max_walk_length))
    p.epsilon_shell = float(s.get("epsilonShell", 1e-3))
    p.min_star_radius = float(s.get("minStarRadius", 1e-3))
    p.silhouette_precision = float(s.get("silhouettePrecision", 1e-3))
    p.russian_roulette_threshold = float(s.get("russianRouletteThreshold", 0.0))
    p.boundary_distance_mask = float(o.get("boundaryDistanceMask", 0.0))
    p.disable_gradient_control_variates = int(bool(s.get("disableGradientControlVariates", False)))
    p.disable_gradient_antithetic_variates = int(bool(s.get("disableGradientAntitheticVariates", False)))
    p.use_cosine_sampling = int(bool(s.get("useCosineSamplingForDirectionalDerivatives", False)))
    p.ignore_dirichlet = int(bool(s.get("ignoreDirichlet", False)))
    p.ignore_neumann = int(bool(s.get("ignoreNeumann", False)))
    p.ignore_source = int(bool(s.get("ignoreSource", False)))
    p.seed = int(s.get("seed", seed))
    p.math_mode = math_mode
    p.n_threads = n_threads or default_threads()
    p.robust_float = int(bool(s.get("robustFloatSemantics", False)))
    return p


def default_threads():
    """Threads for the oracle: the CPUs this process may run on, capped by the
    job's CPU share when the environment states one (OMP_NUM_THREADS; 16 on a
    one-GPU box, whose os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def solve(scene: OracleScene, params: Params, pts, index_base=0, index_stride=1, m2=False):
    """(p, grad, n_est, steps, stats); with m2=True also the per-point Welford M2 of the
    solution estimates (sample variance = m2 / (n_est - 1)) as a sixth element."""
    pts = np.ascontiguousarray(pts, dtype=np.float32)
    n = pts.shape[0]
    p = np.zeros(n, np.float32)
    g = np.zeros((n, scene.dim), np.float32)
    nest = np.zeros(n, np.int32)
    steps = np.zeros(n, np.int32)
    sm2 = np.zeros(n, np.float32) if m2 else None
    st = Stats()
    rc = lib().oracle_solve_m2(C.byref(scene.desc), C.byref(params), pts.ctypes.data, n,
                               index_base, index_stride, p.ctypes.data, g.ctypes.data,
                               nest.ctypes.data, steps.ctypes.data,
                               sm2.ctypes.data if m2 else None, C.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle_solve failed rc={rc}")
    if m2:
        return p, g, nest, steps, st.as_dict(), sm2
    return p, g, nest, steps, st.as_dict()


def point_info(scene: OracleScene, pt):
    pt = np.ascontiguousarray(pt, dtype=np.float32)
    out = [C.c_float(), C.c_float(), C.c_float(), C.c_int32(), C.c_float(), C.c_int32()]
    rc = lib().oracle_point_info(C.byref(scene.desc), pt.ctypes.data, *[C.addressof(o) for o in out])
    if rc != 0:
        raise RuntimeError("oracle_point_info failed")
    keys = ["dirichlet_dist", "neumann_dist", "signed_neumann_dist", "inside", "star_radius", "n_silhouettes"]
    return {k: o.value for k, o in zip(keys, out)}


def fcpw_pick(scene: OracleScene, x, R, us):
    """fcpw's stochastic traversal at ball (x, R) for each uniform in us: (primitive or -1, selection pdf)."""
    xr = np.asarray(x, np.float32).ravel()
    x = np.zeros(3, np.float32)
    x[:len(xr)] = xr
    us = np.ascontiguousarray(us, np.float32)
    sel = np.zeros(len(us), np.int32)
    pdf = np.zeros(len(us), np.float32)
    rc = lib().oracle_fcpw_pick(C.byref(scene.desc), x.ctypes.data, float(R), len(us), us.ctypes.data,
                                sel.ctypes.data, pdf.ctypes.data)
    assert rc == 0, rc
    return sel, pdf


def fcpw_bvh(v, ix, dim, branch=4, leaf=8):
    """The oracle's restatement of fcpw's wide BVH: (box [n, branch, 6], child [n, branch], ref)."""
    v = np.ascontiguousarray(v, np.float32)
    ix = np.ascontiguousarray(ix, np.int32)
    cap = 2 * ix.shape[0] + 8
    box = np.zeros(cap * branch * 6, np.float32)
    child = np.zeros(cap * branch, np.int32)
    ref = np.zeros(ix.shape[0], np.int32)
    n = C.c_int(0)
    rc = lib().oracle_fcpw_bvh(dim, v.ctypes.data, v.shape[0], ix.ctypes.data, ix.shape[0], branch, leaf,
                               box.ctypes.data, child.ctypes.data, ref.ctypes.data, cap, C.byref(n))
    assert rc == 0, rc
    return box[:n.value * branch * 6].reshape(n.value, branch, 6), child[:n.value * branch].reshape(n.value, branch), ref


def lhs(seed, n, dims):
    out = np.zeros(n * dims, np.float32)
    lib().oracle_lhs(seed, n, dims, out.ctypes.data)
    return out


def seed32(key, idx, pair, tag):
    return int(lib().oracle_seed32(key, idx, pair, tag))


def bvc_params(solver=None, output=None, grid_box=None):
    """Oracle copy of the BVC keys (demo.cpp:269-290), same defaults as the product's;
    grid_box = (x0, y0, ex, ey) of the evaluation grid (None: the scene's bounding box)."""
    s = dict(solver or {})
    o = dict(output or {})
    b = BvcParams()
    eps = float(s.get("epsilonShell", 1e-3))
    b.n_walks_solution = int(s.get("nWalksForCachedSolutionEstimates", 128))
    b.n_walks_gradient = int(s.get("nWalksForCachedGradientEstimates", 640))
    b.boundary_cache_size = int(s.get("boundaryCacheSize", 1024))
    b.domain_cache_size = int(s.get("domainCacheSize", 1024))
    b.grid_res = int(o["gridRes"])
    b.use_finite_differences = int(bool(s.get("useFiniteDifferencesForBoundaryDerivatives", False)))
    b.normal_offset = float(s.get("normalOffsetForCachedDirichletSamples", 5.0 * eps))
    b.radius_clamp = float(s.get("radiusClampForKernels", 1e-3))
    b.kernel_regularization = float(s.get("regularizationForKernels", 0.0))
    for k in range(4):
        b.grid_box[k] = 0.0 if grid_box is None else float(grid_box[k])
    return b


def bvc(scene: OracleScene, params: Params, bp: BvcParams):
    """oracle_bvc: (solution [g, g], grad [g, g, 2], samples [k, 8], counts, stats)."""
    g = int(bp.grid_res)
    sol = np.zeros(g * g, np.float32)
    grad = np.zeros(g * g * 2, np.float32)
    cap = 2 * int(bp.boundary_cache_size) + 4 * int(bp.domain_cache_size) + 16
    samples = np.zeros(cap * 8, np.float32)
    counts = np.zeros(4, np.int64)
    st = Stats()
    rc = lib().oracle_bvc(C.byref(scene.desc), C.byref(params), C.byref(bp), sol.ctypes.data, grad.ctypes.data,
                          samples.ctypes.data, cap, counts.ctypes.data, C.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle_bvc failed rc={rc}")
    return (sol.reshape(g, g), grad.reshape(g, g, 2), samples[:int(counts[3]) * 8].reshape(-1, 8).copy(),
            counts, st.as_dict())
