"""Host-side API of the MI355X walk-on-stars engine (thin layer over include/wos.h).

Mirrors the reference's operator interface for the pressure solve:
  Scene(config, source)   <-> bindings/zombie/demo/scene.h:54-77 (2D),
                              bindings/zombie3d/demo/scene_3d.h:22-40 (3D)
  solve(points)           <-> runWalkOnStars_sampled, demo.cpp:119-205 /
                              runWalkOnStars_3d, zombie3d/demo/demo.cpp:15-116
Inputs may be numpy arrays (host) or torch tensors already on the GPU (zero-copy:
device pointers are handed to the C ABI and the kernel runs on torch's current
stream).
"""
import ctypes as C
import os

import numpy as np

from . import _lib
from ._lib import BvcParams, SceneDesc, SceneInfo, SolverParams, Stats, WosError, check

_DEFAULT_SEED = 0x5EED0001


def load_obj(path, dim, flip_orientation=False, normalize=False):
    """OBJ -> (vertices [V,dim] f32, prims [P,dim] i32) with the reference's parsing rules."""
    L = _lib.load()
    m = _lib.Mesh()
    check(L.wos_load_obj(os.fsencode(path), dim, int(flip_orientation), int(normalize), C.byref(m)),
          f"wos_load_obj({path})")
    try:
        v = np.ctypeslib.as_array(m.vertices, shape=(m.n_vertices * dim,)).copy().reshape(-1, dim)
        ix = np.ctypeslib.as_array(m.prims, shape=(m.n_prims * dim,)).copy().reshape(-1, dim)
    finally:
        L.wos_mesh_free(C.byref(m))
    return v.astype(np.float32), ix.astype(np.int32)


def _get_opt(d, key, default, typ):
    v = d.get(key, default) if d is not None else default
    return typ(v)


def solver_params(solver=None, output=None, seed=None, schedule=0):
    """Parse the reference's wost.json "solver" / "output" sections (demo.cpp:121-137,
    grid.h:159), same keys (including the misspelled `setps...`) and defaults."""
    s = dict(solver or {})
    o = dict(output or {})
    p = SolverParams()
    _lib.load().wos_default_params(C.byref(p))
    p.n_walks = _get_opt(s, "nWalks", 128, int)
    p.max_walk_length = _get_opt(s, "maxWalkLength", 1024, int)
    p.steps_before_tikhonov = _get_opt(s, "setpsBeforeApplyingTikhonov", p.max_walk_length, int)
    p.steps_before_maximal_spheres = _get_opt(s, "setpsBeforeUsingMaximalSpheres", p.max_walk_length, int)
    p.epsilon_shell = _get_opt(s, "epsilonShell", 1e-3, float)
    p.min_star_radius = _get_opt(s, "minStarRadius", 1e-3, float)
    p.silhouette_precision = _get_opt(s, "silhouettePrecision", 1e-3, float)
    p.russian_roulette_threshold = _get_opt(s, "russianRouletteThreshold", 0.0, float)
    p.boundary_distance_mask = _get_opt(o, "boundaryDistanceMask", 0.0, float)
    p.disable_gradient_control_variates = int(bool(s.get("disableGradientControlVariates", False)))
    p.disable_gradient_antithetic_variates = int(bool(s.get("disableGradientAntitheticVariates", False)))
    p.use_cosine_sampling = int(bool(s.get("useCosineSamplingForDirectionalDerivatives", False)))
    p.ignore_dirichlet = int(bool(s.get("ignoreDirichlet", False)))
    p.ignore_neumann = int(bool(s.get("ignoreNeumann", False)))
    p.ignore_source = int(bool(s.get("ignoreSource", False)))
    p.seed = int(seed if seed is not None else s.get("seed", _DEFAULT_SEED)) & 0xFFFFFFFFFFFFFFFF
    # extension key (no reference analogue): robust float semantics, SURVEY.md 7.2 hard part 4
    p.robust_float = int(bool(s.get("robustFloatSemantics", False)))
    # GPU scheduling switches (_lib.SCHED_*): never change a result
    p.schedule = int(schedule)
    return p


def bvc_params(solver=None, output=None, grid_box=None):
    """The boundary-value-caching keys runBoundaryValueCaching reads (demo.cpp:269-290):
    same names and defaults; output.gridRes is required.  grid_box = (x0, y0, ex, ey): the
    rectangle of the evaluation grid (None: the scene's bounding box, demo.cpp:311)."""
    s = dict(solver or {})
    o = dict(output or {})
    if "gridRes" not in o:
        raise KeyError("Missing required setting: gridRes")
    b = BvcParams()
    _lib.load().wos_default_bvc_params(C.byref(b))
    eps = _get_opt(s, "epsilonShell", 1e-3, float)
    b.n_walks_solution = _get_opt(s, "nWalksForCachedSolutionEstimates", 128, int)
    b.n_walks_gradient = _get_opt(s, "nWalksForCachedGradientEstimates", 640, int)
    b.boundary_cache_size = _get_opt(s, "boundaryCacheSize", 1024, int)
    b.domain_cache_size = _get_opt(s, "domainCacheSize", 1024, int)
    b.grid_res = int(o["gridRes"])
    b.use_finite_differences = int(bool(s.get("useFiniteDifferencesForBoundaryDerivatives", False)))
    b.normal_offset = _get_opt(s, "normalOffsetForCachedDirichletSamples", 5.0 * eps, float)
    b.radius_clamp = _get_opt(s, "radiusClampForKernels", 1e-3, float)
    b.kernel_regularization = _get_opt(s, "regularizationForKernels", 0.0, float)
    if grid_box is not None:
        for k in range(4):
            b.grid_box[k] = float(grid_box[k])
    return b


def _is_torch(x):
    return type(x).__module__.startswith("torch")


class WosScene:
    """Geometry + source field resident on one GPU."""

    def __init__(self, vertices, prims, source=None, absorption=0.0, *, dvertices=None, dprims=None,
                 dirichlet_value=0.0, dirichlet_image=None, dirichlet_image_box=None, neumann_image=None,
                 neumann_image_box=None, watertight=True, double_sided=False, device=0):
        """dirichlet_image (2D, optional): g as an image [H, W] (row ~ y) over the rectangle
        dirichlet_image_box = (x0, y0, ex, ey), evaluated at each walk's projection onto the
        Dirichlet boundary (the upstream demo's pde.dirichlet, scene.h:202-207); replaces the
        constant dirichlet_value.  neumann_image (2D, optional): the Neumann data h as an image
        [H, W] over neumann_image_box, evaluated at the walks' stochastic boundary samples and at
        BVC's Neumann samples (the upstream demo's pde.neumann, scene.h:175-181); default h = 0."""
        L = _lib.load()
        v = np.ascontiguousarray(vertices, dtype=np.float32)
        ix = np.ascontiguousarray(prims, dtype=np.int32)
        self.dim = int(v.shape[1])
        if self.dim not in (2, 3) or ix.ndim != 2 or ix.shape[1] != self.dim:
            raise WosError("vertices must be [V,2|3] and prims [P,dim]")
        d = SceneDesc()
        d.dim = self.dim
        d.vertices = v.ctypes.data_as(C.POINTER(C.c_float))
        d.prims = ix.ctypes.data_as(C.POINTER(C.c_int32))
        d.n_vertices, d.n_prims = v.shape[0], ix.shape[0]
        keep = [v, ix]
        if dprims is not None and len(dprims):
            dv = np.ascontiguousarray(dvertices, dtype=np.float32)
            dix = np.ascontiguousarray(dprims, dtype=np.int32)
            d.dvertices = dv.ctypes.data_as(C.POINTER(C.c_float))
            d.dprims = dix.ctypes.data_as(C.POINTER(C.c_int32))
            d.n_dvertices, d.n_dprims = dv.shape[0], dix.shape[0]
            keep += [dv, dix]
        d.dirichlet_value = float(dirichlet_value)
        if dirichlet_image is not None:
            if dirichlet_image_box is None or len(dirichlet_image_box) != 4:
                raise WosError("dirichlet_image needs dirichlet_image_box = (x0, y0, ex, ey)")
            if _is_torch(dirichlet_image) and dirichlet_image.is_cuda:
                dimg = dirichlet_image.detach().to(dtype=__import__("torch").float32).contiguous()
                d.dirichlet_image, d.dirichlet_image_on_device = dimg.data_ptr(), 1
            else:
                if _is_torch(dirichlet_image):
                    dirichlet_image = dirichlet_image.detach().cpu().numpy()
                dimg = np.ascontiguousarray(dirichlet_image, dtype=np.float32)
                d.dirichlet_image = dimg.ctypes.data
            if len(dimg.shape) != 2:
                raise WosError(f"dirichlet_image must be 2-D, got shape {tuple(dimg.shape)}")
            d.dirichlet_image_dims[0], d.dirichlet_image_dims[1] = int(dimg.shape[0]), int(dimg.shape[1])
            for k in range(4):
                d.dirichlet_image_box[k] = float(dirichlet_image_box[k])
            keep.append(dimg)
        if neumann_image is not None:
            nimg, on_dev = self._image(neumann_image, neumann_image_box, "neumann_image")
            d.neumann_image, d.neumann_image_on_device = (nimg.data_ptr() if on_dev else nimg.ctypes.data), on_dev
            d.neumann_image_dims[0], d.neumann_image_dims[1] = int(nimg.shape[0]), int(nimg.shape[1])
            for k in range(4):
                d.neumann_image_box[k] = float(neumann_image_box[k])
            keep.append(nimg)
        d.absorption = float(absorption)
        d.is_watertight = int(bool(watertight))
        d.is_double_sided = int(bool(double_sided))
        self.source_shape = None
        if source is not None:
            if _is_torch(source) and source.is_cuda:
                src = source.detach().to(dtype=__import__("torch").float32).contiguous()
                d.source = src.data_ptr()
                d.source_on_device = 1
                keep.append(src)
                shape = tuple(src.shape)
            else:
                if _is_torch(source):
                    source = source.detach().cpu().numpy()
                src = np.ascontiguousarray(source, dtype=np.float32)
                d.source = src.ctypes.data
                keep.append(src)
                shape = src.shape
            if len(shape) != self.dim:
                raise WosError(f"source grid must be {self.dim}-D, got shape {shape}")
            for k in range(3):
                d.source_dims[k] = shape[k] if k < len(shape) else 0
            self.source_shape = tuple(int(s) for s in shape)
        self.device = int(device)
        h = C.c_void_p()
        check(L.wos_scene_create(C.byref(d), self.device, C.byref(h)), "wos_scene_create")
        self._h = h
        del keep

    @staticmethod
    def _image(img, box, name):
        """A 2-D float32 image for the C ABI: (contiguous array or CUDA tensor, on_device)."""
        if box is None or len(box) != 4:
            raise WosError(f"{name} needs {name}_box = (x0, y0, ex, ey)")
        if _is_torch(img) and img.is_cuda:
            out, on_dev = img.detach().to(dtype=__import__("torch").float32).contiguous(), 1
        else:
            if _is_torch(img):
                img = img.detach().cpu().numpy()
            out, on_dev = np.ascontiguousarray(img, dtype=np.float32), 0
        if len(out.shape) != 2:
            raise WosError(f"{name} must be 2-D, got shape {tuple(out.shape)}")
        return out, on_dev

    def set_source(self, source, stream=None):
        """Replace the source grid (-div u) in place: the geometry stays resident.
        `source` is a numpy array or a torch tensor (a CUDA tensor is copied
        device-to-device on torch's current stream, no host round trip).  Replaces
        the reference's per-step Scene(sceneConfig, div) (model_split.py:191)."""
        L = _lib.load()
        dims = (C.c_int32 * 3)(0, 0, 0)
        if _is_torch(source) and source.is_cuda:
            import torch
            src = source.detach().to(dtype=torch.float32).contiguous()
            shape = tuple(src.shape)
            ptr, on_dev = src.data_ptr(), 1
            if stream is None:
                stream = torch.cuda.current_stream(src.device).cuda_stream
        else:
            if _is_torch(source):
                source = source.detach().cpu().numpy()
            src = np.ascontiguousarray(source, dtype=np.float32)
            shape = src.shape
            ptr, on_dev = src.ctypes.data, 0
        if len(shape) != self.dim:
            raise WosError(f"source grid must be {self.dim}-D, got shape {shape}")
        for k in range(len(shape)):
            dims[k] = int(shape[k])
        check(L.wos_scene_set_source(self._h, ptr, dims, on_dev, stream), "wos_scene_set_source")
        # the copy is ordered on `stream`: keep the buffer alive until the next replacement
        self._src_keep = src
        self.source_shape = tuple(int(x) for x in shape)

    @classmethod
    def from_obj(cls, path, dim, source=None, absorption=0.0, flip_orientation=False, normalize=False, **kw):
        v, ix = load_obj(path, dim, flip_orientation, normalize)
        return cls(v, ix, source, absorption, **kw)

    def info(self):
        i = SceneInfo()
        check(_lib.load().wos_scene_get_info(self._h, C.byref(i)), "wos_scene_get_info")
        return {"dim": i.dim, "n_prims": i.n_prims, "n_silhouettes": i.n_silhouettes,
                "n_dprims": i.n_dprims, "device": i.device,
                "bbox_min": list(i.bbox_min)[:i.dim], "bbox_max": list(i.bbox_max)[:i.dim]}

    def solve(self, pts, params=None, *, index_base=0, index_stride=1, counts=False, stream=None,
              sync=True):
        """Solve at query points.  Returns (p [N], grad [N,dim], stats dict[, n_est, steps])
        as numpy arrays for host input, torch tensors for GPU tensor input.  With GPU tensors
        and sync=False the solve is only enqueued on the stream: the stats dict then holds
        just "ticket"; solve_stats(ticket) waits for that solve and returns the full dict.
        `stream`: a torch.cuda.Stream or a raw hipStream_t handle (default: torch's current
        stream)."""
        L = _lib.load()
        params = params if params is not None else solver_params()
        st = Stats()
        if _is_torch(pts) and pts.is_cuda:
            import torch
            x = pts.detach().to(torch.float32).contiguous()
            n = x.shape[0]
            if x.ndim != 2 or x.shape[1] != self.dim:
                raise WosError(f"points must be [N,{self.dim}]")
            p = torch.empty(n, dtype=torch.float32, device=x.device)
            g = torch.empty(n, self.dim, dtype=torch.float32, device=x.device)
            ne = torch.empty(n, dtype=torch.int32, device=x.device) if counts else None
            sp = torch.empty(n, dtype=torch.int32, device=x.device) if counts else None
            cur = torch.cuda.current_stream(x.device)
            ts = None
            if stream is None:
                s = cur.cuda_stream
            else:
                ts = stream if isinstance(stream, torch.cuda.Stream) else torch.cuda.ExternalStream(int(stream),
                                                                                                    device=x.device)
                s = ts.cuda_stream
                # the points and the fresh output buffers belong to torch's current stream:
                # the solve on `stream` starts after the work queued there (the kernel that
                # produced x, the allocator's last user of p / g)
                ts.wait_stream(cur)
            flags = _lib.WOS_PTRS_DEVICE | (0 if sync else _lib.WOS_ASYNC)
            check(L.wos_solve(self._h, C.byref(params), x.data_ptr(), n, index_base, index_stride,
                              p.data_ptr(), g.data_ptr(), ne.data_ptr() if counts else None,
                              sp.data_ptr() if counts else None, C.byref(st), s, flags), "wos_solve")
            if not sync and ts is not None:
                # the buffers were allocated on torch's current stream but the enqueued
                # solve uses them on `stream`: keep the caching allocator from handing
                # their memory out again before that stream has finished with them
                for t in (x, p, g, ne, sp):
                    if t is not None:
                        t.record_stream(ts)
        else:
            if _is_torch(pts):
                pts = pts.detach().cpu().numpy()
            x = np.ascontiguousarray(pts, dtype=np.float32)
            if x.ndim != 2 or x.shape[1] != self.dim:
                raise WosError(f"points must be [N,{self.dim}]")
            n = x.shape[0]
            p = np.empty(n, np.float32)
            g = np.empty((n, self.dim), np.float32)
            ne = np.empty(n, np.int32) if counts else None
            sp = np.empty(n, np.int32) if counts else None
            check(L.wos_solve(self._h, C.byref(params), x.ctypes.data, n, index_base, index_stride,
                              p.ctypes.data, g.ctypes.data, ne.ctypes.data if counts else None,
                              sp.ctypes.data if counts else None, C.byref(st), stream, 0), "wos_solve")
        out = (p, g, st.as_dict())
        if counts:
            out = out + (ne, sp)
        return out

    def bvc(self, params=None, bvc=None, samples=True):
        """Boundary value caching (wos_bvc; the reference's bvc, demo.cpp:265-363) on this
        2D scene (Neumann and Dirichlet boundaries).  Returns (solution [g, g], grad [g, g, 2],
        info) on the evaluation grid (index [i, j] = point (i/g, j/g) of the grid box, masked as
        saveEvaluationGrid masks); info holds the sample counts, the cached samples
        ([k, 8]: x y nx ny pdf value normalDerivative kind, include/wos.h) and the stats."""
        L = _lib.load()
        params = params if params is not None else solver_params()
        if bvc is None:
            raise WosError("bvc parameters required (engine.bvc_params(solver, output))")
        g = int(bvc.grid_res)
        sol = np.empty(g * g, np.float32)
        grad = np.empty(g * g * 2, np.float32)
        counts = np.zeros(4, np.int64)
        st = Stats()
        cap = 0
        buf = None
        if samples:
            cap = 2 * int(bvc.boundary_cache_size) + 4 * int(bvc.domain_cache_size) + 16
            buf = np.empty(cap * 8, np.float32)
        rc = L.wos_bvc(self._h, C.byref(params), C.byref(bvc), sol.ctypes.data, grad.ctypes.data,
                       buf.ctypes.data if samples else None, cap, counts.ctypes.data, C.byref(st))
        if rc == _lib.WOS_E_CAPACITY and samples and int(counts[3]) > cap:
            # the domain sampler keeps more candidates than the first guess (non-watertight
            # scenes, small |signedVolume|): wos_bvc failed before the walks with the exact
            # count in counts[3] -- retry once with a buffer of that size
            cap = int(counts[3])
            buf = np.empty(cap * 8, np.float32)
            rc = L.wos_bvc(self._h, C.byref(params), C.byref(bvc), sol.ctypes.data, grad.ctypes.data,
                           buf.ctypes.data, cap, counts.ctypes.data, C.byref(st))
        check(rc, "wos_bvc")
        info = {"counts": {"boundary": int(counts[0]), "boundary_aligned": int(counts[1]), "domain": int(counts[2]),
                           "total": int(counts[3])}, "stats": st.as_dict()}
        if samples:
            info["samples"] = buf[:int(counts[3]) * 8].reshape(-1, 8).copy()
        return sol.reshape(g, g), grad.reshape(g, g, 2), info

    def solve_stats(self, ticket):
        """Statistics of an enqueued solve (wos_solve_stats); blocks until it has finished."""
        st = Stats()
        check(_lib.load().wos_solve_stats(self._h, int(ticket), C.byref(st)), "wos_solve_stats")
        return st.as_dict()

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().wos_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def release_caches(device=-1):
    """Free the per-device solve workspace and the cached prepared geometries
    (wos_release_caches); live scenes stay valid."""
    check(_lib.load().wos_release_caches(int(device)), "wos_release_caches")


def set_max_batch_tasks(n):
    """Walk tasks per batch (wos_set_max_batch_tasks; n <= 0: the default 2^28).  Returns the
    previous value.  Results do not depend on it; it bounds the per-device workspace."""
    return int(_lib.load().wos_set_max_batch_tasks(int(n)))


def selftest_math(which, x, device=0):
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    check(_lib.load().wos_selftest_math(which, x.ctypes.data, out.ctypes.data, x.size, device),
          "wos_selftest_math")
    return out


def device_count():
    return int(_lib.load().wos_device_count())
