"""Drop-in replacement for the reference's pybind11 module `zombie_bindings`.

Same names, argument meaning and return structure as
  bindings/zombie/demo/demo.cpp:393-401      (2D: Scene(dict), Scene(dict, mat), wost, bvc)
  bindings/zombie3d/demo/demo.cpp:119-125    (3D: Scene(dict, mat3d), wost)
so src/2d/models/model_split.py:185-228 and src/3d/models/model_split.py:190-230
run unchanged with this directory on sys.path.  The solve runs in the HIP kernel
of ../lib/libwos_hip.so (there is no CPU path).

Differences, all deliberate (DESIGN.md "Boundary"):
  * missing required keys raise KeyError instead of abort() (config.h:8-11);
  * RNG seeds are counter-based (solver key "seed", default 0x5EED0001) instead of
    std::chrono::system_clock, so results are reproducible.
Like the reference, 2D and 3D wost solve at the query points they are given
(createSolutionGrid(..., pts), zombie/demo/grid.h:69-102; createSolutionGrid_3d,
zombie3d/demo/grid.h:105-146 iterates the passed points).
bvc (boundary value caching) runs on the GPU too (2D scenes: Neumann and, through
the optional Dirichlet geometry below, mixed boundaries).
Extensions: numpy / torch inputs are accepted without nested-list conversion, a
torch CUDA tensor of points stays on the GPU; optional scene keys
"dirichletBoundary" (OBJ) + "dirichletValue" add Dirichlet geometry, and
"neumannBoundaryValue" (PFM / PNG, the upstream demo's key, scene.h:29) gives the
Neumann data h as an image over the scene's bounding box (default h = 0, as the
reference's pde.neumann).
"""
import os
import warnings

import numpy as np

from wos_amd import engine as _engine

from . import _image

__all__ = ["Scene", "wost", "bvc"]


def _required(d, key):
    if key not in d:
        raise KeyError(f"Missing required setting: {key}")
    return d[key]


# Parsed boundary meshes by (real path, inode, size, mtime, dim, flip, normalize): the time-stepper builds
# a new Scene(sceneConfig, div) every projection (model_split.py:191) on the same OBJ, whose
# parse would otherwise be repeated each time (the geometry's prepared device records are
# cached by content in the library, wos_capi.hip geom_get)
_obj_cache = {}


def _load_boundary(path, dim, flip, normalize):
    try:
        real = os.path.realpath(path)  # a relative path stays right after a chdir
        st = os.stat(real)
        key = (real, st.st_ino, st.st_size, st.st_mtime_ns, dim, flip, normalize)
    except OSError:
        key = None  # let the parser report the missing file
    hit = _obj_cache.get(key) if key is not None else None
    if hit is None:
        hit = _engine.load_obj(path, dim, flip, normalize)
        for a in hit:
            a.setflags(write=False)  # shared by every Scene of this mesh
        if key is not None:
            if len(_obj_cache) >= 16:
                _obj_cache.pop(next(iter(_obj_cache)))
            _obj_cache[key] = hit
    return hit


def _junction_near_misses(v, dv, rel=1e-6):
    """Dirichlet vertices within rel x (scene extent) of a Neumann vertex but not bit-equal to
    one.  Boundary value caching welds the two parts' normals at junction vertices by exact
    position (as the reference's one-mesh computeNormals shares them); two OBJ files whose shared
    corner differs in the last bits would silently not weld -- this makes such a mesh visible."""
    v = np.asarray(v, np.float32)
    dv = np.asarray(dv, np.float32)
    if v.size == 0 or dv.size == 0:
        return 0
    allv = np.concatenate([v, dv])
    tol = rel * float(np.max(allv.max(0) - allv.min(0)))
    exact = {tuple(p) for p in (v + np.float32(0.0)).tolist()}  # +0 == -0
    n = 0
    for s in range(0, dv.shape[0], 1024):
        blk = dv[s:s + 1024]
        d = np.abs(blk[:, None, :].astype(np.float64) - v[None, :, :]).max(-1).min(1)
        for p, dd in zip((blk + np.float32(0.0)).tolist(), d):
            if dd <= tol and tuple(p) not in exact:
                n += 1
    return n


def _read_pfm(path):
    """readPFM (image.h:105-149): file row order, double-precision grayscale."""
    return _image.read_pfm(path)


class Scene:
    """Scene(config) / Scene(config, sourceValue) as in scene.h:22-77 / scene_3d.h:22-40."""

    def __init__(self, config, source=None, device=None):
        config = dict(config)
        boundary = _required(config, "boundary")
        if source is None:
            # Scene(const json&) reads the source image named by "sourceValue" (scene.h:22-52):
            # Image<1>(file) -- PFM or PNG, rows in the file's order (image.h:84-171)
            src = _image.read_image(_required(config, "sourceValue"))
            watertight_default, flip_default = True, True
        else:
            src = source
            watertight_default, flip_default = False, False
        if not hasattr(src, "shape"):
            src = np.asarray(src, dtype=np.float32)
        dim = len(src.shape)
        if dim not in (2, 3):
            raise ValueError(f"source must be a 2D (H,W) or 3D (X,Y,Z) grid, got shape {tuple(src.shape)}")
        self.dim = dim
        self.is_watertight = bool(config.get("isWatertight", watertight_default))
        self.is_double_sided = bool(config.get("isDoubleSided", False))
        absorption = float(config.get("absorptionCoeff", 0.0))
        if dim == 2:
            flip = bool(config.get("flipOrientation", flip_default))
            normalize = bool(config.get("normalizeDomain", False))
        else:  # scene_3d.h reads flipOrientation/normalizeDomain but never applies them
            flip, normalize = False, False
        v, ix = _load_boundary(boundary, dim, flip, normalize)
        dv = dix = None
        self.junction_near_misses = 0
        if config.get("dirichletBoundary"):
            dv, dix = _load_boundary(config["dirichletBoundary"], dim, flip, normalize)
            self.junction_near_misses = _junction_near_misses(v, dv)
            if self.junction_near_misses:
                warnings.warn(f"{self.junction_near_misses} Dirichlet vertices lie within 1e-6 of the scene extent of "
                              "a Neumann vertex without being equal to it: those junctions are not welded (boundary "
                              "value caching's Dirichlet normals, wos_bvc_host.cpp dirichlet_normals)", stacklevel=2)
        nkw = {}
        if config.get("neumannBoundaryValue"):
            if dim != 2:
                raise ValueError("neumannBoundaryValue is 2D (zombie3d's pde.neumann is 0, scene_3d.h:108-111)")
            # the upstream demo's Neumann image (scene.h:29,40 commented in the fork), read as
            # pde.neumann reads it: uv = (x - bbox.pMin) / bbox.extent() (scene.h:175-181), over
            # the FLT_EPSILON-padded box of the boundary (computeBoundingBox)
            allv = v if dv is None else np.concatenate([v, dv])
            eps = np.float32(np.finfo(np.float32).eps)
            lo = (allv.min(0) - eps).astype(np.float32)
            ext = ((allv.max(0) + eps).astype(np.float32) - lo).astype(np.float32)
            nkw = {"neumann_image": _image.read_image(config["neumannBoundaryValue"]),
                   "neumann_image_box": (float(lo[0]), float(lo[1]), float(ext[0]), float(ext[1]))}
        if device is None:
            device = int(os.environ.get("WOS_DEVICE", os.environ.get("LOCAL_RANK", 0)))
        self._scene = _engine.WosScene(v, ix, src, absorption, dvertices=dv, dprims=dix,
                                       dirichlet_value=float(config.get("dirichletValue", 0.0)),
                                       watertight=self.is_watertight, double_sided=self.is_double_sided,
                                       device=device, **nkw)
        self.bbox = self._scene.info()
        self.last_stats = None

    def set_source(self, source):
        """Extension: replace the source grid of this scene in place (a CUDA tensor
        stays on the device), instead of building a new Scene every step."""
        if not hasattr(source, "shape"):
            source = np.asarray(source, dtype=np.float32)
        self._scene.set_source(source)


def wost(scene, solverConfig, outputConfig, pts, return_numpy=False):
    """runWalkOnStars_sampled (demo.cpp:119-205) / runWalkOnStars_3d: returns
    (points, p, grad) as nested lists (numpy arrays if return_numpy; torch
    tensors when pts is a CUDA tensor)."""
    _required(outputConfig, "gridRes")  # required even by the sampled path (demo.cpp:132)
    params = _engine.solver_params(solverConfig, outputConfig)
    if _engine._is_torch(pts) and pts.is_cuda:
        p, g, stats = scene._scene.solve(pts, params)
        scene.last_stats = stats
        return pts, p, g
    x = np.ascontiguousarray(np.asarray(pts, dtype=np.float32).reshape(-1, scene.dim))
    p, g, stats = scene._scene.solve(x, params)
    scene.last_stats = stats
    if return_numpy:
        return x, p, g
    return x.tolist(), p.tolist(), g.tolist()


def _write_image(path, img):
    """Image<3>::write (image.h:97-103, 173-216) of a gray image replicated over three
    channels: .pfm little-endian 'PF' with the rows written bottom to top, anything else
    PNG (8-bit, clamp(int(v * 255), 0, 255)).  Parent directories are created as
    writeSolution does (grid.h:16-17)."""
    import struct
    import zlib
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    h, w = img.shape
    rgb = np.repeat(np.asarray(img, np.float32)[..., None], 3, axis=2)
    if path.lower().endswith(".pfm"):
        with open(path, "wb") as f:
            f.write(b"PF\n%d %d\n-1\n" % (w, h))
            f.write(np.ascontiguousarray(rgb[::-1], "<f4").tobytes())
        return
    v = np.clip((rgb * 255.0).astype(np.int64), 0, 255).astype(np.uint8)
    raw = b"".join(b"\x00" + v[r].tobytes() for r in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) +
                chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b""))


def bvc(scene, solverConfig, outputConfig, return_arrays=False):
    """runBoundaryValueCaching (demo.cpp:265-363): boundary and domain samples, walk-on-stars
    estimates at the boundary samples, splatted onto the gridRes x gridRes evaluation grid
    (GPU: libwos_hip.so wos_bvc), then saveEvaluationGrid (grid.h:370-414): the masked
    solution is written to output["solutionFile"] (default "solution.pfm").  Returns None
    like the reference; return_arrays=True (extension) returns (solution [g, g] indexed
    [i, j] for grid point (i, j), grad [g, g, 2], info with the cached samples and stats).
    The colormapped and debug images of writeSolution are not written."""
    _required(outputConfig, "gridRes")
    if scene.dim != 2:
        raise ValueError("bvc is 2D (the reference's zombie3d module exports no bvc)")
    params = _engine.solver_params(solverConfig, outputConfig)
    bp = _engine.bvc_params(solverConfig, outputConfig)
    sol, grad, info = scene._scene.bvc(params, bp)
    scene.last_stats = info["stats"]
    # Image<3> solution(gridRes, gridRes), solution->get(j, i) = point (i, j) (grid.h:384-409)
    _write_image(outputConfig.get("solutionFile", "solution.pfm"), sol.T)
    if return_arrays:
        return sol, grad, info
    return None
