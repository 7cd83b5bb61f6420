"""ctypes binding of the C ABI in include/wos.h (lib/libwos_hip.so).

The product path: every solve goes through libwos_hip.so's HIP kernel.  There is
no CPU fallback -- if the library cannot be loaded the import fails loudly.
"""
import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("WOS_LIB_PATH") or os.path.join(PKG_DIR, "lib", "libwos_hip.so")

ABI_VERSION = 10  # include/wos.h WOS_ABI_VERSION this binding's structs mirror
WOS_OK = 0
WOS_E_CAPACITY = -4
WOS_PTRS_DEVICE = 0x1
WOS_ASYNC = 0x2


class WosError(RuntimeError):
    pass


class Mesh(C.Structure):
    _fields_ = [("dim", C.c_int32), ("n_vertices", C.c_int32), ("n_prims", C.c_int32),
                ("vertices", C.POINTER(C.c_float)), ("prims", C.POINTER(C.c_int32))]


class SceneDesc(C.Structure):
    _fields_ = [
        ("dim", C.c_int32),
        ("vertices", C.POINTER(C.c_float)), ("prims", C.POINTER(C.c_int32)),
        ("n_vertices", C.c_int32), ("n_prims", C.c_int32),
        ("dvertices", C.POINTER(C.c_float)), ("dprims", C.POINTER(C.c_int32)),
        ("n_dvertices", C.c_int32), ("n_dprims", C.c_int32),
        ("dirichlet_value", C.c_float), ("absorption", C.c_float),
        ("is_watertight", C.c_int32), ("is_double_sided", C.c_int32),
        ("source", C.c_void_p), ("source_dims", C.c_int32 * 3), ("source_on_device", C.c_int32),
        ("dirichlet_image", C.c_void_p), ("dirichlet_image_dims", C.c_int32 * 2),
        ("dirichlet_image_box", C.c_float * 4), ("dirichlet_image_on_device", C.c_int32),
        ("neumann_image", C.c_void_p), ("neumann_image_dims", C.c_int32 * 2),
        ("neumann_image_box", C.c_float * 4), ("neumann_image_on_device", C.c_int32),
    ]


class SceneInfo(C.Structure):
    _fields_ = [("dim", C.c_int32), ("n_prims", C.c_int32), ("n_silhouettes", C.c_int32),
                ("n_dprims", C.c_int32), ("device", C.c_int32),
                ("bbox_min", C.c_float * 3), ("bbox_max", C.c_float * 3)]


class SolverParams(C.Structure):
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
        ("seed", C.c_uint64),
        ("robust_float", C.c_int32),
        ("schedule", C.c_uint32),
    ]


# wos_solver_params.schedule bits (include/wos.h): scheduling only, results bit-identical
SCHED_GEOM_GLOBAL = 0x1
SCHED_FULL_NEUMANN = 0x2
SCHED_NO_STAR_GRID = 0x4
SCHED_NO_DIR_GRID = 0x8
SCHED_NO_TAIL_SPREAD = 0x10
SCHED_NO_GRID_SPREAD = 0x20  # reserved: no effect (include/wos.h)


class BvcParams(C.Structure):
    _fields_ = [("n_walks_solution", C.c_int32), ("n_walks_gradient", C.c_int32),
                ("boundary_cache_size", C.c_int32), ("domain_cache_size", C.c_int32),
                ("grid_res", C.c_int32), ("use_finite_differences", C.c_int32),
                ("normal_offset", C.c_float), ("radius_clamp", C.c_float),
                ("kernel_regularization", C.c_float), ("grid_box", C.c_float * 4)]


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "walk_steps", "wasted_steps", "walks_recorded", "walks_escaped", "walks_max_length",
        "walks_rr", "walks_dirichlet", "points_estimated", "rejection_iters")] + [
        (n, C.c_double) for n in ("kernel_ms", "first_ball_ms", "walk_ms", "fold_ms")] + [("walk_launches", C.c_uint64)] + [
        (n, C.c_int32) for n in ("first_ball_blocks_per_cu", "walk_blocks_per_cu", "walk_lds_bytes", "star_grid",
                                 "geom_global", "dir_grid")] + [("ticket", C.c_uint64)]

    def as_dict(self):
        return {n: (float(getattr(self, n)) if t is C.c_double else int(getattr(self, n))) for n, t in self._fields_}


# exported symbols, exactly those declared in include/wos.h
EXPORTS = (
    "wos_load_obj", "wos_mesh_free", "wos_scene_create", "wos_scene_destroy",
    "wos_scene_get_info", "wos_scene_set_source", "wos_release_caches", "wos_default_params", "wos_solve",
    "wos_solve_stats", "wos_default_bvc_params", "wos_bvc",
    "wos_selftest_math", "wos_last_error", "wos_abi_version", "wos_device_count", "wos_set_max_batch_tasks",
)

_lib = None


def load():
    """Load libwos_hip.so (raises if it is missing -- no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise WosError(f"{LIB_PATH} not built: run `make -C {PKG_DIR}` or __graft_entry__.build()")
    L = C.CDLL(LIB_PATH)
    L.wos_load_obj.restype = C.c_int
    L.wos_load_obj.argtypes = [C.c_char_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(Mesh)]
    L.wos_mesh_free.restype = None
    L.wos_mesh_free.argtypes = [C.POINTER(Mesh)]
    L.wos_scene_create.restype = C.c_int
    L.wos_scene_create.argtypes = [C.POINTER(SceneDesc), C.c_int32, C.POINTER(C.c_void_p)]
    L.wos_scene_destroy.restype = C.c_int
    L.wos_scene_destroy.argtypes = [C.c_void_p]
    L.wos_scene_get_info.restype = C.c_int
    L.wos_scene_get_info.argtypes = [C.c_void_p, C.POINTER(SceneInfo)]
    L.wos_scene_set_source.restype = C.c_int
    L.wos_scene_set_source.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int32), C.c_int32, C.c_void_p]
    L.wos_release_caches.restype = C.c_int
    L.wos_release_caches.argtypes = [C.c_int32]
    L.wos_set_max_batch_tasks.restype = C.c_int64
    L.wos_set_max_batch_tasks.argtypes = [C.c_int64]
    L.wos_default_params.restype = None
    L.wos_default_params.argtypes = [C.POINTER(SolverParams)]
    L.wos_solve.restype = C.c_int
    L.wos_solve.argtypes = [C.c_void_p, C.POINTER(SolverParams), C.c_void_p, C.c_int64, C.c_int64,
                            C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                            C.POINTER(Stats), C.c_void_p, C.c_uint32]
    L.wos_solve_stats.restype = C.c_int
    L.wos_solve_stats.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(Stats)]
    L.wos_default_bvc_params.restype = None
    L.wos_default_bvc_params.argtypes = [C.POINTER(BvcParams)]
    L.wos_bvc.restype = C.c_int
    L.wos_bvc.argtypes = [C.c_void_p, C.POINTER(SolverParams), C.POINTER(BvcParams), C.c_void_p, C.c_void_p,
                          C.c_void_p, C.c_int64, C.c_void_p, C.POINTER(Stats)]
    L.wos_selftest_math.restype = C.c_int
    L.wos_selftest_math.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32]
    L.wos_last_error.restype = C.c_char_p
    L.wos_last_error.argtypes = []
    L.wos_abi_version.restype = C.c_int32
    L.wos_device_count.restype = C.c_int32
    if L.wos_abi_version() != ABI_VERSION:
        raise WosError(f"{LIB_PATH}: ABI {L.wos_abi_version()} != binding ABI {ABI_VERSION}; rebuild the library")
    _lib = L
    return L


def check(rc, what=""):
    if rc != WOS_OK:
        msg = load().wos_last_error().decode(errors="replace")
        raise WosError(f"{what} failed ({rc}): {msg}")
