"""wos_amd -- MI355X-native walk-on-stars pressure-projection engine (host side).

The compute path is the HIP kernel in ../csrc (built into ../lib/libwos_hip.so);
this package only marshals arguments across the C ABI (include/wos.h).
"""
from ._lib import WosError, load as load_library  # noqa: F401
from .engine import WosScene, bvc_params, load_obj, solver_params, selftest_math, device_count, release_caches, set_max_batch_tasks  # noqa: F401

__all__ = ["WosScene", "WosError", "bvc_params", "load_obj", "solver_params", "selftest_math", "device_count", "set_max_batch_tasks",
           "load_library", "release_caches"]
