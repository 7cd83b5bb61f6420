"""C-ABI boundary tests that need no GPU: the library loads, exports exactly what
include/wos.h declares, parses OBJ files like the reference, reports errors as
status codes instead of aborting (the reference abort()s: config.h:8-11)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import objparse
import wos_amd
from wos_amd import _lib, workloads

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "wos.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(wos_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_expected_api():
    assert declared_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = wos_amd.load_library()
    for name in declared_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (wos_[a-z0-9_]+)$", out, flags=re.M))
    assert set(declared_functions()) <= exported


def test_abi_version():
    assert wos_amd.load_library().wos_abi_version() == wos_amd._lib.ABI_VERSION == 10


@pytest.mark.parametrize("path,dim", [(workloads.KARMAN_OBJ, 2), (workloads.SQUARE_OBJ, 2), (workloads.CUBE_OBJ, 3)])
def test_obj_parse_matches_reference_rules(path, dim):
    v, ix = wos_amd.load_obj(path, dim)
    v2, ix2 = objparse.load(path, dim)
    np.testing.assert_array_equal(v, v2)
    np.testing.assert_array_equal(ix, ix2)


def test_obj_flip_and_normalize():
    v, ix = wos_amd.load_obj(workloads.KARMAN_OBJ, 2, flip_orientation=True)
    v2, ix2 = objparse.load(workloads.KARMAN_OBJ, 2, flip=True)
    np.testing.assert_array_equal(ix, ix2)
    vn, _ = wos_amd.load_obj(workloads.KARMAN_OBJ, 2, normalize=True)
    c = v.astype(np.float64).mean(0)
    r = np.linalg.norm(v - c, axis=1).max()
    np.testing.assert_allclose(vn, (v - c) / r, atol=2e-6)


def test_missing_file_is_an_error_not_an_abort():
    with pytest.raises(wos_amd.WosError, match="Error opening file"):
        wos_amd.load_obj("/nonexistent/x.obj", 2)


def test_bad_dim_rejected():
    L = wos_amd.load_library()
    m = _lib.Mesh()
    assert L.wos_load_obj(workloads.KARMAN_OBJ.encode(), 4, 0, 0, C.byref(m)) == -1
    assert b"dim" in L.wos_last_error()


def test_default_params_match_reference_defaults():
    p = wos_amd.solver_params({}, {})
    # demo.cpp:121-137 defaults
    assert (p.n_walks, p.max_walk_length, p.steps_before_tikhonov, p.steps_before_maximal_spheres) == (128, 1024, 1024, 1024)
    assert abs(p.epsilon_shell - 1e-3) < 1e-9 and abs(p.min_star_radius - 1e-3) < 1e-9
    assert p.russian_roulette_threshold == 0.0 and p.boundary_distance_mask == 0.0
    # the misspelled keys are the ones read (demo.cpp:130-131)
    q = wos_amd.solver_params({"setpsBeforeApplyingTikhonov": 0, "maxWalkLength": 10000,
                               "minStarShapedRadius": 0.5}, {"boundaryDistanceMask": 1e-3})
    assert q.steps_before_tikhonov == 0 and q.steps_before_maximal_spheres == 10000
    assert abs(q.min_star_radius - 1e-3) < 1e-9   # "minStarShapedRadius" is never read


def test_scene_create_without_gpu_reports_device_error():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    v, ix = objparse.load(workloads.KARMAN_OBJ, 2)
    with pytest.raises(wos_amd.WosError, match="no HIP device"):
        wos_amd.WosScene(v, ix, np.zeros((4, 4), np.float32), 350.0)


def test_schedule_bits_match_header():
    # wos_solver_params.schedule bits: include/wos.h WOS_SCHED_* == wos_amd._lib SCHED_*
    txt = open(HEADER).read()
    bits = {m.group(1): int(m.group(2), 16) for m in re.finditer(r"#define WOS_(SCHED_\w+)\s+0x([0-9a-fA-F]+)u", txt)}
    assert set(bits) == {"SCHED_GEOM_GLOBAL", "SCHED_FULL_NEUMANN", "SCHED_NO_STAR_GRID", "SCHED_NO_DIR_GRID",
                         "SCHED_NO_TAIL_SPREAD", "SCHED_NO_GRID_SPREAD"}
    for name, v in bits.items():
        assert getattr(_lib, name) == v, name
    assert len(set(bits.values())) == len(bits) and all(v & (v - 1) == 0 for v in bits.values())


def test_max_batch_tasks_setting():
    """wos_set_max_batch_tasks (ABI 10): returns the previous value, clamps to [2^16, 2^30],
    <= 0 restores the default 2^28 -- a host-side setting, no GPU needed."""
    L = wos_amd.load_library()
    first = L.wos_set_max_batch_tasks(0)
    assert L.wos_set_max_batch_tasks(1000) == 1 << 28
    assert L.wos_set_max_batch_tasks(1 << 40) == 1 << 16
    assert L.wos_set_max_batch_tasks(-1) == 1 << 30
    assert wos_amd.set_max_batch_tasks(first) == 1 << 28
