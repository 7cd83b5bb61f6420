"""The zombie_bindings drop-in shim: same call signature and return structure as
the reference's pybind11 module (demo.cpp:393-401), used the way
src/2d/models/model_split.py:185-202 uses it."""
import json
import os

import numpy as np
import pytest

import zombie_bindings
from wos_amd import workloads


def _configs():
    # examples/karman/wost.json with the boundary path pointed at the repo copy
    scene = dict(workloads.SCENE_BASE, boundary=workloads.KARMAN_OBJ)
    solver = dict(workloads.SOLVER_BASE, nWalks=64)
    output = dict(workloads.OUTPUT_BASE, solutionFile="./solutions/wost.png", txtdir="./solutions/")
    return scene, solver, output


def test_api_surface():
    assert callable(zombie_bindings.wost)
    assert callable(zombie_bindings.bvc)
    assert isinstance(zombie_bindings.Scene, type)


def test_missing_required_keys_raise():
    scene, solver, output = _configs()
    with pytest.raises(KeyError, match="boundary"):
        zombie_bindings.Scene({}, [[0.0]])
    with pytest.raises(KeyError, match="gridRes"):
        zombie_bindings.wost(None, solver, {}, np.zeros((1, 2), np.float32))


def test_bvc_requires_grid_res():
    """bvc reads output.gridRes as required (demo.cpp:281 getRequired)."""
    with pytest.raises(KeyError, match="gridRes"):
        zombie_bindings.bvc(None, {}, {})


def test_solution_image_writers(tmp_path):
    """saveEvaluationGrid's Image<3>::write: PFM 'PF' rows bottom-to-top, PNG 8-bit RGB."""
    import zlib
    img = (np.arange(12, dtype=np.float32).reshape(3, 4) / 12.0)
    pfm = tmp_path / "a" / "s.pfm"
    zombie_bindings._write_image(str(pfm), img)
    raw = pfm.read_bytes()
    assert raw.startswith(b"PF\n4 3\n-1\n")
    body = np.frombuffer(raw[len(b"PF\n4 3\n-1\n"):], "<f4").reshape(3, 4, 3)
    np.testing.assert_array_equal(body[::-1, :, 1], img)
    png = tmp_path / "s.png"
    zombie_bindings._write_image(str(png), img)
    data = png.read_bytes()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    idat = data[data.index(b"IDAT") + 4:data.index(b"IEND") - 8]
    rows = zlib.decompress(idat)
    px = np.frombuffer(rows, np.uint8).reshape(3, 1 + 4 * 3)[:, 1:].reshape(3, 4, 3)
    np.testing.assert_array_equal(px[..., 0], np.clip((img * 255).astype(int), 0, 255))


def test_pfm_reader_file_row_order(tmp_path):
    """readPFM keeps the file's row order (image.h:136-147): row 0 of the grid the
    engine gets is the first row stored in the file -- no bottom-to-top flip."""
    img = np.arange(12, dtype=np.float32).reshape(3, 4)
    path = tmp_path / "x.pfm"
    with open(path, "wb") as f:
        f.write(b"Pf\n4 3\n-1.0\n")
        f.write(img.astype("<f4").tobytes())
    np.testing.assert_array_equal(zombie_bindings._read_pfm(str(path)), img)


def _scene_dict_pair(tmp_path, fmt):
    """Scene(dict) on a source image file and Scene(dict, mat) on the grid the reference
    decodes from it, with the same explicit scene flags (the two ctors' defaults differ,
    scene.h:23,33 vs :55,62)."""
    from test_image_reader import quadrant_image
    img = quadrant_image(80, 200)
    if fmt == "pfm":
        path = tmp_path / "src.pfm"
        with open(path, "wb") as f:
            f.write(b"Pf\n200 80\n-1\n" + img.astype("<f4").tobytes())
    else:
        PIL = pytest.importorskip("PIL.Image")
        path = tmp_path / "src.png"
        PIL.fromarray(((img + 2.5) * 50.0).astype(np.uint8), "L").save(path)  # 175 225 75 25
    from zombie_bindings import _image
    grid = _image.read_image(str(path))
    scene_cfg = dict(workloads.SCENE_BASE, boundary=workloads.KARMAN_OBJ, sourceValue=str(path))
    return zombie_bindings.Scene(scene_cfg), zombie_bindings.Scene(scene_cfg, grid.tolist()), grid


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["pfm", "png"])
def test_scene_dict_image_equals_matrix_scene(gpu, tmp_path, fmt):
    """A Scene(dict) solve (source read from a PFM / PNG file) equals the Scene(dict, mat)
    solve on the same decoded grid bit for bit, and the pressure follows the FILE's
    quadrants: with lambda = 350 the screened solution is ~ f / lambda away from the
    quadrant edges, so p * 350 has the sign of the file's quadrant value."""
    s_img, s_mat, grid = _scene_dict_pair(tmp_path, fmt)
    _, solver, output = _configs()
    bb = s_img.bbox
    lo, hi = np.array(bb["bbox_min"], np.float32), np.array(bb["bbox_max"], np.float32)
    ext = hi - lo
    # one point per quadrant, away from the midlines, the walls and the cylinder (x ~ 0)
    fr = np.array([[0.62, 0.2], [0.92, 0.2], [0.62, 0.8], [0.92, 0.8]], np.float32)
    pts = (lo + fr * ext).astype(np.float32)
    _, p1, g1 = zombie_bindings.wost(s_img, solver, output, pts, return_numpy=True)
    _, p2, g2 = zombie_bindings.wost(s_mat, solver, output, pts, return_numpy=True)
    np.testing.assert_array_equal(p1, p2)
    np.testing.assert_array_equal(g1, g2)
    h, w = grid.shape
    for k in range(4):
        i = min(int(np.float32(fr[k, 1]) * h), h - 1)
        j = min(int(np.float32(fr[k, 0]) * w), w - 1)
        f = grid[i, j]
        assert f != 0
        assert abs(p1[k] * 350.0 - f) < 0.25 * abs(f), (k, p1[k] * 350.0, f)


@pytest.mark.gpu
def test_scene_neumann_image_key(gpu, tmp_path):
    """Scene key "neumannBoundaryValue" (the upstream demo's Neumann image, scene.h:29): read
    like the source image, laid over the scene's padded bounding box (pde.neumann's uv,
    scene.h:175-181); equals WosScene with the same image and box bit for bit, and differs
    from h = 0."""
    from wos_amd import WosScene, solver_params
    scene_cfg, solver, output = _configs()
    cfg = workloads.karman_config(n_walks=32)
    img = (np.linspace(-1.0, 1.0, 24 * 40, dtype=np.float32).reshape(24, 40)) ** 3
    path = tmp_path / "h.pfm"
    with open(path, "wb") as f:
        f.write(b"Pf\n40 24\n-1\n" + img.astype("<f4").tobytes())
    sc = zombie_bindings.Scene(dict(scene_cfg, neumannBoundaryValue=str(path)), cfg["source"])
    bb = sc.bbox
    lo, hi = np.array(bb["bbox_min"], np.float32), np.array(bb["bbox_max"], np.float32)
    pts = cfg["points"][:256]
    _, p1, g1 = zombie_bindings.wost(sc, solver, output, pts, return_numpy=True)
    v, ix = zombie_bindings._load_boundary(scene_cfg["boundary"], 2, bool(scene_cfg.get("flipOrientation", False)),
                                           bool(scene_cfg.get("normalizeDomain", False)))
    ws = WosScene(v, ix, cfg["source"], float(scene_cfg["absorptionCoeff"]), watertight=sc.is_watertight,
                  neumann_image=img, neumann_image_box=(lo[0], lo[1], (hi - lo)[0], (hi - lo)[1]))
    p2, g2, _ = ws.solve(pts, solver_params(solver, output))
    ws.close()
    np.testing.assert_array_equal(p1, p2)
    np.testing.assert_array_equal(g1, g2)
    _, p0, _ = zombie_bindings.wost(zombie_bindings.Scene(scene_cfg, cfg["source"]), solver, output, pts,
                                    return_numpy=True)
    assert np.abs(p1 - p0).max() > 0


@pytest.mark.gpu
def test_wost_end_to_end_like_model_split(gpu):
    """model_split.py:185-202: Scene(sceneConfig, div) then wost(...) -> (samples, p, grad)."""
    scene_cfg, solver, output = _configs()
    cfg = workloads.karman_config(n_walks=64)
    div = cfg["source"].tolist()                   # nested lists, like div from .numpy() -> pybind
    pts = cfg["points"][:1000]
    scene = zombie_bindings.Scene(scene_cfg, div)
    samples, p_arr, grad_arr = zombie_bindings.wost(scene, solver, output, pts)
    samples, p, grad = np.array(samples), np.array(p_arr), np.array(grad_arr)
    assert samples.shape == (1000, 2) and p.shape == (1000,) and grad.shape == (1000, 2)
    np.testing.assert_array_equal(samples, pts)
    # same answer as the engine API with the same seed
    from wos_amd import WosScene, solver_params
    sc = WosScene.from_obj(workloads.KARMAN_OBJ, 2, cfg["source"], 350.0, watertight=True)
    p2, g2, _ = sc.solve(pts, solver_params(solver, output))
    np.testing.assert_array_equal(p.astype(np.float32), p2)
    np.testing.assert_array_equal(grad.astype(np.float32), g2)
    assert scene.last_stats["walks_recorded"] > 0


@pytest.mark.gpu
def test_wost_torch_device_points(gpu):
    import torch
    scene_cfg, solver, output = _configs()
    cfg = workloads.karman_config(n_walks=32)
    scene = zombie_bindings.Scene(scene_cfg, torch.from_numpy(cfg["source"]).cuda())
    pts = torch.from_numpy(cfg["points"][:500]).cuda()
    s, p, g = zombie_bindings.wost(scene, solver, output, pts)
    assert p.is_cuda and g.shape == (500, 2)
    _, p2, g2 = zombie_bindings.wost(scene, solver, output, pts.cpu().numpy(), return_numpy=True)
    np.testing.assert_array_equal(p.cpu().numpy(), p2)
    np.testing.assert_array_equal(g.cpu().numpy(), g2)


def test_obj_cache_follows_real_path_and_inode(tmp_path, monkeypatch):
    """The parsed-OBJ cache is keyed by the resolved path and the file's inode:
    a relative path after a chdir, or a file replaced by one of the same size, is re-parsed."""
    import zombie_bindings as zb
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir(); b.mkdir()
    tri = "v 0 0\nv 1 0\nv 0 1\nl 1 2\nl 2 3\nl 3 1\n"
    (a / "m.obj").write_text(tri)
    (b / "m.obj").write_text(tri.replace("v 1 0", "v 2 0"))
    zb._obj_cache.clear()
    monkeypatch.chdir(a)
    va, _ = zb._load_boundary("m.obj", 2, False, False)
    monkeypatch.chdir(b)
    vb, _ = zb._load_boundary("m.obj", 2, False, False)
    assert va[1, 0] == 1.0 and vb[1, 0] == 2.0
    # same size, same mtime, new inode (atomic replace): re-parsed
    st = os.stat(b / "m.obj")
    new = tmp_path / "n.obj"
    new.write_text(tri.replace("v 1 0", "v 3 0"))
    os.utime(new, ns=(st.st_atime_ns, st.st_mtime_ns))
    os.replace(new, b / "m.obj")
    vc, _ = zb._load_boundary("m.obj", 2, False, False)
    assert vc[1, 0] == 3.0
    assert zb._load_boundary(str(b / "m.obj"), 2, False, False)[0] is vc  # same file by absolute path: cached


def test_junction_near_misses_are_counted():
    """A Dirichlet vertex a few ulp away from a Neumann vertex (two OBJ exports that do not
    share the corner bit for bit) is reported; exact junctions and distant vertices are not."""
    import zombie_bindings as zb
    v = np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float32)
    dv = np.array([[1, 1], [0.5, 0.5], [np.nextafter(np.float32(0), np.float32(1)), 1], [-0.0, 0]], np.float32)
    assert zb._junction_near_misses(v, dv) == 1  # (denormal, 1) vs (0, 1); (-0, 0) equals (0, 0)
    assert zb._junction_near_misses(v, dv[:2]) == 0
    dv2 = np.array([[np.nextafter(np.float32(1), np.float32(2)), 1]], np.float32)
    assert zb._junction_near_misses(v, dv2) == 1
