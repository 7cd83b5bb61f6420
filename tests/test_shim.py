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


def test_pfm_reader_roundtrip(tmp_path):
    img = np.arange(12, dtype=np.float32).reshape(3, 4)
    path = tmp_path / "x.pfm"
    with open(path, "wb") as f:
        f.write(b"Pf\n4 3\n-1.0\n")
        f.write(img[::-1].astype("<f4").tobytes())
    np.testing.assert_array_equal(zombie_bindings._read_pfm(str(path)), img)


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
