"""BASELINE.json configs A and E at their full size on the HIP path.

Config A (taylorgreen 2D, 32x32 points, 32 walks, maxWalkLength 10000 as
examples/taylorgreen/wost.json ships it): as shipped every point is "outside"
(square.obj winds clockwise; insideDomain, fcpw_scene_loader.h:642-648) and the
reference returns zeros; flipped, the 2D Yukawa members overflow for mu R > 91.9 and
every walk is poisoned with NaN and runs to maxWalkLength (SURVEY.md section 7.2 hard
part 4) -- 73 M wasted steps and 6.5 G rejection iterations at this size.  The whole
config runs on the GPU; the oracle checks a strided quarter of the points bit for bit
(the full set takes ~2 min of CPU), and the GPU checks shard invariance on the rest.

Config E (smoke3d: cube.obj, 256^3 points x 128 walks, source = -div u of the SIREN
velocity net on the reference's 82^3 vis grid): the source comes from
PressureProjector.source_from_velocity with a 5 x 256 SIREN (num_hidden_layers 5,
hidden_features 256; the reference's smoke3d example uses 5 x 64,
examples/smoke3d/run.sh) on sample_uniform_3d(80) (src/3d/models/model_split.py:268,
src/3d/utils/model_utils.py:3-29), handed to the engine by device pointer.  Checks:
determinism, strided-half shard invariance, the oracle on a sparse strided subset at
global indices (bit for bit, on the same divergence grid), and the projection loss
on the device (3D index range, model_split.py:297-313).
"""
import numpy as np
import pytest
import torch

import objparse
from wos_amd import WosScene, solver_params, workloads
from wos_amd import projection as pj

pytestmark = pytest.mark.gpu


def _bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    na, nb = np.isnan(a), np.isnan(b)
    np.testing.assert_array_equal(na, nb)
    np.testing.assert_array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


@pytest.mark.parametrize("flip", [False, True])
def test_config_a_full_size(gpu, oracle, flip):
    cfg = workloads.taylorgreen_config(n_walks=32, res=32, flip=flip)
    assert cfg["solver"]["maxWalkLength"] == 10000 and cfg["points"].shape[0] == 1024
    v, ix = objparse.load(cfg["obj"], 2, flip=flip)
    sc = WosScene(v, ix, cfg["source"], 350.0, watertight=True)
    prm = solver_params(cfg["solver"], cfg["output"])
    pts = cfg["points"]
    p, g, st, ne, sp = sc.solve(pts, prm, counts=True)
    pe, ge, _ = sc.solve(pts[1::2], prm, index_base=1, index_stride=2)
    _bits_equal(pe, p[1::2])
    _bits_equal(ge, g[1::2])
    sc.close()
    osc = oracle.OracleScene(v, ix, cfg["source"], 350.0)
    sub = np.arange(0, 1024, 4)
    po, go, neo, spo, _ = oracle.solve(osc, oracle.make_params(cfg["solver"], cfg["output"]), pts[sub],
                                       index_base=0, index_stride=4)
    np.testing.assert_array_equal(ne[sub], neo)
    np.testing.assert_array_equal(sp[sub], spo)
    _bits_equal(p[sub], po)
    _bits_equal(g[sub], go)
    if flip:
        assert st["walks_max_length"] > 0 and st["wasted_steps"] > 10 * st["walk_steps"]
        assert np.isnan(p).all()
    else:
        assert st["points_estimated"] == 0 and not p.any() and not g.any()


def test_config_e_full_size_siren_source(gpu, oracle):
    dev = torch.device("cuda", 0)
    cfg = workloads.cube_config(res=256, n_walks=128)
    pts = cfg["points"]
    assert pts.shape == (256 ** 3, 3)
    size = workloads.scene_size(workloads.CUBE_OBJ, 3)
    torch.manual_seed(5)
    net = pj.Siren(3, 3, 5, 256).to(dev)
    samples = torch.from_numpy(pts).to(dev)
    proj = pj.PressureProjector(dict(cfg["scene"]), cfg["solver"], cfg["output"], samples)
    div = proj.source_from_velocity(net, 80, size)
    assert div.is_cuda and tuple(div.shape) == (82, 82, 82)
    assert torch.isfinite(div).all()
    p1, g1 = proj.solve(div)
    st = proj.last_stats
    p2, g2 = proj.solve(div)
    assert torch.equal(p1, p2) and torch.equal(g1, g2)
    assert torch.isfinite(p1).all() and torch.isfinite(g1).all()
    # cube.obj's corners are not exactly +-1 (0.999999 / 1.000001): a handful of the
    # 2.1e9 walks slip through the seams and escape, as they would in the reference
    assert st["points_estimated"] > 0.95 * pts.shape[0]
    assert st["walks_escaped"] <= 1e-7 * st["walks_recorded"], st
    # shard invariance: the odd points solved alone at their global indices
    pe, ge, _ = proj.scene._scene.solve(samples[1::2].contiguous(), proj.params, index_base=1, index_stride=2)
    assert torch.equal(pe, p1[1::2]) and torch.equal(ge, g1[1::2])
    # the oracle on the same divergence grid, at global indices
    stride = 262147
    sub = np.arange(0, pts.shape[0], stride)
    v, ix = objparse.load(workloads.CUBE_OBJ, 3)
    osc = oracle.OracleScene(v, ix, div.cpu().numpy(), 350.0)
    po, go, _, _, _ = oracle.solve(osc, oracle.make_params(cfg["solver"], cfg["output"]), pts[sub],
                                   index_base=0, index_stride=stride)
    _bits_equal(p1.cpu().numpy()[sub], po)
    _bits_equal(g1.cpu().numpy()[sub], go)
    # the projection loss consumes grad p on the device
    net_prev = pj.Siren(3, 3, 5, 256).to(dev)
    loss = proj.projection_loss(net, net_prev, g1, 128 ** 2)
    loss.backward()
    assert torch.isfinite(loss) and all(torch.isfinite(q.grad).all() for q in net.parameters())
