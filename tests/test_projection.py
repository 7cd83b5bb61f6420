"""The device-resident projection step around the engine (wos_amd/projection.py):
the reference's grid sampler, autograd divergence and SIREN on CPU; on the GPU, the
device hand-off (divergence grid by device pointer, grad p consumed on the device)
against the reference's host call pattern, bit for bit."""
import numpy as np
import pytest
import torch

from wos_amd import projection as pj
from wos_amd import workloads


def test_sample_uniform_2d_matches_reference_layout():
    # karman bbox, vis_resolution 1000 (examples/karman/run.sh): res_y = int(1000 * 1.202 / 3.01) = 399
    size = workloads.scene_size(workloads.KARMAN_OBJ)
    g = pj.sample_uniform_2d(1000, size)
    res_x = 1000
    res_y = int(1000 * (size[3] - size[2]) / (size[1] - size[0]))
    assert g.shape == (res_y + 2, res_x + 2, 2)
    # meshgrid 'xy': rows follow y, columns follow x; boundary rows/columns on the bbox
    assert torch.allclose(g[0, :, 1], torch.full((res_x + 2,), float(size[2])))
    assert torch.allclose(g[-1, :, 1], torch.full((res_x + 2,), float(size[3])), atol=1e-5)
    assert torch.allclose(g[:, 0, 0], torch.full((res_y + 2,), float(size[0])))
    assert abs(float(g[0, 1, 0]) - (0.5 / res_x * (size[1] - size[0]) + size[0])) < 1e-6
    # the engine's 2D source grid is that shape: rows ~ y (scene.h:194-198)
    assert tuple(workloads.karman_config(n_walks=2)["source"].shape) == (res_y + 2, res_x + 2)


def test_sample_uniform_3d_shape():
    g = pj.sample_uniform_3d(16, (-1, 1, -1, 1, -1, 1))
    assert g.shape == (18, 18, 18, 3)
    assert float(g[0, 0, 0, 0]) == -1.0 and float(g[-1, 0, 0, 0]) == 1.0
    assert float(g[1, 2, 3, 2]) == pytest.approx(2.5 / 16 * 2 - 1)  # [0, 0.5, 1.5, 2.5, ...] cells


def test_divergence_of_analytic_field():
    x = (torch.rand(500, 2, dtype=torch.float64) * 4 - 2).requires_grad_(True)
    u = torch.stack([torch.sin(x[:, 0]) * x[:, 1], torch.cos(x[:, 1]) + x[:, 0] ** 2], dim=-1)
    d = pj.divergence(u, x)[:, 0]
    ref = torch.cos(x[:, 0]) * x[:, 1] - torch.sin(x[:, 1])
    assert torch.allclose(d, ref.detach(), atol=1e-12)


def test_siren_init_and_shape():
    torch.manual_seed(0)
    net = pj.Siren(2, 2, 2, 128)
    lin = [m for m in net.net if isinstance(m, torch.nn.Linear)]
    assert len(lin) == 4
    assert float(lin[0].weight.abs().max()) <= 1 / 2
    assert float(lin[1].weight.abs().max()) <= np.sqrt(6 / 128) / 30 + 1e-9
    y = net(torch.zeros(7, 2))
    assert y.shape == (7, 2)


@pytest.mark.gpu
def test_device_projection_matches_host_pattern(gpu):
    """divergence of a SIREN on the reference grid -> engine by device pointer ->
    grad p on the device, equal bit for bit to the reference's host pattern
    (div.cpu().numpy() -> Scene(cfg, div) -> wost(lists))."""
    import zombie_bindings
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    cfg = workloads.karman_config(n_walks=32, n_points=4096)
    size = workloads.scene_size(workloads.KARMAN_OBJ)
    u = pj.Siren(2, 2, 2, 128).to(dev)
    samples = torch.from_numpy(cfg["points"]).to(dev)
    scene_cfg = dict(cfg["scene"], boundary=cfg["obj"])
    proj = pj.PressureProjector(scene_cfg, cfg["solver"], cfg["output"], samples)
    div = proj.source_from_velocity(u, 200, size)
    assert div.is_cuda and div.shape == pj.sample_uniform_2d(200, size).shape[:2]
    p, g = proj.solve(div)
    assert p.is_cuda and g.is_cuda and g.shape == samples.shape
    sc = zombie_bindings.Scene(scene_cfg, div.cpu().numpy())
    _, p2, g2 = zombie_bindings.wost(sc, cfg["solver"], cfg["output"], samples.cpu().numpy())
    p2 = np.asarray(p2, np.float32)
    g2 = np.asarray(g2, np.float32)
    assert np.array_equal(p.cpu().numpy().view(np.uint32), p2.view(np.uint32))
    assert np.array_equal(g.cpu().numpy().view(np.uint32), g2.view(np.uint32))
    # oracle leg: the CPU restatement on the same divergence grid and samples, bit for bit
    import objparse
    import oracle_lib
    v, ix = objparse.load(cfg["obj"], 2)
    osc = oracle_lib.OracleScene(v, ix, div.cpu().numpy(), 350.0)
    po, go, _, _, _ = oracle_lib.solve(osc, oracle_lib.make_params(cfg["solver"], cfg["output"]),
                                       samples.cpu().numpy())
    assert np.array_equal(p.cpu().numpy().view(np.uint32), po.view(np.uint32))
    assert np.array_equal(g.cpu().numpy().view(np.uint32), go.view(np.uint32))
    u_prev = pj.Siren(2, 2, 2, 128).to(dev)
    loss = proj.projection_loss(u, u_prev, g, 1024)
    loss.backward()
    assert torch.isfinite(loss) and all(torch.isfinite(q.grad).all() for q in u.parameters())


def test_projection_loss_index_range_matches_reference():
    """2D draws randint(0, N-1) (model_split.py:274: the last sample never drawn),
    3D randint(0, N) (3D model_split.py:297)."""

    class _P(pj.PressureProjector):
        def __init__(self, dim, n):  # no engine needed for the index draw
            self.dim, self.device = dim, torch.device("cpu")
            self.samples = torch.zeros(n, dim)

    ident = lambda x: x[:, :1] * 0  # noqa: E731
    for dim, n, top in ((2, 5, 3), (3, 5, 4)):
        proj = _P(dim, n)
        seen = set()
        gen = torch.Generator().manual_seed(0)
        orig = torch.randint
        try:
            def spy(lo, hi, size, **kw):
                r = orig(lo, hi, size, **kw)
                seen.update(r.tolist())
                return r
            torch.randint = spy
            for _ in range(50):
                proj.projection_loss(ident, ident, torch.zeros(n, dim), 64, generator=gen)
        finally:
            torch.randint = orig
        assert max(seen) == top and min(seen) == 0
