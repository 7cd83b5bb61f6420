"""Device-resident pressure projection: the callers on either side of the walk-on-stars
path, kept on the GPU.

The reference's projection step, per time step (src/2d/models/model_split.py:185-283;
3D: src/3d/models/model_split.py:190-316):
  * get_divergence: grid = sample_uniform_2D(vis_resolution, with_boundary=True)
    (src/2d/utils/model_utils.py:3-20), u = query_velocity(grid) (the SIREN,
    src/2d/models/networks.py:14-68), div = divergence(u, grid)
    (src/2d/utils/diff_ops.py:45-51), then -div[..., 0].detach().cpu().numpy();
  * wost_pressure: Scene(sceneConfig, div) + wost(scene, solver, output,
    pressure_samples.detach().cpu().numpy()) -> nested lists -> numpy;
  * _project_velocity: grad_p = torch.Tensor(grad_p).to(device), then on random
    samples target = u_prev - grad_p[idx], loss = mean((u - target)^2).
Here the divergence grid stays a CUDA tensor and reaches the engine by device
pointer (wos_scene_set_source: one device-to-device copy, the geometry stays
resident), the pressure samples stay a CUDA tensor, and grad p comes back as a CUDA
tensor that the loss indexes in place -- no host round trip anywhere.  The SIREN runs
in PyTorch-ROCm: its Linear layers are the dense contractions (hipBLASLt / MFMA).
"""
import numpy as np
import torch
import torch.nn as nn

from . import engine as _engine


class Sine(nn.Module):
    """sin(30 x) (networks.py:15-21)."""

    def forward(self, x):
        return torch.sin(30.0 * x)


class Siren(nn.Module):
    """The reference's MLP with sine nonlinearity (networks.py:25-68) and its
    initialisation (sine_init / first_layer_sine_init, networks.py:78-90)."""

    def __init__(self, in_features, out_features, num_hidden_layers, hidden_features):
        super().__init__()
        layers = [nn.Linear(in_features, hidden_features), Sine()]
        for _ in range(num_hidden_layers):
            layers += [nn.Linear(hidden_features, hidden_features), Sine()]
        layers.append(nn.Linear(hidden_features, out_features))
        self.net = nn.Sequential(*layers)
        with torch.no_grad():
            for m in self.net:
                if isinstance(m, nn.Linear):
                    n = m.weight.size(-1)
                    m.weight.uniform_(-np.sqrt(6 / n) / 30, np.sqrt(6 / n) / 30)
            first = self.net[0]
            first.weight.uniform_(-1 / in_features, 1 / in_features)

    def forward(self, coords):
        return self.net(coords)


def sample_uniform_2d(resolution, size, with_boundary=True, device="cpu"):
    """sample_uniform_2D (src/2d/utils/model_utils.py:3-20): cell centres of a grid
    over size = (x0, x1, y0, y1) with `resolution` cells along the longer side, plus
    the boundary rows/columns; meshgrid 'xy' -> shape (res_y [+2], res_x [+2], 2)."""
    if (size[1] - size[0]) > (size[3] - size[2]):
        res_x, res_y = resolution, int(resolution * (size[3] - size[2]) / (size[1] - size[0]))
    else:
        res_x, res_y = int(resolution * (size[1] - size[0]) / (size[3] - size[2])), resolution
    x = torch.linspace(0.5, res_x - 0.5, res_x, device=device)
    y = torch.linspace(0.5, res_y - 0.5, res_y, device=device)
    if with_boundary:
        x = torch.cat([torch.zeros(1, device=device), x, torch.full((1,), float(res_x), device=device)])
        y = torch.cat([torch.zeros(1, device=device), y, torch.full((1,), float(res_y), device=device)])
    coords = torch.stack(torch.meshgrid(x, y, indexing="xy"), dim=-1)
    coords[..., 0] = coords[..., 0] / res_x * (size[1] - size[0]) + size[0]
    coords[..., 1] = coords[..., 1] / res_y * (size[3] - size[2]) + size[2]
    return coords


def sample_uniform_3d(resolution, size, with_boundary=True, device="cpu"):
    """The 3D sampler (src/3d/utils/model_utils.py:3-29, named sample_uniform_2D there):
    `resolution` cells along the shortest side, meshgrid 'ij' -> (X, Y, Z, 3).  The
    reference builds the z axis with res_y points (model_utils.py:17); kept."""
    ex, ey, ez = size[1] - size[0], size[3] - size[2], size[5] - size[4]
    if ex < ey:
        if ex < ez:
            res = (resolution, int(resolution * ey / ex), int(resolution * ez / ex))
        else:
            res = (int(resolution * ex / ez), int(resolution * ey / ez), resolution)
    else:
        if ey < ez:
            res = (int(resolution * ex / ey), resolution, int(resolution * ez / ey))
        else:
            res = (int(resolution * ex / ez), int(resolution * ey / ez), resolution)
    rx, ry, rz = res
    axes = [torch.linspace(0.5, rx - 0.5, rx, device=device), torch.linspace(0.5, ry - 0.5, ry, device=device),
            torch.linspace(0.5, rz - 0.5, ry, device=device)]
    if with_boundary:
        axes = [torch.cat([torch.zeros(1, device=device), a, torch.full((1,), float(r), device=device)])
                for a, r in zip(axes, res)]
    coords = torch.stack(torch.meshgrid(*axes, indexing="ij"), dim=-1)
    for k in range(3):
        coords[..., k] = coords[..., k] / res[k] * (size[2 * k + 1] - size[2 * k]) + size[2 * k]
    return coords


def divergence(y, x, create_graph=False):
    """sum_i d y_i / d x_i by autograd (diff_ops.py:45-51)."""
    div = 0.0
    for i in range(y.shape[-1]):
        g = torch.autograd.grad(y[..., i], x, torch.ones_like(y[..., i]), create_graph=create_graph,
                                retain_graph=True)[0]
        div = div + g[..., i:i + 1]
    return div


class PressureProjector:
    """One scene for the whole simulation; each projection replaces its source in
    place and solves at the (device-resident) pressure samples.

        proj = PressureProjector(wost_json["scene"], wost_json["solver"], wost_json["output"],
                                 pressure_samples_cuda)
        div = proj.source_from_velocity(u_prev, vis_resolution, scene_size)
        p, grad_p = proj.solve(div)
        loss = proj.projection_loss(u, u_prev, grad_p, n)

    Multi-GPU (one process per GPU): pass the process group
    (`group=torch.distributed.group.WORLD` after init_process_group("nccl")).  Every
    rank holds the same pressure samples; rank r solves the stride shard r, r + W, ...
    keyed by GLOBAL sample index, and ONE all_gather_into_tensor of [p, grad p] (RCCL
    over xGMI) hands every rank the full field -- bit-identical to a one-GPU solve, so
    projection_loss draws from it unchanged.  `force_gather` runs the collective even in
    a world of one.
    """

    def __init__(self, scene_config, solver_config, output_config, pressure_samples, device=None,
                 group=None, force_gather=False):
        import zombie_bindings  # the drop-in shim parses the reference's scene keys
        self.dim = int(pressure_samples.shape[-1])
        self.device = pressure_samples.device if device is None else torch.device(device)
        placeholder = torch.zeros((2,) * self.dim, dtype=torch.float32, device=self.device)
        self.scene = zombie_bindings.Scene(dict(scene_config), placeholder, device=self.device.index or 0)
        self.params = _engine.solver_params(solver_config, output_config)
        self.samples = pressure_samples.detach().to(self.device, torch.float32).contiguous()
        self.group, self.force_gather = group, force_gather
        self.last_stats = None

    def source_from_velocity(self, velocity_fn, resolution, size):
        """-div u on the reference's grid (get_divergence, model_split.py:230-236),
        computed and kept on the device."""
        sampler = sample_uniform_2d if self.dim == 2 else sample_uniform_3d
        grid = sampler(resolution, size, with_boundary=True, device=self.device).requires_grad_(True)
        u = velocity_fn(grid)
        div = divergence(u, grid)
        return (-div[..., 0]).detach().contiguous()

    def _set_source(self, div):
        self.scene._scene.set_source(div)

    def _solve_points(self, x, index_base, index_stride):
        return self.scene._scene.solve(x, self.params, index_base=index_base, index_stride=index_stride)

    def solve(self, div):
        """wost_pressure (model_split.py:185-202) with device tensors in and out; with a
        process group, this rank's stride shard + one all-gather (wos_amd.dist)."""
        self._set_source(div)
        if self.group is None and not self.force_gather:
            p, g, st = self._solve_points(self.samples, 0, 1)
            self.last_stats = st
            return p, g
        import torch.distributed as tdist
        from . import dist as _dist
        group = self.group if self.group is not None else tdist.group.WORLD
        rank, world = tdist.get_rank(group), tdist.get_world_size(group)

        def solve_local(local, base, stride):
            p, g, st = self._solve_points(local.contiguous(), base, stride)
            self.last_stats = st  # this rank's shard
            return p, g

        return _dist.sharded_projection(solve_local, self.samples, rank, world, self.dim, group=group,
                                        device=self.device, force_gather=self.force_gather)

    def projection_loss(self, velocity, velocity_prev, grad_p, n_samples, generator=None):
        """_project_velocity (model_split.py:272-283): u <- u_prev - grad p on random
        pressure samples, grad p indexed on the device.  The index range is the
        reference's: the 2D caller draws randint(0, N-1) (src/2d/models/model_split.py:274,
        so the last sample is never drawn), the 3D caller randint(0, N)
        (src/3d/models/model_split.py:297)."""
        n = self.samples.shape[0]
        hi = n - 1 if self.dim == 2 else n
        idx = torch.randint(0, hi, (n_samples,), device=self.device, generator=generator)
        x = self.samples[idx]
        with torch.no_grad():
            target = velocity_prev(x) - grad_p[idx]
        return torch.mean((velocity(x) - target) ** 2)
