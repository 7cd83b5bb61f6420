"""Multi-GPU pressure projection: one process per GPU, query points sharded by
stride, one all-gather of [p, grad] per projection (RCCL over xGMI when the
process group uses the "nccl" backend; gloo on CPU for tests).

The walk-on-stars solve has no cross-point state (walk_on_stars.h:76-105 runs
every point independently), so ranks exchange nothing while solving.  The RNG of
a point is keyed by its GLOBAL index, so the gathered field is bit-identical for
any world size.  Stride sharding (rank r owns points r, r+W, ...) balances the
spatially varying per-point cost (near-wall points take more steps).
"""
import numpy as np


def shard(n, rank, world):
    """Global indices owned by `rank` (stride sharding) and the padded shard length."""
    idx = np.arange(rank, n, world)
    n_pad = (n + world - 1) // world
    return idx, n_pad


def sharded_projection(solve_local, pts, rank, world, dim, group=None, device=None):
    """Solve all `pts` ([N, dim], identical on every rank) across `world` ranks.

    solve_local(local_pts, index_base, index_stride) -> (p [n_local], grad [n_local, dim])
    as torch tensors on `device` (any device the process group's backend accepts).
    Returns full (p [N], grad [N, dim]) torch tensors on every rank.
    """
    import torch
    import torch.distributed as dist

    n = pts.shape[0]
    idx, n_pad = shard(n, rank, world)
    local = pts[rank::world]
    p, g = solve_local(local, rank, world)
    p = torch.as_tensor(p, device=device)
    g = torch.as_tensor(g, device=device).reshape(-1, dim)
    send = torch.zeros(n_pad, 1 + dim, dtype=torch.float32, device=device)
    send[: idx.size, 0] = p
    send[: idx.size, 1:] = g
    if world > 1:
        if dist.get_backend(group) == "nccl":
            buf = torch.empty(world * n_pad, 1 + dim, dtype=torch.float32, device=device)
            dist.all_gather_into_tensor(buf, send, group=group)
            parts = list(buf.view(world, n_pad, 1 + dim))
        else:
            parts = [torch.empty_like(send) for _ in range(world)]
            dist.all_gather(parts, send, group=group)
    else:
        parts = [send]
    full = torch.empty(n, 1 + dim, dtype=torch.float32, device=device)
    for r in range(world):
        cnt = len(range(r, n, world))
        full[r::world] = parts[r][:cnt]
    return full[:, 0].contiguous(), full[:, 1:].contiguous()
