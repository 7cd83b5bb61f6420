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


def sharded_projection(solve_local, pts, rank, world, dim, group=None, device=None, force_gather=False):
    """Solve all `pts` ([N, dim], identical on every rank) across `world` ranks.

    solve_local(local_pts, index_base, index_stride) -> (p [n_local], grad [n_local, dim])
    as torch tensors on `device` (any device the process group's backend accepts).
    Returns full (p [N], grad [N, dim]) torch tensors on every rank.

    One code path for every backend: the shard, padded to n_pad rows, goes through ONE
    `all_gather_into_tensor` into a (world * n_pad, 1 + dim) buffer (RCCL over xGMI with
    "nccl", gloo in the CPU tests), and the field is reassembled by a view: global point
    i = j * world + r is row j of rank r's block.  `force_gather` runs the collective even
    at world 1 (exercises the RCCL call on a one-GPU lease).
    """
    import torch
    import torch.distributed as dist

    n = pts.shape[0]
    idx, n_pad = shard(n, rank, world)
    local = pts[rank::world]
    p, g = solve_local(local, rank, world)
    p = torch.as_tensor(p, device=device)
    g = torch.as_tensor(g, device=device).reshape(-1, dim)
    gathered = world > 1 or force_gather
    # gloo has no device collectives: a gloo group (CPU rehearsal of the N-rank path,
    # ranks sharing one GPU) stages the shard through host memory
    staged = gathered and p.device.type != "cpu" and dist.get_backend(group) == "gloo"
    bdev = torch.device("cpu") if staged else p.device
    send = torch.zeros(n_pad, 1 + dim, dtype=torch.float32, device=bdev)
    send[: idx.size, 0] = p.to(bdev)
    send[: idx.size, 1:] = g.to(bdev)
    if gathered:
        buf = torch.empty(world * n_pad, 1 + dim, dtype=torch.float32, device=bdev)
        dist.all_gather_into_tensor(buf, send, group=group)
        if staged:
            buf = buf.to(p.device)
    else:
        buf = send
    # (world, n_pad) blocks -> point order r + world * j; the padded rows (j >= count of
    # rank r) are exactly the indices >= n
    full = buf.view(world, n_pad, 1 + dim).transpose(0, 1).reshape(world * n_pad, 1 + dim)[:n]
    return full[:, 0].contiguous(), full[:, 1:].contiguous()


def make_gather(world, dist, n_local, n_pad, dim, dev, torch):
    """bench.py's per-projection gather, on the same collective as sharded_projection:
    every rank sends its shard padded to n_pad rows into a (world * n_pad, 1 + dim)
    buffer with ONE all_gather_into_tensor.  With the gloo backend (CPU-only rehearsal
    of the N-rank path, tests/test_bench_dist.py) the payload is staged through host
    memory; with nccl (RCCL) it stays in HBM.  None at world 1 (nothing to exchange)."""
    if world == 1:
        return None
    staged = dist.get_backend() == "gloo" and dev.type != "cpu"
    bdev = torch.device("cpu") if staged else dev
    send = torch.zeros(n_pad, 1 + dim, dtype=torch.float32, device=bdev)
    buf = torch.empty(world * n_pad, 1 + dim, dtype=torch.float32, device=bdev)

    def gather(p, g):
        send[:n_local, 0] = p.to(bdev)
        send[:n_local, 1:] = g.to(bdev)
        dist.all_gather_into_tensor(buf, send)

    gather.buf = buf
    return gather
