"""One rank of the multi-process sharded projection on the HIP engine (launched as a
fresh child process by tests/test_distributed.py::test_sharded_projection_hip_engine).

    python tests/dist_engine_worker.py RANK WORLD PORT OUT_DIR [BACKEND]

Every rank drives the engine on GPU 0 (a one-GPU box): it solves its stride shard
of the karman points, keyed by global point index, then the shards are gathered
(wos_amd.dist.sharded_projection, the same path bench.py runs over RCCL) and rank r
writes the full field to OUT_DIR/rank<r>.npz.  BACKEND "gloo" (default): gathered on
CPU tensors.  BACKEND "nccl": RCCL on the device tensors; one GPU allows one rank
(RCCL refuses two ranks on one GPU), so it runs at WORLD 1 with the collective forced
(force_gather) -- the product's RCCL all_gather_into_tensor executed on MI355X."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "neural-monte-carlo-fluid-simulation_amd")]


def main():
    rank, world, port, out_dir = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    backend = sys.argv[5] if len(sys.argv) > 5 else "gloo"
    import numpy as np
    import torch
    import torch.distributed as dist
    from wos_amd import WosScene, solver_params, workloads
    from wos_amd import dist as wdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    if backend == "projector":
        return projector(rank, world, dev, out_dir)
    if backend == "nccl":
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = workloads.config_by_name("B")
    pts = cfg["points"][:4099]
    sc = WosScene(cfg["vertices"], cfg["prims"], torch.from_numpy(cfg["source"]).to(dev), 350.0,
                  watertight=True, device=0)
    prm = solver_params(dict(cfg["solver"], nWalks=64), cfg["output"])

    def solve_local(local, base, stride):
        x = torch.from_numpy(np.ascontiguousarray(local)).to(dev)
        p, g, st = sc.solve(x, prm, index_base=base, index_stride=stride)
        assert st["points_estimated"] > 0
        return (p, g) if backend == "nccl" else (p.cpu(), g.cpu())

    if backend == "nccl":
        p, g = wdist.sharded_projection(solve_local, pts, rank, world, 2, device=dev, force_gather=True)
        assert p.is_cuda and g.is_cuda and dist.get_backend() == "nccl"
        print(f"rank {rank}: RCCL all_gather_into_tensor on {torch.cuda.get_device_name(dev)}, "
              f"rccl {'.'.join(map(str, torch.cuda.nccl.version()))}, world {world}", flush=True)
        p, g = p.cpu(), g.cpu()
    else:
        p, g = wdist.sharded_projection(solve_local, pts, rank, world, 2)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), p=p.numpy(), g=g.numpy())
    dist.barrier()
    dist.destroy_process_group()
    sc.close()


def projector(rank, world, dev, out_dir):
    """BACKEND "projector": the caller-facing PressureProjector over an RCCL group
    (world 1 on a one-GPU box, collective forced) against the same projector unsharded."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from wos_amd import projection as pj
    from wos_amd import workloads
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    cfg = workloads.karman_config(n_walks=32, n_points=4096)
    size = workloads.scene_size(workloads.KARMAN_OBJ)
    scene_cfg = dict(cfg["scene"], boundary=cfg["obj"])
    samples = torch.from_numpy(cfg["points"]).to(dev)
    torch.manual_seed(3)
    u = pj.Siren(2, 2, 2, 64).to(dev)
    sharded = pj.PressureProjector(scene_cfg, cfg["solver"], cfg["output"], samples,
                                   group=dist.group.WORLD, force_gather=True)
    div = sharded.source_from_velocity(u, 200, size)
    p, g = sharded.solve(div)
    assert p.is_cuda and g.is_cuda and dist.get_backend() == "nccl"
    plain = pj.PressureProjector(scene_cfg, cfg["solver"], cfg["output"], samples)
    p1, g1 = plain.solve(div)
    print(f"rank {rank}: PressureProjector over RCCL, world {world}, {samples.shape[0]} samples", flush=True)
    np.savez(os.path.join(out_dir, f"proj{rank}.npz"), p=p.cpu().numpy(), g=g.cpu().numpy(),
             p1=p1.cpu().numpy(), g1=g1.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
