"""Multi-process sharded projection (world_size 2, gloo on CPU).

The product's N-GPU path (bench.py / wos_amd.dist) shards query points by stride,
solves each shard on its own GPU keyed by GLOBAL point index, and all-gathers
[p, grad] once per projection.  Here each rank's local solver is the CPU oracle
(test infrastructure), so the test checks the sharding + gather logic: the
gathered field must be bit-identical to a single-process solve.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "neural-monte-carlo-fluid-simulation_amd")]
    import torch
    import torch.distributed as dist
    import objparse
    import oracle_lib
    from wos_amd import dist as wdist
    from wos_amd import workloads
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = workloads.karman_config(n_walks=32)
    pts = cfg["points"][:301]
    v, ix = objparse.load(cfg["obj"], 2)
    sc = oracle_lib.OracleScene(v, ix, cfg["source"], 350.0)
    prm = oracle_lib.make_params(cfg["solver"], cfg["output"], n_threads=2)

    def solve_local(local, base, stride):
        p, g, _, _, _ = oracle_lib.solve(sc, prm, local, index_base=base, index_stride=stride)
        return torch.from_numpy(p), torch.from_numpy(g)

    p, g = wdist.sharded_projection(solve_local, pts, rank, world, 2)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), p=p.numpy(), g=g.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_projection_matches_single_process(tmp_path, oracle, world):
    from wos_amd import workloads
    import objparse
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True, start_method="spawn")
    cfg = workloads.karman_config(n_walks=32)
    pts = cfg["points"][:301]
    v, ix = objparse.load(cfg["obj"], 2)
    sc = oracle.OracleScene(v, ix, cfg["source"], 350.0)
    p0, g0, _, _, _ = oracle.solve(sc, oracle.make_params(cfg["solver"], cfg["output"]), pts)
    for r in range(world):
        d = np.load(tmp_path / f"rank{r}.npz")
        np.testing.assert_array_equal(d["p"], p0)
        np.testing.assert_array_equal(d["g"], g0)


def test_shard_covers_all_points_once():
    from wos_amd.dist import shard
    for n in (0, 1, 7, 64, 65398):
        for w in (1, 2, 3, 8):
            seen = np.concatenate([shard(n, r, w)[0] for r in range(w)])
            assert sorted(seen.tolist()) == list(range(n))
            assert all(shard(n, r, w)[0].size <= shard(n, r, w)[1] for r in range(w))


def _forced_gather_worker(rank, world, port, out_dir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "neural-monte-carlo-fluid-simulation_amd")]
    import torch
    import torch.distributed as dist
    from wos_amd import dist as wdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1001
    pts = torch.arange(2 * n, dtype=torch.float32).reshape(n, 2)

    def solve_local(local, base, stride):  # a point's "solution" is a function of its global index
        gi = torch.arange(base, n, stride, dtype=torch.float32)
        assert gi.shape[0] == local.shape[0]
        return gi * 0.5, torch.stack([gi, -gi], 1)

    p, g = wdist.sharded_projection(solve_local, pts, rank, world, 2, force_gather=True)
    torch.save({"p": p, "g": g}, os.path.join(out_dir, f"fg{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 4])
def test_forced_gather_reassembles_point_order(tmp_path, world):
    """The one all_gather_into_tensor path (every backend, forced at world 1 as the
    RCCL GPU test runs it) puts global point i = r + world * j back at row i."""
    import torch
    port = _free_port()
    mp.start_processes(_forced_gather_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    gi = torch.arange(1001, dtype=torch.float32)
    for r in range(world):
        d = torch.load(tmp_path / f"fg{r}.pt", weights_only=True)
        assert torch.equal(d["p"], gi * 0.5)
        assert torch.equal(d["g"], torch.stack([gi, -gi], 1))


@pytest.mark.gpu
def test_sharded_projection_rccl_world1(tmp_path, gpu, oracle):
    """The product's RCCL gather on MI355X: a world-1 "nccl" (RCCL) process group on
    the lease's one GPU (RCCL refuses two ranks on one GPU), the device-side
    all_gather_into_tensor forced through wos_amd.dist.sharded_projection; the field
    equals an unsharded engine solve and the oracle, bit for bit."""
    import subprocess
    import sys
    from wos_amd import WosScene, solver_params, workloads
    port = _free_port()
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_engine_worker.py")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, worker, "0", "1", str(port), str(tmp_path), "nccl"], env=env,
                       capture_output=True, text=True, timeout=150)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "RCCL all_gather_into_tensor" in r.stdout
    cfg = workloads.config_by_name("B")
    pts = cfg["points"][:4099]
    prm = solver_params(dict(cfg["solver"], nWalks=64), cfg["output"])
    sc = WosScene(cfg["vertices"], cfg["prims"], cfg["source"], 350.0, watertight=True)
    p1, g1, _ = sc.solve(pts, prm)
    sc.close()
    osc = oracle.OracleScene(cfg["vertices"], cfg["prims"], cfg["source"], 350.0)
    po, go, _, _, _ = oracle.solve(osc, oracle.make_params(dict(cfg["solver"], nWalks=64), cfg["output"]),
                                   pts[::41], index_base=0, index_stride=41)
    np.testing.assert_array_equal(p1[::41], po)
    np.testing.assert_array_equal(g1[::41], go)
    d = np.load(tmp_path / "rank0.npz")
    np.testing.assert_array_equal(d["p"], p1)
    np.testing.assert_array_equal(d["g"], g1)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2])
def test_sharded_projection_hip_engine(tmp_path, gpu, oracle, world):
    """World-2 gloo with the HIP ENGINE as each rank's solver: the ranks are fresh
    child processes (tests/dist_engine_worker.py) sharing GPU 0, the gather runs on
    CPU tensors; the gathered field equals a single-process engine solve and the
    oracle, bit for bit."""
    import subprocess
    import sys
    import torch
    from wos_amd import WosScene, solver_params, workloads
    port = _free_port()
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_engine_worker.py")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, worker, str(r), str(world), str(port), str(tmp_path)], env=env)
             for r in range(world)]
    rcs = [p.wait(timeout=100) for p in procs]
    assert rcs == [0] * world, rcs
    cfg = workloads.config_by_name("B")
    pts = cfg["points"][:4099]
    prm = solver_params(dict(cfg["solver"], nWalks=64), cfg["output"])
    sc = WosScene(cfg["vertices"], cfg["prims"], cfg["source"], 350.0, watertight=True)
    p1, g1, _ = sc.solve(pts, prm)
    sc.close()
    osc = oracle.OracleScene(cfg["vertices"], cfg["prims"], cfg["source"], 350.0)
    po, go, _, _, _ = oracle.solve(osc, oracle.make_params(dict(cfg["solver"], nWalks=64), cfg["output"]),
                                   pts[::37], index_base=0, index_stride=37)
    np.testing.assert_array_equal(p1[::37], po)
    np.testing.assert_array_equal(g1[::37], go)
    for r in range(world):
        d = np.load(tmp_path / f"rank{r}.npz")
        np.testing.assert_array_equal(d["p"], p1)
        np.testing.assert_array_equal(d["g"], g1)


def _oracle_projector(group, force_gather=False):
    """A PressureProjector whose engine calls are the CPU oracle (test infrastructure):
    the sharding / gather / loss logic is the product's, unchanged."""
    import torch
    import objparse
    import oracle_lib
    from wos_amd import projection as pj
    from wos_amd import workloads

    cfg = workloads.karman_config(n_walks=16)
    v, ix = objparse.load(cfg["obj"], 2)
    prm = oracle_lib.make_params(cfg["solver"], cfg["output"], n_threads=2)

    class OracleProjector(pj.PressureProjector):
        def __init__(self):
            self.dim, self.device = 2, torch.device("cpu")
            self.samples = torch.from_numpy(cfg["points"][:257].copy())
            self.group, self.force_gather, self.last_stats = group, force_gather, None

        def _set_source(self, div):
            self.osc = oracle_lib.OracleScene(v, ix, div.numpy(), 350.0)

        def _solve_points(self, x, base, stride):
            p, g, _, _, st = oracle_lib.solve(self.osc, prm, x.numpy(), index_base=base, index_stride=stride)
            return torch.from_numpy(p), torch.from_numpy(g), st

    return OracleProjector(), torch.from_numpy(cfg["source"])


def _projector_worker(rank, world, port, out_dir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "neural-monte-carlo-fluid-simulation_amd")]
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    proj, div = _oracle_projector(dist.group.WORLD)
    p, g = proj.solve(div)
    assert proj.last_stats["points_estimated"] <= (257 + world - 1) // world
    ident = lambda x: x * 0  # noqa: E731
    loss = proj.projection_loss(ident, ident, g, 64, generator=torch.Generator().manual_seed(5))
    np.savez(os.path.join(out_dir, f"proj{rank}.npz"), p=p.numpy(), g=g.numpy(), loss=float(loss))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_pressure_projector_sharded_matches_single_process(tmp_path, oracle, world):
    """PressureProjector(group=WORLD): each rank solves its stride shard of the pressure
    samples, one all-gather hands every rank the full [p, grad p]; bit-identical to the
    one-process projector, and projection_loss on the gathered field equals it too."""
    import torch
    port = _free_port()
    mp.start_processes(_projector_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    proj, div = _oracle_projector(None)
    p0, g0 = proj.solve(div)
    ident = lambda x: x * 0  # noqa: E731
    loss0 = float(proj.projection_loss(ident, ident, g0, 64, generator=torch.Generator().manual_seed(5)))
    for r in range(world):
        d = np.load(tmp_path / f"proj{r}.npz")
        np.testing.assert_array_equal(d["p"], p0.numpy())
        np.testing.assert_array_equal(d["g"], g0.numpy())
        assert float(d["loss"]) == loss0


@pytest.mark.gpu
def test_pressure_projector_rccl_world1(tmp_path, gpu):
    """PressureProjector(group=WORLD, force_gather=True) on a world-1 RCCL group: the
    shard + all_gather_into_tensor path on MI355X equals the unsharded projector bit
    for bit (device tensors throughout)."""
    import subprocess
    import sys
    port = _free_port()
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_engine_worker.py")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, worker, "0", "1", str(port), str(tmp_path), "projector"], env=env,
                       capture_output=True, text=True, timeout=150)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "PressureProjector over RCCL" in r.stdout
    d = np.load(tmp_path / "proj0.npz")
    assert d["p"].shape[0] > 3000
    np.testing.assert_array_equal(d["p"].view(np.uint32), d["p1"].view(np.uint32))
    np.testing.assert_array_equal(d["g"].view(np.uint32), d["g1"].view(np.uint32))
