"""GPU tests of the per-step scene hand-off (wos_scene_set_source, the shared
per-device workspace and the geometry cache of csrc/wos_capi.hip).  The reference
builds a fresh Scene(sceneConfig, div) every projection (model_split.py:185-202);
every cheaper path here must give bit-identical p and grad p."""
import numpy as np
import pytest
import torch

import objparse
import zombie_bindings
from wos_amd import WosScene, release_caches, solver_params, workloads

pytestmark = pytest.mark.gpu


def _cfg():
    cfg = workloads.karman_config(n_walks=32)
    v, ix = objparse.load(cfg["obj"], 2)
    return cfg, v, ix, cfg["points"][:1024]


def _other_source(src):
    h, w = src.shape
    y, x = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
    return np.ascontiguousarray(np.cos(4 * x) * np.sin(3 * y) - 0.3, np.float32)


def _solve(sc, cfg, pts):
    p, g, _ = sc.solve(pts, solver_params(cfg["solver"], cfg["output"]))
    if torch.is_tensor(p):
        p, g = p.cpu().numpy(), g.cpu().numpy()
    return p.view(np.uint32), g.view(np.uint32)


def test_set_source_matches_fresh_scene(gpu):
    cfg, v, ix, pts = _cfg()
    src2 = _other_source(cfg["source"])
    fresh = WosScene(v, ix, src2, 350.0, watertight=True)
    p_ref, g_ref = _solve(fresh, cfg, pts)
    fresh.close()
    sc = WosScene(v, ix, cfg["source"], 350.0, watertight=True)
    p1, _ = _solve(sc, cfg, pts)
    assert not np.array_equal(p1, p_ref)
    sc.set_source(src2)                              # host array
    p2, g2 = _solve(sc, cfg, pts)
    assert np.array_equal(p2, p_ref) and np.array_equal(g2, g_ref)
    dev = torch.device("cuda", 0)
    sc.set_source(torch.from_numpy(cfg["source"]).to(dev))
    sc.set_source(torch.from_numpy(src2).to(dev))   # device tensor, device-to-device
    p3, g3 = _solve(sc, cfg, torch.from_numpy(pts).to(dev))
    assert np.array_equal(p3, p_ref) and np.array_equal(g3, g_ref)
    sc.close()


def test_set_source_resize(gpu):
    """a larger grid reallocates; results equal a fresh scene with that grid"""
    cfg, v, ix, pts = _cfg()
    big = np.ascontiguousarray(np.kron(cfg["source"], np.ones((2, 2), np.float32)))
    fresh = WosScene(v, ix, big, 350.0, watertight=True)
    p_ref, g_ref = _solve(fresh, cfg, pts)
    fresh.close()
    sc = WosScene(v, ix, cfg["source"][:10, :10].copy(), 350.0, watertight=True)
    sc.set_source(big)
    p, g = _solve(sc, cfg, pts)
    assert np.array_equal(p, p_ref) and np.array_equal(g, g_ref)
    sc.close()


def test_geometry_cache_and_concurrent_scenes(gpu):
    """scenes on the same boundary share the prepared geometry but not the source;
    a released cache rebuilds to the same result"""
    cfg, v, ix, pts = _cfg()
    src2 = _other_source(cfg["source"])
    a = WosScene(v, ix, cfg["source"], 350.0, watertight=True)
    pa, ga = _solve(a, cfg, pts)
    b = WosScene(v, ix, src2, 350.0, watertight=True)
    pb, gb = _solve(b, cfg, pts)
    assert not np.array_equal(pa, pb)
    pa2, ga2 = _solve(a, cfg, pts)
    assert np.array_equal(pa, pa2) and np.array_equal(ga, ga2)
    a.close()
    pb2, _ = _solve(b, cfg, pts)
    assert np.array_equal(pb, pb2)
    b.close()
    release_caches(0)
    c = WosScene(v, ix, cfg["source"], 350.0, watertight=True)
    pc, gc = _solve(c, cfg, pts)
    assert np.array_equal(pa, pc) and np.array_equal(ga, gc)
    st = c.solve(pts, solver_params(cfg["solver"], cfg["output"]))[2]
    assert st["walk_blocks_per_cu"] >= 1 and st["first_ball_blocks_per_cu"] >= 1 and st["star_grid"] == 1
    c.close()


def test_shim_per_step_scene_pattern(gpu):
    """zombie_bindings used exactly like model_split.py:191-194 over several steps,
    against one scene whose source is replaced each step"""
    cfg, v, ix, pts = _cfg()
    scene_cfg = dict(cfg["scene"], boundary=cfg["obj"])
    sources = [cfg["source"], _other_source(cfg["source"]), cfg["source"] * 0.5]
    keep = zombie_bindings.Scene(scene_cfg, sources[0])
    for src in sources:
        sc = zombie_bindings.Scene(scene_cfg, src)
        _, p, g = zombie_bindings.wost(sc, cfg["solver"], cfg["output"], pts, return_numpy=True)
        keep.set_source(src)
        _, p2, g2 = zombie_bindings.wost(keep, cfg["solver"], cfg["output"], pts, return_numpy=True)
        assert np.array_equal(p.view(np.uint32), p2.view(np.uint32))
        assert np.array_equal(g.view(np.uint32), g2.view(np.uint32))


def test_streams_are_ordered(gpu):
    """async solves of two scenes on two streams share the device workspace: the
    second waits for the first (ctx_order), so both results stay exact"""
    cfg, v, ix, pts = _cfg()
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(pts).to(dev)
    prm = solver_params(cfg["solver"], cfg["output"])
    a = WosScene(v, ix, cfg["source"], 350.0, watertight=True)
    b = WosScene(v, ix, _other_source(cfg["source"]), 350.0, watertight=True)
    pa_ref = a.solve(x, prm)[0].cpu().numpy()
    pb_ref = b.solve(x, prm)[0].cpu().numpy()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s1):
        pa = a.solve(x, prm, sync=False)[0]
    with torch.cuda.stream(s2):
        pb = b.solve(x, prm, sync=False)[0]
    torch.cuda.synchronize()
    assert np.array_equal(pa.cpu().numpy().view(np.uint32), pa_ref.view(np.uint32))
    assert np.array_equal(pb.cpu().numpy().view(np.uint32), pb_ref.view(np.uint32))
    a.close()
    b.close()


def test_async_solves_report_their_own_stats(gpu):
    """WOS_ASYNC + wos_solve_stats: several solves enqueued back to back (different
    point sets) each report the statistics of a blocking solve of the same points,
    and give the same bit-exact outputs."""
    cfg, v, ix, pts = _cfg()
    dev = torch.device("cuda", 0)
    prm = solver_params(cfg["solver"], cfg["output"])
    sc = WosScene(v, ix, cfg["source"], 350.0, watertight=True)
    sets = [torch.from_numpy(np.ascontiguousarray(pts[k * 256:(k + 1) * 256 + 64 * k])).to(dev) for k in range(3)]
    want = []
    for x in sets:
        p, g, st = sc.solve(x, prm)
        want.append((p.cpu().numpy().view(np.uint32), g.cpu().numpy().view(np.uint32), st))
    enq = [sc.solve(x, prm, sync=False) for x in sets]
    for (p, g, st0), (pw, gw, stw) in zip(enq, want):
        assert set(k for k, v in st0.items() if v) <= {"ticket"} and st0["ticket"] > 0
        st = sc.solve_stats(st0["ticket"])
        assert np.array_equal(p.cpu().numpy().view(np.uint32), pw)
        assert np.array_equal(g.cpu().numpy().view(np.uint32), gw)
        for k in ("walk_steps", "wasted_steps", "walks_recorded", "points_estimated", "rejection_iters"):
            assert st[k] == stw[k], k
        assert st["kernel_ms"] > 0 and st["walk_ms"] > 0
    with pytest.raises(Exception):
        sc.solve_stats(0)
    with pytest.raises(Exception):
        sc.solve_stats(enq[-1][2]["ticket"] + 1000)
    sc.close()


def _stats_equal(st, ref):
    for k in ("walk_steps", "wasted_steps", "walks_recorded", "points_estimated", "rejection_iters"):
        assert st[k] == ref[k], k


def test_async_stats_slot_eviction(gpu):
    """17 async solves (> kStatSlots = 16): the first ticket is evicted (WOS_E_INVALID),
    the newest still reports the stats of a blocking solve of the same points."""
    cfg, v, ix, pts = _cfg()
    dev = torch.device("cuda", 0)
    prm = solver_params(cfg["solver"], cfg["output"])
    sc = WosScene(v, ix, cfg["source"], 350.0, watertight=True)
    x = torch.from_numpy(np.ascontiguousarray(pts[:300])).to(dev)
    p_ref, g_ref, st_ref = sc.solve(x, prm)
    enq = [sc.solve(x, prm, sync=False) for _ in range(17)]
    with pytest.raises(Exception):
        sc.solve_stats(enq[0][2]["ticket"])
    st = sc.solve_stats(enq[-1][2]["ticket"])
    _stats_equal(st, st_ref)
    assert torch.equal(enq[-1][0], p_ref) and torch.equal(enq[-1][1], g_ref)
    sc.close()


def test_async_stats_two_streams_alternating(gpu):
    """async solves alternating between two torch streams (ctx_order + the shared
    device counters): every slot's counters belong to its own solve."""
    cfg, v, ix, pts = _cfg()
    dev = torch.device("cuda", 0)
    prm = solver_params(cfg["solver"], cfg["output"])
    sc = WosScene(v, ix, cfg["source"], 350.0, watertight=True)
    sets = [torch.from_numpy(np.ascontiguousarray(pts[k * 200:(k + 1) * 200 + 50 * k])).to(dev) for k in range(6)]
    want = [sc.solve(x, prm) for x in sets]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    enq = []
    for k, x in enumerate(sets):
        enq.append(sc.solve(x, prm, sync=False, stream=streams[k % 2]))
    for (p, g, st0), (pw, gw, stw) in zip(enq, want):
        st = sc.solve_stats(st0["ticket"])
        _stats_equal(st, stw)
        torch.cuda.synchronize()
        assert torch.equal(p, pw) and torch.equal(g, gw)
    sc.close()
