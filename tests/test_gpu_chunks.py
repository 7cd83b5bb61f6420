"""A solve whose walk tasks exceed one task batch (wos_set_max_batch_tasks, default 2^28 walks)
runs in several walk-kernel launches; each later batch resets only the queue counters and the
bucket histogram (one zero-kernel launch) and keys its points by their global index.  Config E
takes this path (8 batches).  Here the batch is capped at 2^20 walks and karman with
2^20/128 + 1000 points at 128 walks (two batches) must equal the same points solved as two
index_base-keyed halves bit for bit (p, grad, walks and steps per point, the walk-step
statistics), and the oracle on a strided subset of the second batch at the same global indices;
a third solve at the default batch (one launch) must equal them too."""
import numpy as np
import pytest

import objparse
from wos_amd import WosScene, set_max_batch_tasks, solver_params, workloads

pytestmark = pytest.mark.gpu

BATCH = 1 << 20
N_POINTS = BATCH // 128 + 1000


def test_two_batch_solve_equals_halves_and_oracle(gpu, oracle):
    cfg = workloads.karman_config(n_walks=128, n_points=N_POINTS + 2000)
    pts = np.ascontiguousarray(cfg["points"][:N_POINTS], np.float32)
    assert len(pts) == N_POINTS
    v, ix = objparse.load(cfg["obj"], 2)
    sc = WosScene(v, ix, cfg["source"], 350.0, watertight=True)
    prm = solver_params(cfg["solver"], cfg["output"])
    old = set_max_batch_tasks(BATCH)
    try:
        p, g, st, n_est, steps = sc.solve(pts, prm, counts=True)
        assert st["walk_launches"] >= 2, st
        h = N_POINTS // 2
        p1, g1, st1, n1, s1 = sc.solve(pts[:h], prm, counts=True, index_base=0)
        p2, g2, st2, n2, s2 = sc.solve(pts[h:], prm, counts=True, index_base=h)
        assert st1["walk_launches"] == 1 and st2["walk_launches"] == 1
    finally:
        assert set_max_batch_tasks(old) == BATCH
    p3, g3, st3 = sc.solve(pts, prm)
    assert st3["walk_launches"] == 1
    sc.close()
    np.testing.assert_array_equal(p.view(np.uint32), p3.view(np.uint32))
    np.testing.assert_array_equal(g.view(np.uint32), g3.view(np.uint32))
    np.testing.assert_array_equal(p.view(np.uint32), np.concatenate([p1, p2]).view(np.uint32))
    np.testing.assert_array_equal(g.view(np.uint32), np.concatenate([g1, g2]).view(np.uint32))
    np.testing.assert_array_equal(n_est, np.concatenate([n1, n2]))
    np.testing.assert_array_equal(steps, np.concatenate([s1, s2]))
    for k in ("walk_steps", "wasted_steps", "walks_recorded", "walks_rr", "points_estimated", "rejection_iters"):
        assert st[k] == st1[k] + st2[k], k
    # oracle on every 61st point of the second batch (global indices 8192 + 61 k)
    b0 = BATCH // 128
    sel = np.arange(b0, N_POINTS, 61)
    po, go, no, so, _ = oracle.solve(oracle.OracleScene(v, ix, cfg["source"], 350.0),
                                     oracle.make_params(cfg["solver"], cfg["output"]), pts[sel],
                                     index_base=b0, index_stride=61)
    np.testing.assert_array_equal(p[sel].view(np.uint32), po.view(np.uint32))
    np.testing.assert_array_equal(g[sel].view(np.uint32), go.view(np.uint32))
    np.testing.assert_array_equal(n_est[sel], no)
    np.testing.assert_array_equal(steps[sel], so)
