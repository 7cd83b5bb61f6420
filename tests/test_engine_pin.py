"""The oracle and the HIP path against the reference's own outputs: the upstream engine demo's
solutions/wost.pfm and bvc.pfm (fixture tests/golden/engine_scene.npz; the scene rebuilt by
tests/engine_pin.py upstream_scene, DESIGN.md "What pins the oracle" 4).

1. Zero pattern, every one of the 65 536 pixels of both images: the writer's rule (grid.h:316-319)
   on the rebuilt scene zeroes exactly the pixels the reference zeroed -- no residual.  The fork's
   own conventions (no normalisation, the padded non-square box) or the unflipped winding break it.
2. Values: wost.pfm is one 96-walk estimate per pixel of the harmonic Dirichlet problem with
   image-valued g (Neumann walls reflecting).  Per unmasked pixel z = (p_ref - p)/sigma with
   sigma^2 = s^2/96 + Var(p), s^2 the per-walk variance; pass: |mean z| < 0.1, chi^2/N < 1.25,
   at most 1 % of |z| > 4.  This pins the harmonic estimator, Dirichlet termination and the
   projection onto the Dirichlet boundary, Neumann reflection and the star radius on a
   647-segment non-convex outline against the reference itself.
3. The HIP path bit for bit against the oracle on the same scene (GPU).
"""
import numpy as np
import pytest

import engine_pin as ep

Z_MEAN, CHI2, FRAC4 = 0.1, 1.25, 0.01


def _oracle_scene(oracle, U, dirichlet_image=None):
    (nv, nix), (dv, dix) = U["neumann"], U["dirichlet"]
    img = U["dirichlet_image"] if dirichlet_image is None else dirichlet_image
    return oracle.OracleScene(nv, nix, np.zeros((4, 4), np.float32), 0.0, dvertices=dv, dprims=dix,
                              dirichlet_image=img, dirichlet_image_box=U["box"], watertight=True)


def _writer_mask(U, inside, sel=slice(None)):
    pts = U["pts"][sel]
    (nv, nix), (dv, dix) = U["neumann"], U["dirichlet"]
    return ep.writer_mask(inside, ep.near_boundary(dv, dix, pts, ep.MASK), ep.near_boundary(nv, nix, pts, ep.MASK))


def _zstats(ref, p, var_walk, n_ours):
    sig = np.sqrt(var_walk / ep.WOST_WALKS + var_walk / n_ours)
    z = np.where(sig > 0, (ref - p) / np.where(sig > 0, sig, 1.0), np.where(ref == p, 0.0, np.inf))
    return {"n": int(z.size), "mean_z": float(z.mean()), "chi2_n": float((z * z).mean()),
            "frac_z4": float((np.abs(z) > 4).mean()), "max_z": float(np.abs(z).max()),
            "mean_diff": float((ref - p).mean())}


def _check(st):
    assert abs(st["mean_z"]) < Z_MEAN, st
    assert st["chi2_n"] < CHI2, st
    assert st["frac_z4"] <= FRAC4, st


def _inside(oracle, U):
    """estimated <=> inside the domain (insideDomain, fcpw_scene_loader.h:642-648): a 1-step
    solve (a point's step count is > 0 iff it was estimated)."""
    osc = _oracle_scene(oracle, U)
    solver = dict(ep.WOST_SOLVER, nWalks=1, maxWalkLength=1)
    _, _, _, steps, _ = oracle.solve(osc, oracle.make_params(solver, ep.WOST_OUTPUT), U["pts"])
    return steps > 0


def test_zero_pattern_matches_reference_images(oracle):
    U = ep.upstream_scene()
    assert U["n_neumann"] == 410 and len(U["dirichlet"][1]) == 237  # outer walls / the five holes
    mask = _writer_mask(U, _inside(oracle, U))
    for name in ("values", "bvc_values"):
        zero = U[name] == 0
        assert int((mask & ~zero).sum()) == 0 and int((~mask & zero).sum()) == 0, name
    assert int(mask.sum()) == 36665
    # negative controls: the fork's Scene conventions (scene.h:32,144) or the unflipped winding
    for kw in ({"normalize": False, "square": False}, {"square": False}, {"normalize": False},
               {"flip": False}):
        V = ep.upstream_scene(**kw)
        m = _writer_mask(V, _inside(oracle, V))
        zero = V["values"] == 0
        assert int((m != zero).sum()) > 1000, kw


def test_oracle_values_match_reference_wost(oracle):
    """The oracle's estimate (256 walks) against wost.pfm on every 29th pixel."""
    U = ep.upstream_scene()
    sel = np.arange(0, U["pts"].shape[0], 29)
    osc = _oracle_scene(oracle, U)
    solver = dict(ep.WOST_SOLVER, nWalks=256)
    p, _, n_est, _, st, m2 = oracle.solve(osc, oracle.make_params(solver, ep.WOST_OUTPUT), U["pts"][sel],
                                          index_base=0, index_stride=29, m2=True)
    assert st["walks_escaped"] == 0 and st["walks_max_length"] == 0
    assert st["walks_dirichlet"] == st["walks_recorded"] > 0
    ok = ~_writer_mask(U, n_est > 0, sel)
    var = m2 / np.maximum(n_est - 1, 1)
    stats = _zstats(U["values"][sel][ok], p[ok], var[ok], n_est[ok])
    print("oracle vs wost.pfm", stats)
    assert stats["n"] > 1000
    _check(stats)
    # the pin discriminates: the fork's file-order reading of the Dirichlet image fails it
    bad = _oracle_scene(oracle, U, np.ascontiguousarray(U["dirichlet_image"][::-1]))
    pb, _, nb, _, _, m2b = oracle.solve(bad, oracle.make_params(solver, ep.WOST_OUTPUT), U["pts"][sel],
                                        index_base=0, index_stride=29, m2=True)
    vb = m2b / np.maximum(nb - 1, 1)
    sb = _zstats(U["values"][sel][ok], pb[ok], vb[ok], nb[ok])
    assert sb["chi2_n"] > 10 * CHI2, sb


def _hip_scene(U, dirichlet_image=None):
    from wos_amd import WosScene
    (nv, nix), (dv, dix) = U["neumann"], U["dirichlet"]
    img = U["dirichlet_image"] if dirichlet_image is None else dirichlet_image
    return WosScene(nv, nix, np.zeros((4, 4), np.float32), 0.0, dvertices=dv, dprims=dix,
                    dirichlet_image=img, dirichlet_image_box=U["box"], watertight=True)


@pytest.mark.gpu
def test_hip_upstream_engine_bit_exact(gpu, oracle):
    """Image-valued Dirichlet data on the mixed engine scene: HIP path == oracle bit for bit
    (p, grad, walks and steps per point) on every 13th grid point."""
    from wos_amd import solver_params
    U = ep.upstream_scene()
    sel = np.arange(0, U["pts"].shape[0], 13)
    pts = U["pts"][sel]
    sc = _hip_scene(U)
    p, g, st, n_est, steps = sc.solve(pts, solver_params(ep.WOST_SOLVER, ep.WOST_OUTPUT), counts=True,
                                      index_base=0, index_stride=13)
    sc.close()
    po, go, no, so, sto = oracle.solve(_oracle_scene(oracle, U), oracle.make_params(ep.WOST_SOLVER, ep.WOST_OUTPUT),
                                       pts, index_base=0, index_stride=13)
    assert st["walks_dirichlet"] == sto["walks_dirichlet"] > 0
    np.testing.assert_array_equal(n_est, no)
    np.testing.assert_array_equal(steps, so)
    np.testing.assert_array_equal(p.view(np.uint32), po.view(np.uint32))
    np.testing.assert_array_equal(g.view(np.uint32), go.view(np.uint32))


@pytest.mark.gpu
def test_hip_values_match_reference_wost(gpu, oracle):
    """The HIP engine on all 65 536 pixels: zero pattern exact, values within the Monte-Carlo
    error of wost.pfm.  The per-walk variance comes from a second solve with g^2 on the same
    walks (the walk value is g at the exit point: s^2 = E[g^2] - E[g]^2)."""
    from wos_amd import solver_params
    U = ep.upstream_scene()
    sc, sc2 = _hip_scene(U), _hip_scene(U, U["dirichlet_image"] ** 2)
    p = p2 = n_est = 0
    steps = 0
    for key in range(4):  # 4 x 512 walks (one solve's nWalks is bounded by the first-ball LDS)
        prm = solver_params(dict(ep.WOST_SOLVER, nWalks=512, seed=0x5EED4000 + key), ep.WOST_OUTPUT)
        pk, _, st, nk, _ = sc.solve(U["pts"], prm, counts=True)
        p2k, _, _, n2k, _ = sc2.solve(U["pts"], prm, counts=True)
        np.testing.assert_array_equal(nk, n2k)
        p, p2, n_est = p + pk.astype(np.float64) * nk, p2 + p2k.astype(np.float64) * nk, n_est + nk
        steps += st["walk_steps"]
    sc.close()
    sc2.close()
    p, p2 = p / np.maximum(n_est, 1), p2 / np.maximum(n_est, 1)
    mask = _writer_mask(U, n_est > 0)
    zero = U["values"] == 0
    assert int((mask != zero).sum()) == 0
    ok = ~mask
    var = np.maximum(p2 - p * p, 0.0)
    stats = _zstats(U["values"][ok], p[ok], var[ok], n_est[ok])
    print("HIP engine vs wost.pfm", stats, "walk steps", steps)
    assert stats["n"] == 65536 - 36665
    _check(stats)
