"""The LiDAR-like scene (icp_synth_scene: ground + walls scanned from two poses, range-dependent
density, 1 mm LAS grid): the 2.5-D surface data the reference's LAS flow feeds it
(lasio.cpp:7-125, icp_registration.cpp:248-378), where early iterates leave every query ~0.1-1 m
off surfaces sampled every few mm (search boxes overflow, the follow-up searches carry the load)
and the 1 mm grid makes exact ties. Parity against the CPU oracle (pinned to the reference by
tests/test_oracle_golden.py): every iterate's correspondences and residuals bit for bit, the final
transform to the north star's 1e-6 RMSE (observed ~1e-15) and the oracle's engine loop to 1e-9.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1_000_000
ITERS = 5


@pytest.fixture(scope="module")
def scene(icp):
    return icp.synth_scene(N)


def _Tres(res):
    T = np.eye(4)
    T[:3, :3] = np.array(res.final_R).reshape(3, 3)
    T[:3, 3] = res.final_t
    return T


def test_scene_correspondences_every_iterate(icp, oracle, scene):
    tgt, src, _ = scene
    tree = oracle.OracleTree(tgt)
    fallback = 0
    with icp.Context(0) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        T = None
        for it in range(ITERS):
            st = ctx.iterate(T, it, icp.RULES_ENGINE, 3.0)
            q = ctx.get_source()
            idx, d = ctx.get_correspondences()
            oidx, od = tree.nn(q, init_best=oracle.DBL_MAX)
            np.testing.assert_array_equal(idx, oidx, err_msg=f"iterate {it}")
            np.testing.assert_array_equal(d, od, err_msg=f"iterate {it}")
            fallback += st.n_fallback
            T = icp.best_fit_from_stats(st)
    # the reference-order DFS takes the exact ties (the 1 mm grid's duplicates) and little else
    assert fallback <= 0.005 * N * ITERS


def test_scene_registration_vs_oracle(icp, oracle, scene):
    tgt, src, T_true = scene
    p = icp.params_default(max_iterations=ITERS, tolerance=0.0)
    rc, res, hist, _ = icp.engine_register(p, src, tgt, device=0)
    assert rc == 0 and res.success and res.total_iterations == ITERS
    orc, ores, ohist, _ = oracle.icp(src, tgt, oracle.SEM_ENGINE, ITERS, p.tolerance)
    assert orc == 0
    assert [h.valid_points for h in hist] == [h.valid for h in ohist]
    T, To = _Tres(res), _Tres(ores)
    assert float(np.sqrt(np.mean((T - To) ** 2))) <= 1e-6
    np.testing.assert_allclose(T, To, atol=1e-9)
    np.testing.assert_allclose(res.final_rmse, ores.final_rmse, rtol=1e-9)
    # the registration moves towards the known pose (5 iterates of a 2 deg / 0.36 m offset)
    err0 = np.abs(np.eye(4) - T_true)[:3, 3].max()
    assert np.abs(T - T_true)[:3, 3].max() < err0


@pytest.mark.parametrize("which", ["scene", "blob"])
def test_ball_modes_agree(icp, oracle, scene, which):
    """k_nn_ball's two ways through the queries the wave search left (config.ball_mode: 1 the
    four-per-wave ball walk with its follow-ups, 2 a whole query per wave by the cooperative
    search, 0 the size rule between them): the same correspondences, residuals and statistics bit
    for bit over the first iterates (long lists of far queries on the scene, short ones on the
    blob), and the oracle's on the last one."""
    if which == "scene":
        tgt, src, _ = scene
    else:
        tgt, src, _ = icp.synth_pair(300_000, yaw_deg=3.0)
    out = {}
    for mode in (0, 1, 2):
        with icp.Context(0, icp.config(ball_mode=mode)) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            T, recs = None, []
            for it in range(3):
                st = ctx.iterate(T, it, icp.RULES_ENGINE, 3.0)
                recs.append((st.valid, st.mean, st.std, st.rmse, tuple(st.H)))
                T = icp.best_fit_from_stats(st)
            idx, d = ctx.get_correspondences()
            out[mode] = (recs, idx, d, ctx.get_source())
    for mode in (1, 2):
        assert out[mode][0] == out[0][0]
        for k in (1, 2, 3):
            np.testing.assert_array_equal(out[mode][k], out[0][k])
    oidx, od = oracle.OracleTree(tgt).nn(out[0][3], init_best=oracle.DBL_MAX)
    np.testing.assert_array_equal(out[0][1], oidx)
    np.testing.assert_array_equal(out[0][2], od)


@pytest.mark.parametrize("which", ["scene", "blob"])
def test_wide_pass_modes_agree(icp, oracle, scene, which):
    """The wide pass (config.wide_pass: 1 never, 2 always, 0 the rule; k_nn_wide walks and scans an
    overflowed wave's box in segments) against the ball search taking those queries: the same
    correspondences, residuals and statistics bit for bit over 4 iterates (every iterate's
    correspondences checked against the oracle with the pass always on), also without the half
    pass of the first iterate."""
    if which == "scene":
        tgt, src, _ = scene
    else:
        tgt, src, _ = icp.synth_pair(300_000, yaw_deg=3.0)
    tree = oracle.OracleTree(tgt)
    out = {}
    for key in ((0, 1), (1, 1), (2, 1), (2, 0)):
        wide, halves = key
        with icp.Context(0, icp.config(wide_pass=wide, overflow_halves=halves)) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            T, recs, corr = None, [], []
            for it in range(4):
                st = ctx.iterate(T, it, icp.RULES_ENGINE, 3.0)
                recs.append((st.valid, st.mean, st.std, st.rmse, tuple(st.H)))
                idx, d = ctx.get_correspondences()
                corr.append((idx, d))
                if key == (2, 1):
                    oidx, od = tree.nn(ctx.get_source(), init_best=oracle.DBL_MAX)
                    np.testing.assert_array_equal(idx, oidx, err_msg=f"iterate {it}")
                    np.testing.assert_array_equal(d, od, err_msg=f"iterate {it}")
                T = icp.best_fit_from_stats(st)
            out[key] = (recs, corr)
    for key in out:
        assert out[key][0] == out[(1, 1)][0], key
        for (i0, d0), (i1, d1) in zip(out[key][1], out[(1, 1)][1]):
            np.testing.assert_array_equal(i0, i1)
            np.testing.assert_array_equal(d0, d1)


def test_scene_vs_reference_fixture(icp, golden_scene, golden_meta):
    """The HIP path on the REFERENCE's own surface fixture (tests/golden/scene_ref.npz, made by
    oracle/_ref from icp_registration.cpp and core/icpengine.cpp): the CLI octree's correspondences
    and residuals of the source and of the CLI ICP's final source bit for bit; the CLI ICP's 20
    cumulative transforms; the core engine's 10-iterate registration (north star: 1e-6 RMSE;
    asserted to 1e-9)."""
    g, m = golden_scene, golden_meta["scene_ref"]
    src, tgt = g["scene_source"], g["scene_target"]
    with icp.Context(0) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_CLI)
        for q, key in ((src, "iter0"), (g["scene_cli_source_out"], "final")):
            idx, d = ctx.nn(q)
            np.testing.assert_array_equal(idx, g[f"scene_idx_{key}_cli"], err_msg=key)
            np.testing.assert_array_equal(d, g[f"scene_dist_{key}_cli"], err_msg=key)
    R, t, tcums, out = icp.cli_icp(src, tgt, m["cli_iterations"], m["cli_tolerance"], device=0)
    ref = g["scene_cli_T_cums"]
    assert tcums.shape == ref.shape
    assert _trmse(tcums[-1], ref[-1]) < 1e-6
    np.testing.assert_allclose(tcums, ref, atol=1e-9)
    np.testing.assert_allclose(out, g["scene_cli_source_out"], atol=1e-8)
    e = m["engine"]
    p = icp.params_default(max_iterations=e["iterations"], tolerance=e["tolerance"], sigma_multiplier=e["sigma"])
    rc, res, hist, out = icp.engine_register(p, src, tgt, device=0)
    assert rc == 0 and res.success and res.total_iterations == e["total_iterations"]
    Tg, Tr = _Tres(res), np.eye(4)
    Tr[:3, :3] = g["scene_engine_R"]
    Tr[:3, 3] = g["scene_engine_t"]
    assert _trmse(Tg, Tr) < 1e-6
    np.testing.assert_allclose(Tg, Tr, atol=1e-9)
    np.testing.assert_allclose(res.final_rmse, e["final_rmse"], rtol=1e-9)
    np.testing.assert_allclose(out, g["scene_engine_source_out"], atol=1e-8)
    h = g["scene_engine_history"]
    assert [r.valid_points for r in hist] == [int(x) for x in h[: len(hist), 2]]


def _trmse(a, b):
    return float(np.sqrt(np.mean((np.asarray(a) - np.asarray(b)) ** 2)))
