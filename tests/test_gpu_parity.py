"""GPU parity tests: the HIP path through the C-ABI against the golden vectors of the reference
and the CPU oracle on the same inputs.

Bar (BASELINE.json north_star): correspondence indices bit-exact against the CPU octree for
identical query coordinates (residuals too — they are sqrt of the same best distance);
per-iteration statistics within 1e-12 relative (the GPU sums in a different order);
final 4x4 transform within 1e-6 RMSE of the CPU/Eigen reference (observed ~1e-14).
"""
import numpy as np
import pytest

from conftest import ENGINE_CASES, KAT_CASES, engine_expected, fnv1a

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-6  # final transform, north_star


def t_rmse(a, b):
    return float(np.sqrt(np.mean((np.asarray(a) - np.asarray(b)) ** 2)))


@pytest.mark.parametrize("case", KAT_CASES)
def test_nn_kat_cli_rules(icp, gpu_ctx, golden_nn, case):
    t, q = golden_nn[f"{case}_target"], golden_nn[f"{case}_query"]
    gpu_ctx.set_target(t, 10, 20, icp.RULES_CLI)
    idx, d = gpu_ctx.nn(q)
    np.testing.assert_array_equal(idx, golden_nn[f"{case}_idx_cli"])
    np.testing.assert_array_equal(d, golden_nn[f"{case}_dist_cli"])


@pytest.mark.parametrize("case", KAT_CASES)
def test_nn_kat_engine_rules(icp, oracle, gpu_ctx, golden_nn, case):
    t, q = golden_nn[f"{case}_target"], golden_nn[f"{case}_query"]
    gpu_ctx.set_target(t, 10, 20, icp.RULES_ENGINE)
    idx, d = gpu_ctx.nn(q)
    oidx, od = oracle.OracleTree(t).nn(q, init_best=oracle.DBL_MAX)
    np.testing.assert_array_equal(idx, oidx)
    np.testing.assert_array_equal(d, od)


@pytest.mark.parametrize("mp,md", [(5, 10), (100, 50), (10, 3)])
def test_nn_octree_params(icp, gpu_ctx, golden_nn, mp, md):
    t, q = golden_nn["gauss_target"], golden_nn["gauss_query"]
    gpu_ctx.set_target(t, mp, md, icp.RULES_CLI)
    idx, _ = gpu_ctx.nn(q)
    np.testing.assert_array_equal(idx, golden_nn[f"gauss_idx_cli_p{mp}_d{md}"])


def test_nn_100k_reference_hash_and_work(icp, gpu_ctx, golden_meta):
    m = golden_meta["nn_100k"]
    tgt, src, _ = icp.synth_pair(m["n"])
    gpu_ctx.set_target(tgt, 10, 20, icp.RULES_CLI)
    idx, _ = gpu_ctx.nn(src)
    assert fnv1a(idx) == m["idx_fnv1a"]
    gpu_ctx.set_source(src)
    gpu_ctx.iterate(None, 0, icp.RULES_CLI, 3.0)
    v, p = gpu_ctx.traversal_counts()
    # the kernel counts the reference DFS's node entries / scanned points exactly
    assert v == pytest.approx(m["mean_node_entries"], rel=0, abs=1e-9)
    assert p == pytest.approx(m["mean_leaf_points"], rel=0, abs=1e-9)


def test_nn_edge_queries(icp, oracle, gpu_ctx):
    rng = np.random.default_rng(5)
    t = rng.normal(size=(3000, 3))
    q = np.concatenate([
        t[:50],                                   # exact hits
        np.array([[np.nan, 0, 0], [0, np.inf, 0], [-np.inf, 1, 1], [np.nan] * 3]),
        np.zeros((3, 3)), rng.normal(size=(50, 3)) * 100])
    for rules, init in [(icp.RULES_ENGINE, oracle.DBL_MAX), (icp.RULES_CLI, 1e20)]:
        gpu_ctx.set_target(t, 10, 20, rules)
        idx, d = gpu_ctx.nn(q)
        oidx, od = oracle.OracleTree(t).nn(q, init_best=init)
        np.testing.assert_array_equal(idx, oidx)
        np.testing.assert_array_equal(np.isnan(d), np.isnan(od))
        np.testing.assert_array_equal(d[~np.isnan(d)], od[~np.isnan(od)])
    np.testing.assert_array_equal(idx[:50], np.arange(50))


def test_apply_bits_match_eigen(icp, gpu_ctx, golden_svd):
    pts = golden_svd["pts"]
    gpu_ctx.set_target(pts, 10, 20, icp.RULES_ENGINE)
    gpu_ctx.set_source(pts)
    gpu_ctx.apply(golden_svd["T"])
    np.testing.assert_array_equal(gpu_ctx.get_source(), golden_svd["T_pts"])  # Eigen T*src bits


def test_iterate_stats_match_oracle(icp, oracle, gpu_ctx):
    tgt, src, _ = icp.synth_pair(20000, yaw_deg=4.0)
    gpu_ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
    gpu_ctx.set_source(src)
    st = gpu_ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
    oidx, od = oracle.OracleTree(tgt).nn(src, init_best=oracle.DBL_MAX)
    idx, d = gpu_ctx.get_correspondences()
    np.testing.assert_array_equal(idx, oidx)
    np.testing.assert_array_equal(d, od)
    mean = od.sum() / len(od)
    sd = np.sqrt(((od - mean) ** 2).sum() / len(od))
    thr = mean + max(3.0 * sd, 0.5 * mean)
    v = od <= thr
    assert st.n == len(src) and st.valid == int(v.sum())
    np.testing.assert_allclose([st.mean, st.std, st.threshold], [mean, sd, thr], rtol=1e-12)
    np.testing.assert_allclose(st.rmse, np.sqrt((od[v] ** 2).sum() / v.sum()), rtol=1e-12)
    a, b = src[v], tgt[oidx[v]]
    np.testing.assert_allclose(st.centroid_src, a.mean(0), rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(st.centroid_tgt, b.mean(0), rtol=1e-12, atol=1e-13)
    H = (a - a.mean(0)).T @ (b - b.mean(0))
    np.testing.assert_allclose(np.array(st.H).reshape(3, 3), H, rtol=1e-10, atol=1e-10 * np.abs(H).max())
    assert st.min_d == od.min() and st.max_d == od.max() and st.n_bad == 0
    # host best fit from the device moments vs the oracle's (Eigen-equivalent) best fit
    np.testing.assert_allclose(icp.best_fit_from_stats(st), oracle.best_fit(a, b), atol=1e-12)


@pytest.mark.parametrize("name", ["cfg1_1k", "g10k"])
def test_cli_icp_vs_reference(icp, golden_icp, golden_meta, name):
    m = golden_meta["icp_cli"][name]
    R, t, tcums, out = icp.cli_icp(golden_icp[f"{name}_source"], golden_icp[f"{name}_target"],
                                   m["iterations"], m["tolerance"], device=0)
    ref = golden_icp[f"{name}_T_cums"]
    assert tcums.shape == ref.shape
    assert t_rmse(tcums[-1], ref[-1]) < RMSE_TOL
    np.testing.assert_allclose(tcums, ref, atol=1e-9)
    np.testing.assert_allclose(R, golden_icp[f"{name}_R_final"], atol=1e-9)  # last incremental T quirk
    np.testing.assert_allclose(t, golden_icp[f"{name}_t_final"], atol=1e-9)
    np.testing.assert_allclose(out, golden_icp[f"{name}_source_out"], atol=1e-8)


@pytest.mark.parametrize("n,yaw", [(5000, 2.0), (30000, 6.0)])
def test_engine_register_vs_oracle(icp, oracle, n, yaw):
    tgt, src, T_true = icp.synth_pair(n, yaw_deg=yaw)
    p = icp.params_default(max_iterations=50, tolerance=1e-9)
    rc, res, hist, out = icp.engine_register(p, src, tgt, device=0)
    orc, ores, ohist, oout = oracle.icp(src, tgt, oracle.SEM_ENGINE, 50, 1e-9)
    assert rc == 0 and orc == 0 and res.success
    assert res.total_iterations == ores.total_iterations
    assert [h.valid_points for h in hist] == [h.valid for h in ohist]
    T = np.eye(4)
    T[:3, :3] = np.array(res.final_R).reshape(3, 3)
    T[:3, 3] = res.final_t
    To = np.eye(4)
    To[:3, :3] = np.array(ores.final_R).reshape(3, 3)
    To[:3, 3] = ores.final_t
    assert t_rmse(T, To) < RMSE_TOL
    np.testing.assert_allclose(T, To, atol=1e-10)
    np.testing.assert_allclose(res.final_rmse, ores.final_rmse, rtol=1e-9, atol=1e-15)
    np.testing.assert_allclose(out, oout, atol=1e-9)
    for h, o in zip(hist, ohist):
        np.testing.assert_allclose(np.array(h.transform), np.array(o.T_cum), atol=1e-10)


@pytest.mark.parametrize("name", ENGINE_CASES)
def test_engine_register_vs_core_reference(icp, golden_engine, golden_meta, name):
    """The product's ICPEngine drop-in (icp_engine_register: device search + statistics, host SVD)
    against the REAL core engine (core/icpengine.cpp + moc + conda Qt, tests/golden/engine_rules.npz):
    iteration count, per-iteration valid/outlier counts and RMSE, cumulative transforms, the
    convergence record, final R/t = T_cumulative within 1e-6 RMSE (observed ~1e-15), write-back
    or none, the divergence break, cancellation via stop() at iteration 3."""
    m, g, hist = engine_expected(golden_engine, golden_meta, name)
    p = m["params"]
    params = icp.params_default(max_iterations=p["max_iterations"], tolerance=p["tolerance"],
                                sigma_multiplier=p["sigma"], octree_max_points=p["max_points"],
                                octree_max_depth=p["max_depth"])
    rc, res, rh, out = icp.engine_register(params, g["source"], g["target"], device=0, stop_at=m["stop_at"])
    assert len(rh) == len(hist)
    for r, h in zip(rh, hist):
        assert r.iteration == int(h[0]) and r.valid_points == int(h[2]) and r.outlier_points == int(h[3])
        np.testing.assert_allclose(r.rmse, h[1], rtol=1e-9, atol=1e-15)
        np.testing.assert_allclose(np.array(r.transform).reshape(4, 4), h[4:20].reshape(4, 4), atol=1e-10)
        if r.has_transform:
            # acos((tr - 1) / 2) is ill-conditioned near 0: at 1.6e-4 deg (sin ~ 3e-6) a 1e-16 change
            # of the trace moves the angle by ~1e-8 deg, so the angle gets an absolute 1e-6 deg bound
            np.testing.assert_allclose(r.rotation_angle_deg, h[20], rtol=1e-6, atol=1e-6)
            np.testing.assert_allclose(r.translation_distance, h[21], rtol=1e-6, atol=1e-9)
        else:  # the convergence record leaves them unset in the reference
            assert np.isnan(h[20])
    if m["finished"] == 0:
        assert rc != 0 and not res.success
        np.testing.assert_array_equal(out, g["source"])  # finished(false): no write-back
        return
    assert rc == 0 and res.success and res.total_iterations == m["total_iterations"]
    T = np.eye(4)
    T[:3, :3] = np.array(res.final_R).reshape(3, 3)
    T[:3, 3] = res.final_t
    Tr = np.eye(4)
    Tr[:3, :3] = g["final_R"]
    Tr[:3, 3] = g["final_t"]
    assert t_rmse(T, Tr) < RMSE_TOL
    np.testing.assert_allclose(T, Tr, atol=1e-10)
    np.testing.assert_allclose(res.final_rmse, m["final_rmse"], rtol=1e-9, atol=1e-15)
    np.testing.assert_allclose(out, g["source_out"], atol=1e-9)


def test_engine_too_few_pairs_keeps_source(icp):
    tgt = np.random.default_rng(1).normal(size=(100, 3))
    src = tgt[:2] + 0.01  # 2 points: valid < 3 on the first iteration
    p = icp.params_default()
    rc, res, hist, out = icp.engine_register(p, src, tgt, device=0)
    assert rc == -11 and not res.success  # ICP_ENGINE_TOO_FEW, finished(false) (icpengine.cpp:319-323)
    np.testing.assert_array_equal(out, src)  # no write-back
    R, t, tr, out2 = icp.cli_icp(src, tgt, 20, 1e-2, device=0)  # CLI breaks and writes back
    np.testing.assert_array_equal(R, np.eye(3))
    np.testing.assert_array_equal(out2, src)


def test_engine_stop_flag(icp):
    import ctypes
    tgt, src, _ = icp.synth_pair(5000)
    flag = ctypes.c_int32(1)
    rc, res, hist, out = icp.engine_register(icp.params_default(), src, tgt, device=0, stop_flag=flag)
    assert rc == -10 and res.status == 4 and not res.success
    np.testing.assert_array_equal(out, src)


def test_empty_inputs_rejected(icp):
    p = icp.params_default()
    rc, res, _, _ = icp.engine_register(p, np.zeros((0, 3)), np.ones((5, 3)), device=0)
    assert rc != 0 and not res.success  # icpengine.cpp:31-34
    rc, res, _, _ = icp.engine_register(p, np.ones((5, 3)), np.zeros((0, 3)), device=0)
    assert rc != 0 and not res.success


def test_kernel_variants_agree(icp, oracle):
    """The certified wave search (default) and the literal reference-order kernel agree bit for
    bit, including on inputs full of exact ties (lattice) where the exact DFS does the work."""
    rng = np.random.default_rng(9)
    tgt = rng.normal(size=(200000, 3)) * [5, 5, 1]
    q = np.concatenate([rng.normal(size=(100000, 3)) * [6, 6, 1.2], tgt[:2000]])
    lat = np.stack(np.meshgrid(np.arange(40), np.arange(40), np.arange(10), indexing="ij"), -1).reshape(-1, 3) * 0.5
    lq = np.concatenate([lat[rng.integers(0, len(lat), 5000)] + 0.25, rng.uniform(-1, 21, size=(5000, 3))])
    outs = {}
    for name, cfg in [("reference", {"search": icp.SEARCH_REFERENCE}), ("certified", {}),
                      ("certified_fp64", {"scan32": 0}), ("certified_root", {"cell_starts": 0})]:
        with icp.Context(0, cfg) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            a = ctx.nn(q)
            ctx.set_target(lat.astype(float), 10, 20, icp.RULES_CLI)
            b = ctx.nn(lq)
        outs[name] = (a, b)
    for name in outs:
        for k in range(2):
            np.testing.assert_array_equal(outs[name][k][0], outs["reference"][k][0])
            np.testing.assert_array_equal(outs[name][k][1], outs["reference"][k][1])
    oidx, _ = oracle.OracleTree(lat.astype(float)).nn(lq, init_best=1e20)
    np.testing.assert_array_equal(outs["reference"][1][0], oidx)
    np.testing.assert_array_equal(outs["certified"][1][0], oidx)


def test_fallback_share_small_on_scans(icp, gpu_ctx):
    tgt, src, _ = icp.synth_pair(500000)
    gpu_ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
    gpu_ctx.set_source(src)
    st = gpu_ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
    assert st.n_fallback <= 0.001 * len(src)


@pytest.mark.parametrize("n,cfg", [(300_000, {"scan32": 0}), (1_000_000, {"scan32": 0}),
                                   (1_000_000, {"cell_starts": 0}),
                                   (300_000, {"cell_starts": 0, "scan32": 0}),
                                   (1_000_000, {"join_factor": 1e6}),
                                   (300_000, {"octree_builder": 1}),
                                   (1_000_000, {"scan_groups": 1}), (1_000_000, {"scan_groups": 2}),
                                   (300_000, {"xcd_blocks": 0}),
                                   (1_000_000, {"candidate_cache": 0}), (300_000, {"candidate_margin": 0}),
                                   (300_000, {"candidate_margin": 256}),
                                   (1_000_000, {"overflow_halves": 1}), (1_000_000, {"wide_pass": 1}),
                                   (1_000_000, {"wide_pass": 2}), (1_000_000, {"certify_prev": 3}),
                                   (300_000, {"certify_prev": 2, "candidate_cache": 0})])
def test_scan32_matches_fp64_scan(icp, n, cfg):
    """Every configuration of the certified search (fp32 filter scan vs fp64 scan, cell-table
    starts vs root descent, join rule, host-built octree) returns exactly the default's
    correspondences and residuals, iteration after iteration of the real loop (previous-residual
    guesses, fused transform)."""
    tgt, src, _ = icp.synth_pair(n)

    def run(conf):
        out = []
        with icp.Context(0, conf) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            T = None
            for it in range(4):
                st = ctx.iterate(T, it, icp.RULES_ENGINE, 3.0)
                out.append(ctx.get_correspondences() + (st.n_fallback, st.n_ball_search))
                T = icp.best_fit_from_stats(st)
        return out

    a = run(None)
    b = run(cfg)
    for it, ((ia, da, fa, ba), (ib, db, fb, bb)) in enumerate(zip(a, b)):
        np.testing.assert_array_equal(ia, ib)
        np.testing.assert_array_equal(da, db)
        assert fa == fb
        # the same candidate sets (the candidate cache's enlarged boxes overflow other waves; the
        # first iterate's wide pass, which takes overflowed halves instead of the ball search,
        # runs with the fp32 scan only)
        if set(cfg) <= {"octree_builder", "scan_groups", "xcd_blocks"} or (set(cfg) <= {"scan32"} and it > 0):
            assert ba == bb


def test_candidate_cache_motion_and_invalidation(icp):
    """The wave search's candidate cache (reuse of a wave's enlarged-box candidate list while its
    new box lies inside) against the cache-free search: small and large motions between iterates
    (reuse and re-walk), a new target of the same size and a new source (older generations never
    reused). Correspondences and residuals identical at every step."""
    rng = np.random.default_rng(21)
    tgt, src, _ = icp.synth_pair(400_000)
    tgt2 = tgt[rng.permutation(len(tgt))] * 1.01 + 0.003
    src2 = src[rng.permutation(len(src))][:300_000] + 0.01

    def rot(deg, t):
        c, s_ = np.cos(np.radians(deg)), np.sin(np.radians(deg))
        T = np.eye(4)
        T[:3, :3] = [[c, -s_, 0], [s_, c, 0], [0, 0, 1]]
        T[:3, 3] = t
        return T

    steps = [("iter", None), ("iter", rot(0.01, [0.001, 0, 0])), ("iter", rot(0.01, [0, 0.001, 0])),
             ("iter", rot(3.0, [0.5, -0.2, 0.1])), ("iter", rot(0.02, [0, 0, 0.001])),
             ("target", tgt2), ("iter", rot(0.01, [0.001, 0, 0])), ("iter", None),
             ("source", src2), ("iter", None), ("iter", rot(0.01, [0, 0, 0.002])), ("iter", rot(-5.0, [1.0, 0, 0]))]

    def run(conf):
        out = []
        with icp.Context(0, conf) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            k = 0
            for kind, arg in steps:
                if kind == "target":
                    ctx.set_target(arg, 10, 20, icp.RULES_ENGINE)
                elif kind == "source":
                    ctx.set_source(arg)
                else:
                    st = ctx.iterate(arg, k, icp.RULES_ENGINE, 3.0)
                    k += 1
                    idx, d = ctx.get_correspondences()
                    out.append((idx.copy(), d.copy(), st.valid))
        return out

    a = run({"candidate_cache": 0})
    b = run({"debug_counters": 0})
    assert len(a) == len(b) == 10
    for (ia, da, va), (ib, db, vb) in zip(a, b):
        np.testing.assert_array_equal(ia, ib)
        np.testing.assert_array_equal(da, db)
        assert va == vb


def test_candidate_cache_reuses(icp):
    """The first iterate (descent guesses, loose boxes) stores nothing; the second stores nearly
    every wave's list; without motion the third reuses every list the second stored (debug
    counters)."""
    tgt, src, _ = icp.synth_pair(500_000)
    with icp.Context(0, {"debug_counters": 1}) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        c0 = ctx.debug_counters()
        ctx.iterate(np.eye(4), 1, icp.RULES_ENGINE, 3.0)
        c1 = ctx.debug_counters()
        ctx.iterate(np.eye(4), 2, icp.RULES_ENGINE, 3.0)
        c2 = ctx.debug_counters()
    assert c0["cache_hits"] == 0 and c0["cache_stores"] == 0
    assert c1["cache_hits"] == 0 and c1["cache_stores"] > 0.9 * c1["waves"]
    assert c2["cache_hits"] > 0.9 * c1["cache_stores"]


def test_scan32_ties_and_self_queries(icp, oracle, golden_nn):
    """Exact ties (lattice, duplicates) and zero distances (queries on target points) under the
    fp32 filter: identical to the reference-order kernel."""
    rng = np.random.default_rng(11)
    for case in ("lattice", "duplicates", "gauss"):
        t = golden_nn[f"{case}_target"]
        q = np.concatenate([t[rng.integers(0, len(t), 3000)], golden_nn[f"{case}_query"]])

        def run():
            with icp.Context(0) as ctx:
                ctx.set_target(t, 10, 20, icp.RULES_CLI)
                ctx.set_source(q)
                ctx.iterate(None, 0, icp.RULES_CLI, 3.0)
                ctx.iterate(np.eye(4), 1, icp.RULES_CLI, 3.0)  # second pass: previous-residual guesses
                return ctx.get_correspondences()

        idx, d = run()
        oidx, od = oracle.OracleTree(t).nn(q, init_best=1e20)
        np.testing.assert_array_equal(idx, oidx)
        np.testing.assert_array_equal(d, od)


def test_wave_repeated_targets(icp, oracle):
    """Every target point stored 2 or 3 times (bench --duplicates): each query's nearest point has
    exact copies, which the wave kernel's fp64 rescan resolves to the lowest slot; identical
    indices and distances to the reference-order search."""
    tgt, src, _ = icp.synth_pair(60_000, yaw_deg=2.0)
    for rep in (2, 3):
        t = np.repeat(tgt[: 60_000 // rep + 1], rep, axis=0)[:60_000]
        with icp.Context(0) as ctx:
            ctx.set_target(t, 10, 20, icp.RULES_CLI)
            ctx.set_source(src)
            ctx.iterate(None, 0, icp.RULES_CLI, 3.0)
            ctx.iterate(np.eye(4), 1, icp.RULES_CLI, 3.0)
            idx, d = ctx.get_correspondences()
        oidx, od = oracle.OracleTree(t).nn(src, init_best=1e20)
        np.testing.assert_array_equal(idx, oidx)
        np.testing.assert_array_equal(d, od)


def test_session_step_n_equals_steps(icp):
    """icp_session_step_n (the bench's timed loop) is the same loop as repeated icp_session_step:
    identical transforms bit for bit; it stops at convergence like the step loop."""
    tgt, src, _ = icp.synth_pair(200_000, yaw_deg=4.0)

    def run(native: bool):
        with icp.Context(0) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            sess = ctx.session(icp.params_default(max_iterations=40, tolerance=1e-9))
            if native:
                taken = sess.step_n(1000)
            else:
                taken = 0
                while not sess.done:
                    sess.step()
                    taken += 1
            return taken, sess.transform().copy()

    na, Ta = run(True)
    nb, Tb = run(False)
    assert na == nb and 0 < na <= 40
    assert np.array_equal(Ta, Tb)


def test_overflowing_waves_take_the_half_pass(icp, oracle):
    """A wave whose search box overflows its candidate list (the first iterate's descent guesses,
    at 1M: ~16 % of the waves) is searched again as two 32-query halves with their own smaller
    boxes (k_nn_half) before anything goes to the ball search; every result stays the reference's."""
    tgt, src, _ = icp.synth_pair(1_000_000)
    with icp.Context(0, {"debug_counters": 1, "overflow_halves": 1}) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        st = ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        c = ctx.debug_counters()
        idx, d = ctx.get_correspondences()
    assert c["overflow_waves"] > 0 and c["halves"] > 0, c
    oidx, od = oracle.OracleTree(tgt).nn(src, init_best=oracle.DBL_MAX)
    np.testing.assert_array_equal(idx, oidx)
    np.testing.assert_array_equal(d, od)
    # the halves took most of the overflowed queries off the ball search
    assert st.n_ball_search < 64 * c["overflow_waves"], (st.n_ball_search, c)


def test_overflowing_waves_take_the_wide_pass(icp, oracle):
    """By default (overflow_halves 0, wide_pass 0) a wave whose box overflows its candidate list
    in the first iterate is searched again by the wide pass (k_nn_wide: the same 64 lanes, the box
    walked and scanned in segments, bounds tightened after each); the results stay the reference's
    and most overflowed queries never reach the ball search."""
    tgt, src, _ = icp.synth_pair(1_000_000)
    with icp.Context(0, {"debug_counters": 1}) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        st = ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        c = ctx.debug_counters()
        idx, d = ctx.get_correspondences()
    assert c["overflow_waves"] > 0 and c["wide_waves"] == c["overflow_waves"] and c["halves"] == 0, c
    oidx, od = oracle.OracleTree(tgt).nn(src, init_best=oracle.DBL_MAX)
    np.testing.assert_array_equal(idx, oidx)
    np.testing.assert_array_equal(d, od)
    assert st.n_ball_search < 16 * c["overflow_waves"], (st.n_ball_search, c)


def test_host_and_device_query_orders(icp, oracle):
    """The source's kd order built on the device (default) or on the host (query_order = 1): the
    first iterate searches the same queries, so identical correspondences and residuals; later
    iterates move the queries by transforms whose statistics were summed in another query order
    (rounding only): transforms within 1e-12, correspondences equal."""
    tgt, src, _ = icp.synth_pair(1_000_000)

    def run(conf):
        out = []
        with icp.Context(0, conf) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            sess = ctx.session(icp.params_default(max_iterations=4, tolerance=0.0))
            for _ in range(4):
                rec = sess.step()
                out.append(ctx.get_correspondences() + (np.array(rec.transform[:]),))
            sess.close()
        return out

    dev, host = run({"query_order": 0}), run({"query_order": 1})
    np.testing.assert_array_equal(dev[0][0], host[0][0])
    np.testing.assert_array_equal(dev[0][1], host[0][1])
    for (ia, da, Ta), (ib, db, Tb) in zip(dev, host):
        np.testing.assert_array_equal(ia, ib)
        np.testing.assert_allclose(da, db, rtol=1e-10)
        np.testing.assert_allclose(Ta, Tb, rtol=0, atol=1e-12)
    oidx, od = oracle.OracleTree(tgt).nn(src, init_best=oracle.DBL_MAX)
    np.testing.assert_array_equal(dev[0][0], oidx)
    np.testing.assert_array_equal(dev[0][1], od)


def test_outlier_first_query_keeps_statistics_precise(icp, oracle):
    """Far outliers (3e10 m) wherever the query order puts them, the first slot included: the
    shifts of the moment and covariance sums come from the bulk of the data (the smallest finite
    residual / the first valid pair of the first 64 queries), not from an outlier, so the
    transform matches the oracle's to 1e-10 (an outlier shift cancelled ~6 digits)."""
    rng = np.random.default_rng(17)
    t = rng.normal(size=(3000, 3)) * [4, 4, 1]
    far = np.array([[-3e10, -3e10, -3e10], [3e10, -2e10, 1e10], [-1e10, 3e10, -2e10], [2e10, 1e10, 3e10]])
    s = np.concatenate([far, t[:1500] + rng.normal(size=(1500, 3)) * 0.01 + [0.05, -0.02, 0.01]])
    p = icp.params_default(max_iterations=6, tolerance=0.0)
    for conf in ({"query_order": 0}, {"query_order": 1}):
        with icp.Context(0, conf) as ctx:
            ctx.set_target(t, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(s)
            rc, res, hist = ctx.run(p)
        orc, ores, ohist, _ = oracle.icp(s, t, oracle.SEM_ENGINE, 6, 0.0)
        oh = [h for h in ohist if h.has_transform]
        assert [h.valid_points for h in hist] == [h.valid for h in oh]
        for h, o in zip(hist, oh):
            np.testing.assert_allclose(np.array(h.transform), np.array(o.T_cum), rtol=0, atol=1e-10)
