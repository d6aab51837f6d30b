"""The previous-match certificate (icp_hip_config.certify_prev).

After an iterate on the same queries, a query's previous match p* is kept without a search when
p*'s separation S (a lower bound of p*'s distance to every other target point, computed once per
target by k_target_sep) and the moved query's exact fl(d2) u to p* satisfy the reference's window
certificate with the lower bound (S - sqrt(u))^2. Checked here:
  * the separations are lower bounds of the true nearest-other distances, and tight (scipy KD
    tree on the CPU), 0 exactly where a point has a duplicate;
  * every mode (1: whole waves skip, 2: certified lanes settle and the rest of the wave
    searches, 3: the rest go to the ball search) returns exactly the correspondences and
    residuals of certify_prev = 0, iterate after iterate of the real loop, and the CPU oracle's;
  * exact ties, lattices and duplicated targets (no certificate may hide a tie).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_separation_is_a_tight_lower_bound(icp):
    from scipy.spatial import cKDTree

    tgt, _, _ = icp.synth_pair(200_000)
    tgt = np.concatenate([tgt, tgt[:50]])  # 50 exact duplicates: separation 0
    with icp.Context(0, {"certify_prev": 3}) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        sep = ctx.target_separation().astype(np.float64)
    d, _ = cKDTree(tgt).query(tgt, k=2)
    true = d[:, 1]
    assert np.all(sep <= true)
    dup = true == 0
    assert dup.sum() == 100 and np.all(sep[dup] == 0)
    np.testing.assert_allclose(sep[~dup], true[~dup], rtol=1e-6)


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_modes_equal_full_search_over_iterations(icp, oracle, mode):
    # a registration near convergence: an anisotropic cloud (spacing ~5 cm) moved by a few mm with
    # 0.5 mm noise, so residuals stay far below the point spacing and most previous matches
    # certify (config 4's yaw-symmetric pair keeps sliding by ~cm: ~0.2 % do)
    tgt, src, _ = icp.synth_pair(1_000_000, sigma=[8.0, 4.0, 1.5], yaw_deg=0.02, pitch_deg=0.0, roll_deg=0.0,
                                 t=[0.002, -0.001, 0.0005], noise_sigma=0.0005)

    def run(conf):
        out, settled = [], []
        with icp.Context(0, conf) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            sess = ctx.session(icp.params_default(max_iterations=8, tolerance=0.0))
            for _ in range(8):
                sess.step()
                idx, d = ctx.get_correspondences()
                out.append((idx, d))
                settled.append(ctx.debug_counters().get("prev_cert_lanes", 0))
            moved = ctx.get_source()
            sess.close()
        return out, settled, moved

    base, _, moved = run({"certify_prev": 0})
    got, settled, moved2 = run({"certify_prev": mode, "debug_counters": 1})
    for k, ((ia, da), (ib, db)) in enumerate(zip(base, got)):
        np.testing.assert_array_equal(ia, ib, err_msg=f"iterate {k}")
        np.testing.assert_array_equal(da, db, err_msg=f"iterate {k}")
    np.testing.assert_array_equal(moved, moved2)
    # the certificate does the work once previous matches exist
    assert max(settled[2:]) > 0.5 * len(src), settled
    # the source as the last iterate searched it (the session's pending transform is not applied)
    oidx, od = oracle.OracleTree(tgt).nn(moved2, init_best=oracle.DBL_MAX)
    np.testing.assert_array_equal(got[-1][0], oidx)
    np.testing.assert_array_equal(got[-1][1], od)


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_modes_on_ties_lattices_duplicates(icp, oracle, golden_nn, mode):
    rng = np.random.default_rng(12)
    for case in ("lattice", "duplicates", "gauss", "far"):
        t = golden_nn[f"{case}_target"]
        q = np.concatenate([t[rng.integers(0, len(t), 3000)], golden_nn[f"{case}_query"]])
        for rules, init in ((icp.RULES_CLI, 1e20), (icp.RULES_ENGINE, oracle.DBL_MAX)):
            with icp.Context(0, {"certify_prev": mode}) as ctx:
                ctx.set_target(t, 10, 20, rules)
                ctx.set_source(q)
                ctx.iterate(None, 0, rules, 3.0)
                ctx.iterate(np.eye(4), 1, rules, 3.0)  # the previous matches are now certified
                idx, d = ctx.get_correspondences()
            oidx, od = oracle.OracleTree(t).nn(q, init_best=init)
            np.testing.assert_array_equal(idx, oidx, err_msg=case)
            np.testing.assert_array_equal(d, od, err_msg=case)


@pytest.mark.parametrize("mode", [2, 3])
def test_modes_repeated_targets_and_motion(icp, oracle, mode):
    """Duplicated targets (separation 0: never certified) and a large motion between iterates (the
    previous matches are far off: the certificate must fail, not mislead)."""
    tgt, src, _ = icp.synth_pair(60_000, yaw_deg=2.0)
    t = np.repeat(tgt[: 60_000 // 2 + 1], 2, axis=0)[:60_000]
    c, s_ = np.cos(np.radians(8.0)), np.sin(np.radians(8.0))
    big = np.eye(4)
    big[:3, :3] = [[c, -s_, 0], [s_, c, 0], [0, 0, 1]]
    big[:3, 3] = [0.7, -0.2, 0.05]
    for target in (t, tgt):
        with icp.Context(0, {"certify_prev": mode}) as ctx:
            ctx.set_target(target, 10, 20, icp.RULES_CLI)
            ctx.set_source(src)
            ctx.iterate(None, 0, icp.RULES_CLI, 3.0)
            ctx.iterate(big, 1, icp.RULES_CLI, 3.0)
            idx, d = ctx.get_correspondences()
            moved = ctx.get_source()
        oidx, od = oracle.OracleTree(target).nn(moved, init_best=1e20)
        np.testing.assert_array_equal(idx, oidx)
        np.testing.assert_array_equal(d, od)
