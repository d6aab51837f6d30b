"""The fused covariance sums (wave_stats.h): from a source's second iterate on, the wave search
sums the covariance terms of its pairs below a band around the previous threshold and the cull
pass settles only the band and the waves the search left unfinished.

Checked here, every iterate, against the oracle's statistics of the same correspondences
(icpengine.cpp:235-290: moments, 3-sigma cull, centroids, H), and against the full cull pass
(fused_cull = 0); the path taken is asserted (icp_hip_last_cull_path) so a silent fallback to the
full pass cannot pass for the fused one. Tolerances: the north star's 1e-12 relative for the
moments and centroids (the GPU sums in another order), 1e-10 for H; valid counts exact.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def oracle_stats(src_moved, tgt, idx, d, iteration, sigma=3.0):
    n = len(d)
    mean = d.sum() / n
    sd = np.sqrt(((d - mean) ** 2).sum() / n)
    thr = mean + max(sigma * sd, 0.5 * mean) if iteration == 0 else mean + sigma * sd
    v = d <= thr
    a, b = src_moved[v], tgt[idx[v]]
    H = (a - a.mean(0)).T @ (b - b.mean(0))
    return dict(mean=mean, sd=sd, thr=thr, valid=int(v.sum()), rmse=np.sqrt((d[v] ** 2).sum() / v.sum()),
                ca=a.mean(0), cb=b.mean(0), H=H)


def check_stats(st, o):
    assert st.valid == o["valid"]
    np.testing.assert_allclose([st.mean, st.std, st.threshold, st.rmse], [o["mean"], o["sd"], o["thr"], o["rmse"]],
                               rtol=1e-12)
    np.testing.assert_allclose(st.centroid_src, o["ca"], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(st.centroid_tgt, o["cb"], rtol=1e-12, atol=1e-13)
    H = o["H"]
    np.testing.assert_allclose(np.array(st.H).reshape(3, 3), H, rtol=1e-10, atol=1e-10 * np.abs(H).max())


@pytest.mark.parametrize("n,yaw", [(300_000, 3.0), (1_000_000, 1.0)])
def test_fused_cull_every_iterate_vs_oracle(icp, n, yaw):
    tgt, src, _ = icp.synth_pair(n, yaw_deg=yaw)
    with icp.Context(0) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        T = None
        paths = []
        for it in range(6):
            st = ctx.iterate(T, it, icp.RULES_ENGINE, 3.0)
            paths.append(ctx.last_cull_path())
            idx, d = ctx.get_correspondences()
            check_stats(st, oracle_stats(ctx.get_source(), tgt, idx, d, it))
            T = icp.best_fit_from_stats(st)
    # the first iterate of a source has no band; the threshold then moves well inside it
    assert paths[0] == 0 and all(p == 1 for p in paths[2:]), paths


def test_fused_cull_equals_full_pass(icp):
    """fused_cull 1 and 0 on the same trajectory: the same correspondences and valid counts,
    statistics equal to the summation order (so the transforms, and with them the moved queries'
    residuals, may differ in their last bits from the second iterate on)."""
    tgt, src, _ = icp.synth_pair(500_000, yaw_deg=2.0)
    runs = []
    for fused in (1, 0):
        out = []
        with icp.Context(0, icp.config(fused_cull=fused)) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            T = None
            for it in range(5):
                st = ctx.iterate(T, it, icp.RULES_ENGINE, 3.0)
                out.append((ctx.get_correspondences(), st.as_dict(), ctx.last_cull_path()))
                T = icp.best_fit_from_stats(st)
        runs.append(out)
    for k, ((ca, sa, pa), (cb, sb, pb)) in enumerate(zip(*runs)):
        np.testing.assert_array_equal(ca[0], cb[0])
        np.testing.assert_allclose(ca[1], cb[1], rtol=1e-9, atol=1e-15)
        assert sa["valid"] == sb["valid"] and sa["n"] == sb["n"]
        for key in ("mean", "std", "threshold", "rmse"):
            np.testing.assert_allclose(sa[key], sb[key], rtol=1e-12)
        np.testing.assert_allclose(sa["H"], sb["H"], rtol=1e-10, atol=1e-10 * np.abs(sb["H"]).max())
        assert pb == 0 and (k == 0 or pa == 1)


def test_threshold_leaving_the_band_falls_back(icp):
    """A sigma multiplier that jumps between iterates moves the threshold out of the band: that
    iterate's cull is a full pass (path 0) with the oracle's statistics; the next band is set
    around the new threshold (path 1 again)."""
    tgt, src, _ = icp.synth_pair(300_000, yaw_deg=2.0)
    with icp.Context(0) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        T = None
        sigmas = [3.0, 3.0, 3.0, 1.0, 1.0, 1.0]
        paths = []
        for it, sg in enumerate(sigmas):
            st = ctx.iterate(T, it, icp.RULES_ENGINE, sg)
            paths.append(ctx.last_cull_path())
            idx, d = ctx.get_correspondences()
            check_stats(st, oracle_stats(ctx.get_source(), tgt, idx, d, it, sg))
            T = icp.best_fit_from_stats(st)
    assert paths[3] == 0 and paths[5] == 1, paths


@pytest.mark.parametrize("cfg", [{"candidate_cache": 0}, {"certify_prev": 3}, {"scan_groups": 1},
                                 {"candidate_margin": 0}])
def test_fused_sums_do_not_depend_on_the_search_path(icp, cfg):
    """Configurations that settle different queries by different search paths (the wave, the
    ball search, the previous-match certificate) give bit-identical statistics: a wave whose
    queries were not all settled by the wave search is recomputed canonically by the cull."""
    tgt, src, _ = icp.synth_pair(400_000, yaw_deg=2.0)

    def run(conf):
        out = []
        with icp.Context(0, icp.config(**conf) if conf else None) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            T = None
            for it in range(5):
                st = ctx.iterate(T, it, icp.RULES_ENGINE, 3.0)
                out.append((st.as_dict(), ctx.last_cull_path(), st.n_ball_search))
                T = icp.best_fit_from_stats(st)
        return out

    a, b = run({}), run(cfg)
    for (sa, pa, _), (sb, pb, _) in zip(a, b):
        assert pa == pb
        for key in sa:
            if key.startswith("n_"):
                continue  # the search paths' own counts differ by design
            np.testing.assert_array_equal(np.asarray(sa[key]), np.asarray(sb[key]), err_msg=key)


def test_fused_cull_nonfinite_and_ragged(icp):
    """Sources with non-finite points and a last partial wave: the same statistics as the full
    pass (a non-finite residual makes the mean NaN: no valid pairs, no band, full passes)."""
    tgt, src, _ = icp.synth_pair(100_003, yaw_deg=1.0)
    for bad in (False, True):
        s = src.copy()
        if bad:
            s[[5, 777, 100_002]] = np.nan
        res = []
        for fused in (1, 0):
            out = []
            with icp.Context(0, icp.config(fused_cull=fused)) as ctx:
                ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
                ctx.set_source(s)
                T = None
                for it in range(4):
                    st = ctx.iterate(T, it, icp.RULES_ENGINE, 3.0)
                    out.append((st.as_dict(), ctx.last_cull_path()))
                    T = icp.best_fit_from_stats(st) if not bad else None
            res.append(out)
        for (sa, pa), (sb, pb) in zip(*res):
            assert sa["valid"] == sb["valid"] and sa["n_bad"] == sb["n_bad"]
            np.testing.assert_allclose(sa["rmse"], sb["rmse"], rtol=1e-12)
            np.testing.assert_allclose(sa["H"], sb["H"], rtol=1e-10, atol=1e-10 * max(1e-300, np.abs(sb["H"]).max()))
            if bad:
                assert pa == 0  # NaN threshold: never a band


@pytest.mark.parametrize("n", [100_000, 1_000_000])
def test_fused_cull_is_deterministic(icp, n):
    """Two contexts, the same inputs and history: bit-identical statistics every iterate (the
    wave records, the recomputed waves, the band pairs and the folds are fixed-order)."""
    tgt, src, _ = icp.synth_pair(n, yaw_deg=2.0)

    def run():
        out = []
        with icp.Context(0) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            T = None
            for it in range(6):
                st = ctx.iterate(T, it, icp.RULES_ENGINE, 3.0)
                out.append(st.as_dict())
                T = icp.best_fit_from_stats(st)
        return out

    a, b = run(), run()
    for sa, sb in zip(a, b):
        for key in sa:
            np.testing.assert_array_equal(np.asarray(sa[key]), np.asarray(sb[key]), err_msg=key)


def test_fused_cull_path_in_a_device_group(icp):
    """The multi-rank path (members of an in-process group, host gather): each member decides the
    band and the pair shift in k_finalize_moments; the cull is still the fused one (path 1) from the
    second iterate on, with the single-context statistics to the merge order."""
    tgt, src, _ = icp.synth_pair(300_000, yaw_deg=2.0)
    runs = []
    for devices in (None, [0, 0]):
        out = []
        ctx = icp.Context(0) if devices is None else icp.Context(devices=devices, transport=icp.XPORT_HOST)
        with ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            T = None
            for it in range(5):
                st = ctx.iterate(T, it, icp.RULES_ENGINE, 3.0)
                out.append((st.as_dict(), ctx.last_cull_path()))
                T = icp.best_fit_from_stats(st)
        runs.append(out)
    for k, ((sa, pa), (sb, pb)) in enumerate(zip(*runs)):
        assert sa["valid"] == sb["valid"]
        np.testing.assert_allclose(sb["rmse"], sa["rmse"], rtol=1e-12)
        np.testing.assert_allclose(sb["H"], sa["H"], rtol=1e-10, atol=1e-10 * np.abs(sa["H"]).max())
        if k >= 2:
            assert pa == 1 and pb == 1, (k, pa, pb)


def _session_records(icp, tgt, src, iters, **cfg):
    with icp.Context(0, icp.config(**cfg)) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        rc, res, hist = ctx.run(icp.params_default(max_iterations=iters, tolerance=0.0, flags=icp.FLAG_NO_EARLY_STOP))
        assert rc == 0
        return [(h.valid_points, h.rmse, h.mean, h.std, h.threshold, tuple(h.transform)) for h in hist]


def test_fused_cull_in_the_device_loop(icp):
    """The device-resident loop takes the fused cull too (its last level is k_merge_cov_last, the
    fused launch's fold order): its records equal the host loop's bit for bit, and the full pass
    (fused_cull 0) to the summation order."""
    tgt, src, _ = icp.synth_pair(400_000, yaw_deg=2.0)
    host = _session_records(icp, tgt, src, 8, device_loop=0)
    dev = _session_records(icp, tgt, src, 8, device_loop=1)
    full = _session_records(icp, tgt, src, 8, device_loop=1, fused_cull=0)
    assert host == dev
    for (va, ra, *_), (vb, rb, *_) in zip(dev, full):
        assert va == vb
        np.testing.assert_allclose(ra, rb, rtol=1e-12)


def test_fused_tail_handoff_repeated(icp):
    """The fused last levels hand their blocks' parts to the last-arriving block with relaxed
    agent-scope atomics and write-through stores (reduce_kernels.hip publish_part_last). A stale
    part would change a record: 60 iterates on a 2M source (489 moment parts, fused; its cull
    blocks fused), run twice, give the same records bit for bit, and the device loop (the cull's
    separate last-level launch) gives them too."""
    tgt, src, _ = icp.synth_pair(2_000_000, yaw_deg=2.0)
    a = _session_records(icp, tgt, src, 60)
    b = _session_records(icp, tgt, src, 60)
    c = _session_records(icp, tgt, src, 60, device_loop=1)
    assert len(a) == 60 and a == b and a == c
