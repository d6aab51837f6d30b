"""One process driving several devices (icp_hip_create_multi; SURVEY.md §8(b) icp_hip_create(ctx,
n_devices, device_ids)): the multi-GPU path behind the single-process drop-in
(ICPEngine::registerPointClouds, icpengine.cpp:24-60; ICP(), icp_registration.cpp:443-446).

The one-GPU box runs it two ways:
  * N members on the same device (the in-process host gather: RCCL refuses two ranks on one
    device), every member with its own driver thread, spatial shard and octree replica: the same
    code path as N GPUs except the transport. Checked against a plain one-device run: every
    iteration's statistics and transform to 1e-12 (merge order only), correspondences bit for bit
    in the caller's order.
  * devices = {0} over RCCL (ncclCommInitAll of one device, ncclAllGather on the member's
    stream, rank-order device merges): bit-identical to the plain run.
And the drop-in entry points with a device list: icp_engine_register_devices, icp_cli_icp_devices,
the CLI's --devices.
"""
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
N = 300_000
ITERS = 5


def _run(icp, ctx, tgt, src):
    ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
    ctx.set_source(src)
    sess = ctx.session(icp.params_default(max_iterations=ITERS, tolerance=0.0))
    recs, corr = [], []
    for _ in range(ITERS):
        r = sess.step()
        recs.append((r.valid_points, r.rmse, r.mean, r.std, r.threshold, np.array(r.transform[:])))
        corr.append(ctx.get_correspondences())
    rc, res = sess.finish()
    sess.close()
    assert rc == 0 and res.success
    return recs, corr, ctx.get_source()


@pytest.fixture(scope="module")
def pair(icp):
    tgt, src, _ = icp.synth_pair(N, yaw_deg=3.0)
    return tgt, src


@pytest.fixture(scope="module")
def plain(icp, pair):
    with icp.Context(0) as ctx:
        return _run(icp, ctx, *pair)


@pytest.mark.parametrize("members", [2, 3, 8])
def test_group_host_gather_matches_plain(icp, pair, plain, members):
    with icp.Context(devices=[0] * members) as ctx:
        ids, transport = ctx.devices()
        assert ids == [0] * members and transport == icp.XPORT_HOST
        recs, corr, moved = _run(icp, ctx, *pair)
        # an iterate's search paths are summed over the members
        st = ctx.iterate(None, ITERS, icp.RULES_ENGINE, 3.0)
        assert st.n == N
    p_recs, p_corr, p_moved = plain
    for (v, rmse, mean, sd, thr, T), (pv, prmse, pmean, psd, pthr, pT) in zip(recs, p_recs):
        assert v == pv
        np.testing.assert_allclose([rmse, mean, sd, thr], [prmse, pmean, psd, pthr], rtol=1e-12)
        np.testing.assert_allclose(T, pT, rtol=0, atol=1e-12)
    # the first iterate searches the unmoved source: identical correspondences and residuals
    np.testing.assert_array_equal(corr[0][0], p_corr[0][0])
    np.testing.assert_array_equal(corr[0][1], p_corr[0][1])
    # later ones searched sources moved by transforms equal to 1e-12: indices equal
    for (idx, _), (pidx, _) in zip(corr, p_corr):
        assert np.count_nonzero(idx != pidx) <= 1e-5 * N
    np.testing.assert_allclose(moved, p_moved, rtol=0, atol=1e-9)


def test_group_rccl_one_device_bit_identical(icp, pair, plain):
    with icp.Context(devices=[0], transport=icp.XPORT_RCCL) as ctx:
        ids, transport = ctx.devices()
        assert ids == [0] and transport == icp.XPORT_RCCL
        recs, corr, moved = _run(icp, ctx, *pair)
    p_recs, p_corr, p_moved = plain
    for a, b in zip(recs, p_recs):
        assert a[:5] == b[:5]
        np.testing.assert_array_equal(a[5], b[5])
    for (idx, d), (pidx, pd) in zip(corr, p_corr):
        np.testing.assert_array_equal(idx, pidx)
        np.testing.assert_array_equal(d, pd)
    np.testing.assert_array_equal(moved, p_moved)


def test_group_argument_errors(icp, pair):
    tgt, src = pair
    with pytest.raises(icp.IcpError):
        icp.Context(devices=[0, 0], transport=icp.XPORT_RCCL)  # RCCL: one rank per GPU
    with icp.Context(devices=[0, 0, 0]) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        with pytest.raises(icp.IcpError):
            ctx.set_source(src[:2])  # fewer points than devices
        with pytest.raises(icp.IcpError):
            ctx.comm_init_host(2, 0, lambda local: np.stack([local, local]))


def test_group_member_failure_host_gather(icp, pair, plain):
    """A member failing before the record exchange (icp_hip_debug_inject_failure) fails the iterate
    with its own error in bounded time (the peers waiting in the host gather give up), harmless
    errors do not poison the group, and the same group then runs a clean registration that equals
    the plain run (the abort flag and the exchange count are reset per job)."""
    import time
    tgt, src = pair
    with icp.Context(devices=[0, 0, 0]) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        with pytest.raises(icp.IcpError) as e:
            ctx.get_correspondences()  # no iterate yet: a harmless error
        assert e.value.code == icp.ENOTREADY
        ctx.inject_failure(member=1)
        t0 = time.perf_counter()
        with pytest.raises(icp.IcpError) as e:
            ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        assert time.perf_counter() - t0 < 30.0
        assert e.value.code == icp.EDEVICE and "injected" in str(e.value)
        recs, corr, moved = _run(icp, ctx, tgt, src)
    p_recs, _, p_moved = plain
    for (v, rmse, *_r), (pv, prmse, *_p) in zip(recs, p_recs):
        assert v == pv
        np.testing.assert_allclose(rmse, prmse, rtol=1e-12)
    np.testing.assert_allclose(moved, p_moved, rtol=0, atol=1e-9)


def test_group_member_failure_rccl_aborts(icp, pair):
    """Over RCCL a failed iterate aborts every member's communicator (ncclCommAbort) and leaves the
    group dead: later calls fail with EDEVICE instead of hanging on a collective a failed peer never
    joined, and destroy returns. One device here (ncclCommInitAll of one rank): the same code path
    as N GPUs."""
    import time
    tgt, src = pair
    ctx = icp.Context(devices=[0], transport=icp.XPORT_RCCL)
    try:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)  # a good iterate first
        ctx.inject_failure(member=0)
        t0 = time.perf_counter()
        with pytest.raises(icp.IcpError) as e:
            ctx.iterate(None, 1, icp.RULES_ENGINE, 3.0)
        assert e.value.code == icp.EDEVICE
        with pytest.raises(icp.IcpError) as e:
            ctx.iterate(None, 2, icp.RULES_ENGINE, 3.0)
        assert e.value.code == icp.EDEVICE and "destroy" in str(e.value)
        assert time.perf_counter() - t0 < 30.0
    finally:
        t0 = time.perf_counter()
        ctx.close()
        assert time.perf_counter() - t0 < 30.0


def test_comm_abort_single_rank(icp, pair):
    """icp_hip_comm_abort on a one-rank RCCL communicator: iterates fail with ERCCL until the next
    comm_init, which restores the bit-identical multi-rank path."""
    tgt, src = pair
    with icp.Context(0) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        ctx.comm_init(1, 0, icp.Context.unique_id())
        a = ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        ctx.comm_abort()
        with pytest.raises(icp.IcpError) as e:
            ctx.iterate(None, 1, icp.RULES_ENGINE, 3.0)
        assert e.value.code == icp.ERCCL
        ctx.comm_init(1, 0, icp.Context.unique_id())
        ctx.set_source(src)
        b = ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
    assert (a.valid, a.rmse) == (b.valid, b.rmse)


def test_engine_and_cli_with_device_lists(icp, pair):
    tgt, src = pair
    p = icp.params_default(max_iterations=20, tolerance=1e-9)
    rc1, res1, hist1, out1 = icp.engine_register(p, src, tgt, devices=[0])
    rc2, res2, hist2, out2 = icp.engine_register(p, src, tgt, devices=[0, 0, 0, 0])
    assert rc1 == 0 and rc2 == 0 and res1.success and res2.success
    assert res1.total_iterations == res2.total_iterations
    assert [h.valid_points for h in hist1] == [h.valid_points for h in hist2]
    np.testing.assert_allclose(np.array(res2.final_R), np.array(res1.final_R), atol=1e-12)
    np.testing.assert_allclose(np.array(res2.final_t), np.array(res1.final_t), atol=1e-12)
    np.testing.assert_allclose(out2, out1, atol=1e-9)
    R1, t1, tr1, s1 = icp.cli_icp(src, tgt, 10, 1e-2, devices=[0])
    R2, t2, tr2, s2 = icp.cli_icp(src, tgt, 10, 1e-2, devices=[0, 0])
    assert len(tr1) == len(tr2)
    np.testing.assert_allclose(R2, R1, atol=1e-12)
    np.testing.assert_allclose(t2, t1, atol=1e-12)


def test_cli_binary_devices_flag(icp, pair, tmp_path):
    tgt, src = pair
    cli = ROOT / "iterativeclosestpoint_amd" / "bin" / "icp_registration"
    if not cli.exists():
        pytest.skip("CLI binary not built")
    icp.las_write_cli(tmp_path / "Scan_096_origin.las", src[:100000])
    icp.las_write_cli(tmp_path / "Scannew_099.las", tgt[:100000])
    outs = {}
    for tag, flag in (("one", ["--device", "0"]), ("two", ["--devices", "0,0"])):
        d = tmp_path / tag
        d.mkdir()
        r = subprocess.run([str(cli), "--source", str(tmp_path / "Scan_096_origin.las"), "--target",
                            str(tmp_path / "Scannew_099.las"), "--sample-rate", "5", "--outdir", str(d)] + flag,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        outs[tag] = (r.stdout, (d / "icp_transformation.txt").read_text())
    assert "devices: 2 GPUs" in outs["two"][0] and "devices:" not in outs["one"][0]
    # same report shape (one block per cumulative transform)
    assert len(outs["one"][1].splitlines()) == len(outs["two"][1].splitlines())


def test_comm_abort_device_loop(icp, pair):
    """After icp_hip_comm_abort, the device-resident loop (config.device_loop = 1) fails with ERCCL
    too, instead of registering on as a world of one with the local shard's statistics."""
    tgt, src = pair
    with icp.Context(0, icp.config(device_loop=1)) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        ctx.comm_init(1, 0, icp.Context.unique_id())
        p = icp.params_default(max_iterations=8, tolerance=0.0, flags=icp.FLAG_NO_EARLY_STOP)
        s = ctx.session(p)
        assert s.step_n(3) == 3
        s.close()
        ctx.comm_abort()
        s = ctx.session(p)
        with pytest.raises(icp.IcpError) as e:
            s.step_n(3)
        assert e.value.code == icp.ERCCL
        s.close()


def test_host_exchange_deadline(icp, pair):
    """A host-exchange peer that stalls past config.peer_timeout_ms: the iterate returns EEXCHANGE
    in bounded time, later iterates fail with ERCCL until comm_init_host, which waits for the
    stalled callback and restores the path; the context then destroys cleanly (icp_hip.h,
    icp_hip_comm_abort's notes)."""
    import time
    tgt, src = pair
    stall = {"s": 0.0}

    def exchange(local):
        if stall["s"] > 0:
            time.sleep(stall["s"])
        return np.stack([local, local])  # a world of two whose peer mirrors this rank

    with icp.Context(0, icp.config(peer_timeout_ms=300)) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        ctx.comm_init_host(2, 0, exchange)
        a = ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        assert a.n == 2 * src.shape[0]
        stall["s"] = 2.0
        t0 = time.perf_counter()
        with pytest.raises(icp.IcpError) as e:
            ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        assert e.value.code == icp.EEXCHANGE and "peer_timeout_ms" in str(e.value)
        assert time.perf_counter() - t0 < 1.5
        with pytest.raises(icp.IcpError) as e:
            ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        assert e.value.code == icp.ERCCL
        stall["s"] = 0.0
        t0 = time.perf_counter()
        ctx.comm_init_host(2, 0, exchange)  # joins the exchange thread once the stalled call returns
        assert time.perf_counter() - t0 < 10.0
        ctx.set_source(src)
        b = ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        assert (a.valid, a.rmse) == (b.valid, b.rmse)
        stall["s"] = 1.0
        with pytest.raises(icp.IcpError):
            ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        t0 = time.perf_counter()
    # destroy waits for the callback still sleeping on the exchange thread
    assert time.perf_counter() - t0 < 10.0


def test_rccl_deadline_aborts_and_recovers(icp):
    """config.peer_timeout_ms over an RCCL communicator: an iterate that outlasts it (a 1 ms
    deadline on an iterate of a 5M source with the reference-order search: tens of ms of device
    time, so the deadline is certain to pass whatever the certified search's speed) is abandoned
    with ncclCommAbort and ERCCL in bounded time; comm_init restores the multi-rank path."""
    import time
    tgt, src, _ = icp.synth_pair(5_000_000)
    with icp.Context(0, icp.config(peer_timeout_ms=1, search=icp.SEARCH_REFERENCE)) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        ctx.synchronize()
        ctx.comm_init(1, 0, icp.Context.unique_id())
        t0 = time.perf_counter()
        with pytest.raises(icp.IcpError) as e:
            ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        assert e.value.code == icp.ERCCL and "peer_timeout_ms" in str(e.value)
        assert time.perf_counter() - t0 < 5.0
        with pytest.raises(icp.IcpError) as e:
            ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        assert e.value.code == icp.ERCCL
        ctx.comm_init(1, 0, icp.Context.unique_id())
    with icp.Context(0, icp.config(peer_timeout_ms=60000)) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        ctx.comm_init(1, 0, icp.Context.unique_id())
        st = ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        assert st.n == src.shape[0]


def test_device_loop_batch_longer_than_deadline(icp):
    """config.peer_timeout_ms bounds ONE iterate, not a device-loop batch: a batch of 80 healthy
    iterates over an RCCL communicator that takes several times the deadline completes (the ring
    records the device publishes restart the deadline)."""
    import time
    tgt, src, _ = icp.synth_pair(5_000_000)
    with icp.Context(0, icp.config(peer_timeout_ms=8, device_loop=1)) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        ctx.synchronize()
        ctx.comm_init(1, 0, icp.Context.unique_id())
        p = icp.params_default(max_iterations=100, tolerance=0.0, flags=icp.FLAG_NO_EARLY_STOP)
        s = ctx.session(p)
        assert s.step_n(2) == 2
        t0 = time.perf_counter()
        assert s.step_n(80) == 80
        wall_ms = (time.perf_counter() - t0) * 1e3
        assert wall_ms > 2 * 8, wall_ms  # the batch really outlasted the per-iterate deadline
        s.close()


def test_comm_info_and_exchange_timings(icp, pair):
    """What a launcher can verify about the exchange: RCCL's own view of the communicator
    (ncclCommCount / ncclCommUserRank / ncclCommCuDevice through icp_hip_comm_info) and the time
    of the two record all-gathers of each timed iterate (icp_hip_exchange_timings)."""
    tgt, src = pair
    with icp.Context(0, icp.config(timing_stride=1)) as ctx:
        assert ctx.comm_info() == {"count": 1, "rank": 0, "device": 0, "transport": icp.XPORT_AUTO}
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        assert np.isnan(ctx.exchange_timings(1)).all()  # no peers: no exchange
        ctx.comm_init(1, 0, icp.Context.unique_id())
        assert ctx.comm_info() == {"count": 1, "rank": 0, "device": 0, "transport": icp.XPORT_RCCL}
        for it in range(3):
            ctx.iterate(None, it, icp.RULES_ENGINE, 3.0)
        x = ctx.exchange_timings(3)
        assert np.isfinite(x).all() and (x > 0).all() and (x < 50).all(), x
        # the host exchange: the callback's world, timed by the host clock
        ctx.comm_init_host(2, 1, lambda local: np.stack([local, local]))
        assert ctx.comm_info() == {"count": 2, "rank": 1, "device": 0, "transport": icp.XPORT_CALLBACK}
        ctx.set_source(src)
        ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        assert np.isfinite(ctx.exchange_timings(1)).all()
    with icp.Context(devices=[0, 0, 0]) as g:  # an in-process group (host gather) of three members
        for m in range(3):
            info = g.comm_info(m)
            assert info["count"] == 3 and info["rank"] == m and info["device"] == 0
        with pytest.raises(icp.IcpError):
            g.comm_info(3)
