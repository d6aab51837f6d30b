"""The device-resident loop (icp_hip_config.device_loop; session_step.h, reduce_kernels.hip
loop_step) against the host loop: each iteration's last kernel takes the session's decisions
(icpengine.cpp:287-346) and computes the transform with the host's own code, so a registration
gives the same records, transforms, moved source and correspondences bit for bit as one stepped
by the host (icp_session_step), whatever the stop that ends it."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _anisotropic(icp, n, yaw_deg=4.0, seed=5):
    """A cloud whose motion is observable (unlike config 4's yaw-symmetric blob)."""
    rng = np.random.default_rng(seed)
    tgt = rng.normal(size=(n, 3)) * np.array([6.0, 2.0, 0.7])
    tgt[:, 2] += 0.3 * np.sin(tgt[:, 0])
    a = np.deg2rad(yaw_deg)
    R = np.array([[np.cos(a), -np.sin(a), 0.0], [np.sin(a), np.cos(a), 0.0], [0.0, 0.0, 1.0]])
    src = (tgt - np.array([0.2, -0.1, 0.05])) @ R + rng.normal(scale=0.002, size=(n, 3))
    return tgt, src


def _rec(h):
    return bytes(memoryview(h))


def _register(icp, loop, tgt, src, params):
    with icp.Context(0, icp.config(device_loop=loop)) as ctx:
        ctx.set_target(tgt, 10, 20, params.rules)
        ctx.set_source(src)
        rc, res, hist = ctx.run(params)
        moved = ctx.get_source()
        idx, d = ctx.get_correspondences()
    return rc, res, [_rec(h) for h in hist], moved, idx, d


@pytest.mark.parametrize("rules,tol", [(0, 1e-4), (1, 1e-4)])
def test_device_loop_registration_equals_host_loop(icp, rules, tol):
    """icp_engine_run to convergence: the engine's converged record (T_cum, NaN angle) or the CLI's
    break, every record, the final transform and the written-back source equal the host loop's."""
    tgt, src = _anisotropic(icp, 200_000)
    params = icp.params_default(max_iterations=100, tolerance=tol, rules=rules)
    a = _register(icp, 1, tgt, src, params)
    b = _register(icp, 0, tgt, src, params)
    assert a[0] == b[0] == 0
    ra, rb = a[1], b[1]
    assert ra.status == rb.status and ra.total_iterations == rb.total_iterations and ra.n_history == rb.n_history
    assert ra.status == 1 and 2 <= ra.total_iterations < 100
    assert bytes(memoryview(ra)) == bytes(memoryview(rb))
    assert a[2] == b[2]
    for k in range(3, 6):
        assert np.array_equal(a[k], b[k])


def test_device_loop_stops_on_divergence_and_max_iterations(icp):
    """A loop enqueued past its end does nothing: max_iterations inside a batch, and a divergence
    stop (a target far from the source: the second iteration's RMSE jumps) leave the same state
    as the host loop."""
    tgt, src = _anisotropic(icp, 50_000)
    params = icp.params_default(max_iterations=7, tolerance=0.0)
    a = _register(icp, 1, tgt, src, params)
    b = _register(icp, 0, tgt, src, params)
    assert a[1].total_iterations == b[1].total_iterations == 7 and a[1].status == 0
    assert a[2] == b[2] and np.array_equal(a[3], b[3])
    far = src + np.array([40.0, 0.0, 0.0])
    far[:1000] -= np.array([40.0, 0.0, 0.0])  # a few queries near the target, the rest far
    params = icp.params_default(max_iterations=30, tolerance=1e-9)
    a = _register(icp, 1, tgt, far, params)
    b = _register(icp, 0, tgt, far, params)
    assert a[0] == b[0] and a[1].status == b[1].status and a[1].total_iterations == b[1].total_iterations
    assert a[2] == b[2] and np.array_equal(a[3], b[3])


def test_device_loop_batches_equal_steps(icp):
    """The bench's loop: icp_session_step_n_timed over 40 iterations (no early stop) in batches of
    7 and 33 equals 40 host steps; the device times are positive."""
    tgt, src, _ = icp.synth_pair(1_000_000, yaw_deg=3.0)
    params = icp.params_default(max_iterations=41, tolerance=1e-6, flags=icp.FLAG_NO_EARLY_STOP)

    def run(loop):
        with icp.Context(0, icp.config(device_loop=loop)) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            sess = ctx.session(params)
            ms = np.concatenate([sess.step_n_timed(7), sess.step_n_timed(33)])
            T = sess.transform().copy()
            idx, d = ctx.get_correspondences()
            rc, res = sess.finish()
            moved = ctx.get_source()
            sess.close()
        return ms, T, idx, d, rc, bytes(memoryview(res)), moved

    a, b = run(1), run(0)
    assert len(a[0]) == len(b[0]) == 40 and np.all(a[0] > 0) and np.all(np.isfinite(a[0]))
    for k in range(1, 7):
        assert np.array_equal(a[k], b[k]) if isinstance(a[k], np.ndarray) else a[k] == b[k]


def test_device_loop_over_rccl_one_rank(icp):
    """The device loop over the RCCL path (ncclAllGather + rank-order merges on the stream, the
    session stepped by k_finalize_cov) equals the plain host loop bit for bit."""
    tgt, src, _ = icp.synth_pair(300_000, yaw_deg=3.0)
    params = icp.params_default(max_iterations=12, tolerance=1e-6, flags=icp.FLAG_NO_EARLY_STOP)

    def run(rccl, loop):
        with icp.Context(0, icp.config(device_loop=loop)) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            if rccl:
                ctx.comm_init(1, 0, icp.Context.unique_id())
            sess = ctx.session(params)
            assert sess.step_n(12) == 12
            T = sess.transform().copy()
            idx, d = ctx.get_correspondences()
            sess.close()
        return T, idx, d

    a, b = run(True, 1), run(False, 0)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_device_loop_hooks_and_cancel(icp):
    """The engine drop-in's hooks: log and progress calls in iteration order. A session with a stop
    flag always steps on the host (the flag is checked before every iteration against the previous
    iteration's hooks, icpengine.cpp:160-164): raised from iteration 3's progress hook, it stops
    the registration after exactly 3 records with the reference's cancellation result."""
    tgt, src = _anisotropic(icp, 100_000)
    logs, prog = [], []
    rc, res, hist, _ = icp.engine_register(icp.params_default(max_iterations=40, tolerance=1e-12), src, tgt,
                                           device=0, on_log=logs.append,
                                           on_progress=lambda it, total, rmse: prog.append(it))
    assert rc == 0 and prog == list(range(1, len(prog) + 1)) and len(prog) == res.n_history
    its = [int(m.split()[1].rstrip(":")) for m in logs if m.startswith("iteration ")]
    assert its == list(range(1, res.total_iterations + 1)) or res.status != 0
    rc, res, hist, out = icp.engine_register(icp.params_default(max_iterations=200, tolerance=0.0), src, tgt,
                                             device=0, stop_at=3)
    assert res.status == 4 and not res.success and res.n_history == 3
    assert np.array_equal(out, np.asarray(src, dtype=np.float64))  # no write-back on cancel
