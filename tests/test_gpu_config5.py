"""BASELINE config 5 on one GPU: 50M <-> 50M, octree depth 20 / leaf 10, the fp32 correspondence
path (the fp32 filter scan of k_nn_wave with its fp64 certificate).

  * the device-built octree has the host builder's shape (node/leaf counts, depth);
  * the transform: 3 engine iterations (tolerance 0) of the whole 50M <-> 50M pair on the GPU and
    on the CPU oracle (OpenMP NN loop; icpengine.cpp:117-394 restated, pinned to the real core
    engine by tests/golden/engine_rules.npz): equal valid counts per iteration, cumulative
    transforms within 1e-9, final transform RMSE <= 1e-6 (north star);
  * after three real ICP iterations (fused transforms, previous-residual guesses), a random sample
    of 20k correspondences equals the CPU oracle's on the transformed source, bit for bit;
  * the fp32 and fp64 scans give identical correspondences on that iteration;
  * the device statistics equal those of the returned residual array.
"""
import os
import time

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

N = 50_000_000


@pytest.fixture(scope="module")
def pair50(icp):
    t0 = time.time()
    tgt, src, _ = icp.synth_pair(N)
    print(f"synthesised in {time.time() - t0:.0f} s", flush=True)
    return tgt, src


def test_config5_transform_vs_oracle(icp, oracle, pair50):
    tgt, src = pair50
    t0 = time.time()
    with icp.Context(0) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        p = icp.params_default(max_iterations=3, tolerance=0.0)
        rc, res, hist = ctx.run(p)
    assert rc == 0 and res.success and res.total_iterations == 3
    print(f"GPU registration done at {time.time() - t0:.0f} s", flush=True)
    oracle.set_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    orc, ores, ohist, _ = oracle.icp(src, tgt, oracle.SEM_ENGINE, 3, 0.0)
    print(f"oracle registration done at {time.time() - t0:.0f} s", flush=True)
    assert orc == 0 and ores.total_iterations == 3
    oh = [h for h in ohist if h.has_transform]
    assert [h.valid_points for h in hist] == [h.valid for h in oh]
    for h, o in zip(hist, oh):
        np.testing.assert_allclose(h.rmse, o.rmse, rtol=1e-9)
        np.testing.assert_allclose(np.array(h.transform), np.array(o.T_cum), atol=1e-9)
    T = np.eye(4)
    T[:3, :3] = np.array(res.final_R).reshape(3, 3)
    T[:3, 3] = res.final_t
    To = np.eye(4)
    To[:3, :3] = np.array(ores.final_R).reshape(3, 3)
    To[:3, 3] = ores.final_t
    rmse = float(np.sqrt(np.mean((T - To) ** 2)))
    print(f"config 5 final transform RMSE vs CPU oracle: {rmse:.3e}", flush=True)
    assert rmse <= 1e-6
    np.testing.assert_allclose(T, To, atol=1e-9)
    np.testing.assert_allclose(res.final_rmse, ores.final_rmse, rtol=1e-9)


def test_config5_50m(icp, oracle, pair50):
    tgt, src = pair50
    t0 = time.time()
    with icp.Context(0) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        on_dev, ms = ctx.target_build_info()
        assert on_dev
        info = ctx.target_info()
        print(f"50M device octree: {info['n_nodes']} nodes, {info['n_leaves']} leaves, {ms:.0f} ms")
        ctx.set_source(src)
        print(f"source set at {time.time() - t0:.0f} s", flush=True)
        T = None
        for it in range(3):
            st = ctx.iterate(T, it, icp.RULES_ENGINE, 3.0)
            T = icp.best_fit_from_stats(st)
        st = ctx.iterate(T, 3, icp.RULES_ENGINE, 3.0)
        idx, d = ctx.get_correspondences()
        moved = ctx.get_source()
    mean = d.mean()
    np.testing.assert_allclose([st.mean, st.std], [mean, np.sqrt(((d - mean) ** 2).mean())], rtol=1e-11)
    print(f"iterations done at {time.time() - t0:.0f} s", flush=True)
    rng = np.random.default_rng(5)
    sample = rng.choice(N, 20000, replace=False)
    oidx, od = oracle.OracleTree(tgt).nn(moved[sample], init_best=oracle.DBL_MAX)
    np.testing.assert_array_equal(idx[sample], oidx)
    np.testing.assert_array_equal(d[sample], od)
    print(f"oracle sample checked at {time.time() - t0:.0f} s", flush=True)

    # the same iteration with the fp64 scan: identical correspondences
    with icp.Context(0, {"scan32": 0}) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(moved)
        ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
        idx64, d64 = ctx.get_correspondences()
    np.testing.assert_array_equal(idx64, idx)
    np.testing.assert_array_equal(d64, d)
