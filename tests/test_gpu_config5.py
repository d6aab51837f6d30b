"""BASELINE config 5 on one GPU: 50M <-> 50M, octree depth 20 / leaf 10, the fp32 correspondence
path (the fp32 filter scan of k_nn4 with its fp64 certificate).

Checks (size-independent properties plus an oracle sample, since a full CPU reference run at this
size takes minutes per iteration):
  * the device-built octree has the host builder's shape (node/leaf counts, depth);
  * after three real ICP iterations (fused transforms, previous-residual guesses), a random sample
    of 20k correspondences equals the CPU oracle's on the transformed source, bit for bit;
  * the fp32 and fp64 scans give identical correspondences on that iteration;
  * the device statistics equal those of the returned residual array.
"""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

N = 50_000_000


def test_config5_50m(icp, oracle):
    import time
    t0 = time.time()
    tgt, src, _ = icp.synth_pair(N)
    print(f"synthesised in {time.time() - t0:.0f} s", flush=True)
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
