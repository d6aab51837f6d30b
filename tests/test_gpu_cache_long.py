"""The bench's timed regime, checked for exactness: a long run of the real engine loop with the
wave search's candidate cache carrying state from iterate to iterate (reuse, loose re-walks,
quarter-margin overflow retries), as bench.py times it.

60 engine iterations (tolerance 0, no early stop) of a 1M <-> 1M synthetic pair. Every 10th
iterate, the state the loop holds (its moved source, correspondences and residuals) must equal
  * a cache-free context (candidate_cache = 0) searching the same moved source, and
  * the CPU oracle's octree NN (octree.cpp:128-184 restated, OpenMP) on it,
bit for bit; and the debug counters must show the cache in use (most waves reuse their list).
"""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

N = 1_000_000
ITERS = 60


def test_candidate_cache_long_run_matches_cache_free_and_oracle(icp, oracle):
    tgt, src, _ = icp.synth_pair(N)
    tree = oracle.OracleTree(tgt)
    oracle.set_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    hit_share, stored, checked = [], [], 0
    with icp.Context(0, {"debug_counters": 1}) as ctx, icp.Context(0, {"candidate_cache": 0}) as free:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        free.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        sess = ctx.session(icp.params_default(max_iterations=ITERS, tolerance=0.0, flags=icp.FLAG_NO_EARLY_STOP))
        for it in range(ITERS):
            rec = sess.step()
            assert rec is not None and rec.valid_points > 0
            c = ctx.debug_counters()
            hit_share.append(c["cache_hits"] / max(1, c["waves"]))
            stored.append(c["cache_stores"])
            if (it + 1) % 10 == 0:
                moved = ctx.get_source()
                idx, d = ctx.get_correspondences()
                free.set_source(moved)
                free.iterate(None, 0, icp.RULES_ENGINE, 3.0)
                fidx, fd = free.get_correspondences()
                np.testing.assert_array_equal(idx, fidx, err_msg=f"iterate {it + 1}: cache vs cache-free")
                np.testing.assert_array_equal(d, fd, err_msg=f"iterate {it + 1}: cache vs cache-free")
                oidx, od = tree.nn(moved, init_best=oracle.DBL_MAX)
                np.testing.assert_array_equal(idx, oidx, err_msg=f"iterate {it + 1}: GPU vs oracle")
                np.testing.assert_array_equal(d, od, err_msg=f"iterate {it + 1}: GPU vs oracle")
                checked += 1
        assert sess.done
        sess.close()
    assert checked == ITERS // 10
    # the cache carried state: after the first iterates most waves reuse their stored list, and
    # re-walks keep happening (the registration keeps moving)
    assert np.mean(hit_share[5:]) > 0.5, hit_share
    assert sum(stored[5:]) > 0
