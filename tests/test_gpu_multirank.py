"""Multi-rank path on the GPU: W ranks (processes) on one MI355X, all-gathers over the host.

RCCL refuses two ranks on one device, so the one-GPU box cannot run the RCCL transport. What it
can run is everything else of the sharded registration: each rank holds the
full target octree and one spatial source shard (bench.py's `icp_source_shard_order` ranges),
reduces its shard to one Moments and one CovMoments record per iteration, exchanges them
(`icp_hip_comm_init_host`: a gloo all-gather instead of ncclAllGather) and merges them in rank
order on the device (k_finalize_moments / k_finalize_cov) before the host SVD.

Checked against a one-rank run of the whole cloud on the same GPU: every iteration's statistics
and transform (merge order only: 1e-12), bitwise-identical transforms across ranks, and the
shards' correspondences equal to the whole-cloud ones after the first iteration.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
N = 200_000
ITERS = 5

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _records(sess, k):
    out = []
    for _ in range(k):
        r = sess.step()
        out.append((r.valid_points, r.rmse, r.mean, r.std, r.threshold, np.array(r.increment[:])))
    return out


def _worker(rank, world, port, q):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import torch
        import torch.distributed as dist
        import iterativeclosestpoint_amd as icp
        from bench import shard_range

        dist.init_process_group("gloo", rank=rank, world_size=world)
        tgt, src, _ = icp.synth_pair(N, yaw_deg=3.0)
        lo, hi = shard_range(N, rank, world)
        rows = icp.source_shard_order(src)[lo:hi]

        def exchange(local):
            t = torch.from_numpy(local)
            out = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(out, t)
            return torch.stack(out).numpy()

        with icp.Context(0) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src[rows])
            ctx.comm_init_host(world, rank, exchange)
            params = icp.params_default(max_iterations=ITERS + 1, tolerance=1e-6, flags=icp.FLAG_NO_EARLY_STOP)
            sess = ctx.session(params)
            recs = _records(sess, 1)
            idx0, _ = ctx.get_correspondences()
            recs += _records(sess, ITERS - 1)
            sess.close()
        q.put((rank, rows, idx0, recs, None))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, None, None, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_host_exchange_ranks_match_one_rank(icp, world):
    pytest.importorskip("torch")
    import torch.multiprocessing as mp

    ctx_mp = mp.get_context("spawn")
    q = ctx_mp.Queue()
    port = _free_port()
    procs = [ctx_mp.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        results = sorted((q.get(timeout=100) for _ in range(world)), key=lambda r: r[0])
        for p in procs:
            p.join(timeout=30)
    finally:
        # a rank that died without reporting leaves its peers blocked in the gloo all-gather:
        # end every process still alive so none holds the GPU past the test
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    for r in results:
        assert r[4] is None, f"rank {r[0]} failed: {r[4]}"
    assert all(p.exitcode == 0 for p in procs)

    tgt, src, _ = icp.synth_pair(N, yaw_deg=3.0)
    with icp.Context(0) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        params = icp.params_default(max_iterations=ITERS + 1, tolerance=1e-6, flags=icp.FLAG_NO_EARLY_STOP)
        sess = ctx.session(params)
        ref = _records(sess, 1)
        ref_idx0, _ = ctx.get_correspondences()
        ref += _records(sess, ITERS - 1)
        sess.close()

    # every rank holds the same statistics and transform, bit for bit (rank-order merge)
    for _, _, _, recs, _ in results[1:]:
        for a, b in zip(results[0][3], recs):
            assert a[0] == b[0] and a[1:5] == b[1:5] and np.array_equal(a[5], b[5])
    # ... equal to the one-rank run up to the merge order of the partial sums
    for a, b in zip(results[0][3], ref):
        assert a[0] == b[0]
        np.testing.assert_allclose(a[1:5], b[1:5], rtol=1e-12)
        np.testing.assert_allclose(a[5], b[5], atol=1e-12)
    # the shards' first correspondences are the whole cloud's (same queries, no transform yet)
    for _, rows, idx0, _, _ in results:
        assert np.array_equal(idx0, ref_idx0[rows])
    assert sum(len(r[1]) for r in results) == N


def test_rccl_one_rank_communicator_matches_plain(icp):
    """The RCCL transport on the one GPU a box has: a communicator of one rank
    (icp_hip_get_unique_id + icp_hip_comm_init(ctx, 1, 0, id)) makes every iteration run the
    multi-rank path — ncclAllGather of the Moments and CovMoments records on the compute stream,
    the rank-order device merges k_finalize_moments / k_finalize_cov, the publish from
    k_finalize_cov. With one record the rank-order merge is the identity, so every statistic,
    transform and correspondence equals the communicator-free run's bit for bit."""
    tgt, src, _ = icp.synth_pair(N, yaw_deg=3.0)

    def run(rccl: bool):
        with icp.Context(0) as ctx:
            ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
            ctx.set_source(src)
            if rccl:
                ctx.comm_init(1, 0, icp.Context.unique_id())
            params = icp.params_default(max_iterations=ITERS + 1, tolerance=1e-6, flags=icp.FLAG_NO_EARLY_STOP)
            sess = ctx.session(params)
            recs = _records(sess, ITERS)
            idx, d = ctx.get_correspondences()
            T = sess.transform().copy()
            sess.close()
        return recs, idx, d, T

    a, ia, da, Ta = run(True)
    b, ib, db, Tb = run(False)
    for x, y in zip(a, b):
        assert x[:5] == y[:5] and np.array_equal(x[5], y[5])
    assert np.array_equal(Ta, Tb)
    assert np.array_equal(ia, ib) and np.array_equal(da, db)
