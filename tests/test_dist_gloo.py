"""Multi-rank path on CPU (world_size 2, gloo): the exchange step of the sharded registration.

Shards are what the product uses: contiguous ranges of the source's kd order
(icp_source_shard_order, include/icp_host.h; bench.py and icp_group.cpp), spatially compact.
On the GPU each rank reduces its shard to one Moments and one CovMoments record, all-gathers
them over RCCL and merges them in rank order on the device. Here the same records are built by
the product's host functions from each rank's shard (residuals from the CPU oracle, the test
checker), all-gathered over gloo, merged with the product's rank-order merge, and the resulting
threshold / best-fit transform is compared with the single-process whole-cloud computation
(and across ranks, bit for bit).
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stats_from(icp, mom, cov):
    st = icp._lib.IterStats()
    st.n = int(mom[0])
    st.mean = mom[1]
    st.valid = int(cov[0])
    st.centroid_src[:] = list(cov[2:5])
    st.centroid_tgt[:] = list(cov[5:8])
    st.H[:] = list(cov[8:17])
    return st


def _worker(rank, world, port, n, q):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import iterativeclosestpoint_amd as icp
    import oracle_py
    from bench import shard_range

    dist.init_process_group("gloo", rank=rank, world_size=world)
    tgt, src, _ = icp.synth_pair(n, yaw_deg=3.0)
    # the product's sharding (bench.py, icp_group.cpp): rank r takes a contiguous range of the
    # kd order of the source (icp_source_shard_order), a spatially compact shard
    lo, hi = shard_range(n, rank, world)
    shard = src[icp.source_shard_order(src)[lo:hi]]
    idx, d = oracle_py.OracleTree(tgt).nn(shard, init_best=oracle_py.DBL_MAX)

    def gather(vec):
        t = torch.tensor(vec, dtype=torch.float64)
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return np.stack([o.numpy() for o in out])  # rank order

    mom = icp.moments_merge(gather(icp.moments_from_values(d)))
    sd = np.sqrt(mom[2] / mom[0])
    thr = icp.cull_threshold(mom[1], sd, 3.0, 0, 1)
    cov = icp.cov_merge(gather(icp.cov_from_pairs(shard, tgt[idx], d, thr)))
    T = icp.best_fit_from_stats(_stats_from(icp, mom, cov))
    allT = gather(T.reshape(16))
    q.put((rank, mom, thr, cov, T, bool(np.all(allT == allT[0]))))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_exchange_matches_single_process(icp, oracle, world):
    import torch.multiprocessing as mp
    n = 20000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # whole-cloud reference
    tgt, src, _ = icp.synth_pair(n, yaw_deg=3.0)
    idx, d = oracle.OracleTree(tgt).nn(src, init_best=oracle.DBL_MAX)
    mean = d.sum() / n
    sd = np.sqrt(((d - mean) ** 2).sum() / n)
    thr = mean + max(3.0 * sd, 0.5 * mean)
    v = d <= thr
    T_ref = oracle.best_fit(src[v], tgt[idx[v]])
    for rank, mom, thr_r, cov, T, same in results:
        assert same, "ranks disagree on T"
        assert mom[0] == n and cov[0] == v.sum()
        np.testing.assert_allclose(thr_r, thr, rtol=1e-13)
        np.testing.assert_allclose(T, T_ref, atol=1e-12)
    # bitwise identical across ranks
    assert all(np.array_equal(results[0][4], r[4]) for r in results)


def test_kd_shards_are_spatially_compact(icp):
    """The kd-order shards partition the source, and each rank's shard is spatially compact:
    the shards' bounding boxes are far smaller than the cloud's (contiguous ranges of the shuffled
    cloud would each span all of it)."""
    sys.path.insert(0, str(ROOT))
    from bench import shard_range
    n, world = 20000, 4
    _, src, _ = icp.synth_pair(n, yaw_deg=3.0)
    order = icp.source_shard_order(src)
    assert np.array_equal(np.sort(order), np.arange(n))
    vol = lambda a: float(np.prod(a.max(0) - a.min(0)))
    for r in range(world):
        lo, hi = shard_range(n, r, world)
        assert vol(src[order[lo:hi]]) < 0.6 * vol(src)
        assert vol(src[lo:hi]) > 0.8 * vol(src)


def test_shard_range_partitions():
    sys.path.insert(0, str(ROOT))
    from bench import shard_range
    for n in (0, 1, 7, 10_000_000):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[k][1] == spans[k + 1][0] for k in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
