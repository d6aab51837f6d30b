"""CPU tests of the product's host code (libicp_hip.so host exports; no GPU calls).

The linear octree the device walks is checked node-for-node against the oracle's pointer
octree (same boxes, same leaves, same point order); the 3x3 SVD against Eigen's JacobiSVD
fixtures; the rank merges of the multi-GPU exchange against whole-array statistics.
"""
import numpy as np
import pytest

from conftest import KAT_CASES, fnv1a


def canonical_preorder(flat):
    """Walk the flat arrays root-first, children in ascending octant order (as the oracle dumps)."""
    box, first, meta, depth = flat["box"], flat["first"], flat["meta"], flat["depth"]
    rows, leaf_idx = [], []
    stack = [(0, -1)]
    while stack:
        k, oct_ = stack.pop()
        leaf = bool(meta[k] & 0x80000000)
        cnt = int(meta[k] & 0x7FFFFFFF) if leaf else 0
        # flat box is lo[3], hi[3]; the oracle dump is min_x,max_x,min_y,max_y,min_z,max_z
        b = box[k]
        rows.append((int(depth[k]), oct_, (b[0], b[3], b[1], b[4], b[2], b[5]), int(leaf), cnt))
        if leaf:
            leaf_idx.extend(flat["orig"][first[k]:first[k] + cnt].tolist())
        else:
            mask = int(meta[k] & 0xFF)
            kids = []
            slot = 0
            for o in range(8):
                if mask >> o & 1:
                    kids.append((int(first[k]) + slot, o))
                    slot += 1
            stack.extend(reversed(kids))
    return rows, np.array(leaf_idx, np.int32)


@pytest.mark.parametrize("case", KAT_CASES)
def test_flat_octree_matches_reference_tree(icp, oracle, golden_nn, case):
    t = golden_nn[f"{case}_target"]
    flat = icp.octree_build(t, 10, 20)
    ref = oracle.OracleTree(t, 10, 20).dump()
    rows, leaf_idx = canonical_preorder(flat)
    assert len(rows) == len(ref["depth"])
    np.testing.assert_array_equal([r[0] for r in rows], ref["depth"])
    np.testing.assert_array_equal([r[1] for r in rows], ref["octant"])
    np.testing.assert_array_equal(np.array([r[2] for r in rows]), ref["box"])  # bit-exact boxes
    np.testing.assert_array_equal([r[3] for r in rows], ref["is_leaf"])
    np.testing.assert_array_equal([r[4] for r in rows], ref["npts"])
    np.testing.assert_array_equal(leaf_idx, ref["leaf_idx"])
    # leaf-ordered coordinates are the caller's points
    np.testing.assert_array_equal(flat["pts"], t[flat["orig"]])
    assert flat["orig"][flat["pos_of_orig0"]] == 0


@pytest.mark.parametrize("mp,md", [(5, 10), (100, 50), (10, 3), (1, 20)])
def test_flat_octree_params(icp, oracle, golden_nn, mp, md):
    t = golden_nn["gauss_target"]
    flat = icp.octree_build(t, mp, md)
    ref = oracle.OracleTree(t, mp, md).dump()
    rows, leaf_idx = canonical_preorder(flat)
    np.testing.assert_array_equal(np.array([r[2] for r in rows]), ref["box"])
    np.testing.assert_array_equal(leaf_idx, ref["leaf_idx"])
    assert flat["max_depth"] == ref["depth"].max()


def test_octree_rejects_non_finite(icp):
    t = np.random.default_rng(0).normal(size=(100, 3))
    t[5, 1] = np.nan
    with pytest.raises(icp.IcpError):
        icp.octree_build(t)


def test_host_svd_matches_eigen(icp, golden_svd):
    for k, H in enumerate(golden_svd["H"]):
        U, S, V = icp.jacobi_svd3(H)
        np.testing.assert_array_equal(U, golden_svd["U_fixed"][k])
        np.testing.assert_array_equal(S, golden_svd["S_fixed"][k])
        np.testing.assert_array_equal(V, golden_svd["V_fixed"][k])
        np.testing.assert_allclose(U @ np.diag(S) @ V.T, H, atol=1e-12 * max(1.0, np.abs(H).max()))


def test_host_best_fit_matches_reference(icp, golden_svd):
    for k in range(len(golden_svd["T_bestfit"])):
        T = icp.best_fit_transform(golden_svd[f"bf_A{k}"], golden_svd[f"bf_B{k}"])
        np.testing.assert_allclose(T, golden_svd["T_bestfit"][k], rtol=0, atol=1e-12)


def test_host_mat4_matches_eigen(icp, golden_svd):
    import ctypes as C
    A, B = golden_svd["T"].copy(), golden_svd["T2"].copy()
    out = np.empty(16)
    icp.lib().icp_mat4_mul(A.ctypes.data_as(C.c_void_p), B.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p))
    np.testing.assert_array_equal(out.reshape(4, 4), golden_svd["T_T2"])


def test_synth_deterministic(icp, golden_meta):
    m = golden_meta["nn_100k"]
    tgt, src, T = icp.synth_pair(m["n"])
    assert fnv1a(tgt) == m["target_fnv1a"]
    assert fnv1a(src) == m["source_fnv1a"]
    # ground truth maps the (non-outlier) source onto the target up to the noise
    tgt2, src2, T2 = icp.synth_pair(2000, outlier_fraction=0.0, noise_sigma=0.0)
    mapped = src2 @ T2[:3, :3].T + T2[:3, 3]
    d = np.min(np.linalg.norm(mapped[:200, None, :] - tgt2[None, :, :], axis=2), axis=1)
    assert d.max() < 1e-9


def test_moments_merge_equals_whole(icp):
    rng = np.random.default_rng(3)
    d = np.abs(rng.normal(size=100001)) * 0.3 + 1e3  # large offset: tests the centered merge
    whole = icp.moments_from_values(d)
    parts = [icp.moments_from_values(c) for c in np.array_split(d, 7)]
    merged = icp.moments_merge(np.array(parts))
    assert merged[0] == len(d)
    np.testing.assert_allclose(merged[1], d.mean(), rtol=1e-15)
    np.testing.assert_allclose(merged[2], whole[2], rtol=1e-9)
    np.testing.assert_allclose(merged[2], ((d - d.mean()) ** 2).sum(), rtol=1e-9)
    assert merged[3] == d.min() and merged[4] == d.max()


def test_cov_merge_equals_whole(icp):
    rng = np.random.default_rng(4)
    a = rng.normal(size=(50000, 3)) * [5, 5, 1] + [4e5, 5e6, 100]  # LAS-like offsets
    b = a + rng.normal(size=a.shape) * 0.01
    d = np.linalg.norm(a - b, axis=1)
    thr = np.quantile(d, 0.9)
    whole = icp.cov_from_pairs(a, b, d, thr)
    parts = [icp.cov_from_pairs(a[s], b[s], d[s], thr) for s in np.array_split(np.arange(len(d)), 5)]
    merged = icp.cov_merge(np.array(parts))
    v = d <= thr
    av, bv = a[v], b[v]
    H = (av - av.mean(0)).T @ (bv - bv.mean(0))
    assert merged[0] == v.sum()
    np.testing.assert_allclose(merged[2:5], av.mean(0), rtol=1e-13)
    np.testing.assert_allclose(merged[8:17].reshape(3, 3), H, rtol=1e-9, atol=1e-9 * np.abs(H).max())
    np.testing.assert_allclose(merged[8:17], whole[8:17], rtol=1e-9, atol=1e-9 * np.abs(H).max())


def test_threshold_rules(icp):
    # engine iteration 0: mean + max(k*std, mean/2) (icpengine.cpp:250-252)
    assert icp.cull_threshold(2.0, 0.1, 3.0, 0, 1) == 2.0 + 1.0
    assert icp.cull_threshold(2.0, 0.5, 3.0, 0, 1) == 2.0 + 1.5
    assert icp.cull_threshold(2.0, 0.1, 3.0, 1, 1) == 2.0 + 3.0 * 0.1
    # CLI: always mean + 3 std (icp_registration.cpp:523)
    assert icp.cull_threshold(2.0, 0.1, 3.0, 0, 0) == 2.0 + 3.0 * 0.1


def test_params_default_mirror_reference(icp):
    p = icp.params_default()
    assert (p.max_iterations, p.tolerance, p.sigma_multiplier, p.octree_max_points, p.octree_max_depth) == \
        (50, 1e-6, 3.0, 10, 20)  # ICPParameters, icpengine.h:13-19


def test_source_shard_order_is_a_spatial_permutation(icp):
    """Contiguous ranges of icp_source_shard_order are spatially compact: 8 shards of a shuffled
    cloud cover far less volume each than 8 plain ranges (which span the whole cloud)."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from bench import shard_range
    _, src, _ = icp.synth_pair(200_000)
    order = icp.source_shard_order(src)
    assert order.dtype == np.int32 and np.array_equal(np.sort(order), np.arange(len(src)))
    vol_kd, vol_plain = 0.0, 0.0
    for r in range(8):
        lo, hi = shard_range(len(src), r, 8)
        a, b = src[order[lo:hi]], src[lo:hi]
        a, b = a[np.all(np.abs(a) < 30, 1)], b[np.all(np.abs(b) < 30, 1)]  # outliers aside
        vol_kd += np.prod(np.percentile(a, 95, 0) - np.percentile(a, 5, 0))
        vol_plain += np.prod(np.percentile(b, 95, 0) - np.percentile(b, 5, 0))
    assert vol_kd < 0.4 * vol_plain


def test_synth_outlier_fraction_is_validated(icp):
    """outlier_fraction outside [0, 1] (or NaN) is refused; 1.0 makes every source point an outlier
    (no undefined float -> uint64 cast of 2^64)."""
    for f in (-0.1, 1.5, float("nan")):
        with pytest.raises(icp.IcpError):
            icp.synth_pair(100, outlier_fraction=f)
        with pytest.raises(icp.IcpError):
            icp.synth_scene(100, outlier_fraction=f)
    tgt, src, _ = icp.synth_pair(500, outlier_fraction=1.0, noise_sigma=0.0)
    lo, hi = tgt.min(axis=0), tgt.max(axis=0)
    assert np.all((src >= lo) & (src <= hi))
    _, src0, _ = icp.synth_pair(500, outlier_fraction=0.0, noise_sigma=0.0)
    assert not np.any(np.all(src == src0, axis=1))  # no point kept its inlier position
    tgt_s, src_s, _ = icp.synth_scene(500, outlier_fraction=1.0)
    assert np.isfinite(src_s).all()
