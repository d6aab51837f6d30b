"""Device octree build (octree_gpu.hip) against the host builder
(octree_build.cpp), which is pinned to the reference's pointer tree by
tests/test_host.py::test_flat_octree_matches_reference_tree (octree.cpp:41-126).

Bar: the resident arrays are identical — every node record (box bits, first, meta, depth) in the
same numbering and every leaf-ordered point with its original index.
"""
import numpy as np
import pytest

from conftest import KAT_CASES

pytestmark = pytest.mark.gpu


def device_tree(icp, ctx, xyz, mp, md):
    ctx.set_target(xyz, mp, md, icp.RULES_ENGINE)
    on_dev, _ = ctx.target_build_info()
    assert on_dev, "expected the device builder"
    return ctx.copy_target()


def assert_same_tree(h, d):
    assert len(h["first"]) == len(d["first"]), (len(h["first"]), len(d["first"]))
    np.testing.assert_array_equal(h["box"].view(np.uint64), d["box"].view(np.uint64))
    np.testing.assert_array_equal(h["first"], d["first"])
    np.testing.assert_array_equal(h["meta"], d["meta"])
    np.testing.assert_array_equal(h["depth"], d["depth"])
    np.testing.assert_array_equal(h["orig"], d["orig"])
    np.testing.assert_array_equal(h["pts"].view(np.uint64), d["pts"].view(np.uint64))
    assert h["n_leaves"] == d["n_leaves"]
    assert h["max_depth"] == d["max_depth"]


@pytest.mark.parametrize("case", KAT_CASES)
@pytest.mark.parametrize("mp,md", [(10, 20), (5, 10), (3, 2), (0, 5), (100, 20), (1, 21), (10, 0), (64, 20)])
def test_device_build_matches_host_kat(icp, gpu_ctx, golden_nn, case, mp, md):
    t = golden_nn[f"{case}_target"]
    assert_same_tree(icp.octree_build(t, mp, md), device_tree(icp, gpu_ctx, t, mp, md))


@pytest.mark.parametrize("name", ["gauss200k", "rounded", "identical", "two", "plane", "huge_leaf"])
def test_device_build_matches_host_shapes(icp, gpu_ctx, name):
    rng = np.random.default_rng(7)
    mp, md = 10, 20
    if name == "gauss200k":
        t = rng.normal(size=(200_000, 3)) * [5, 5, 1]
    elif name == "rounded":  # many exact duplicates and points on split planes
        t = np.round(rng.normal(size=(50_000, 3)), 1)
    elif name == "identical":  # one leaf at max depth holding every point
        t = np.ones((5000, 3)) * 0.25
    elif name == "two":
        t = np.array([[0.0, 0.0, 0.0], [1.0, 2.0, 3.0]])
    elif name == "plane":  # degenerate axis: z constant
        t = np.c_[rng.uniform(-1, 1, size=(30_000, 2)), np.zeros(30_000)]
    else:  # leaf capacity larger than the doubling threshold of the range max
        t = rng.uniform(-3, 3, size=(100_000, 3))
        mp = 300
    assert_same_tree(icp.octree_build(t, mp, md), device_tree(icp, gpu_ctx, t, mp, md))


def test_device_build_10m(icp, gpu_ctx):
    """Config 4's target: identical arrays at full size, and the build time."""
    tgt, _, _ = icp.synth_pair(10_000_000, 1000)
    d = device_tree(icp, gpu_ctx, tgt, 10, 20)
    _, ms = gpu_ctx.target_build_info()
    print(f"device build of 10M points: {ms:.1f} ms (upload included)")
    assert_same_tree(icp.octree_build(tgt, 10, 20), d)


def test_device_build_rejects_non_finite(icp, gpu_ctx):
    t = np.random.default_rng(3).normal(size=(1000, 3))
    t[517, 1] = np.nan
    with pytest.raises(icp.IcpError):
        gpu_ctx.set_target(t, 10, 20, icp.RULES_ENGINE)
    t[517, 1] = np.inf
    with pytest.raises(icp.IcpError):
        gpu_ctx.set_target(t, 10, 20, icp.RULES_ENGINE)


def test_deep_tree_uses_host_builder(icp, gpu_ctx, golden_nn):
    t = golden_nn["duplicates_target"]
    gpu_ctx.set_target(t, 10, 30, icp.RULES_ENGINE)
    on_dev, _ = gpu_ctx.target_build_info()
    assert not on_dev
    assert_same_tree(icp.octree_build(t, 10, 30), gpu_ctx.copy_target())
