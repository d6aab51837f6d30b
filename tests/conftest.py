import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP path")


@pytest.fixture(scope="session")
def golden_nn():
    return np.load(GOLDEN / "nn_known_answers.npz")


@pytest.fixture(scope="session")
def golden_svd():
    return np.load(GOLDEN / "svd_transform.npz")


@pytest.fixture(scope="session")
def golden_icp():
    return np.load(GOLDEN / "icp_cli.npz")


@pytest.fixture(scope="session")
def golden_engine():
    """Engine-rule cases run by the real core engine (gen_golden.py engine_cases)."""
    return np.load(GOLDEN / "engine_rules.npz")


@pytest.fixture(scope="session")
def golden_scene():
    """A LiDAR-like surface pair run through the reference (gen_golden.py scene_cases)."""
    return np.load(GOLDEN / "scene_ref.npz")


@pytest.fixture(scope="session")
def golden_core_las():
    return np.load(GOLDEN / "core_las.npz")


@pytest.fixture(scope="session")
def golden_meta():
    import json
    return json.loads((GOLDEN / "golden.json").read_text())


@pytest.fixture(scope="session")
def icp():
    import iterativeclosestpoint_amd as m
    if not m.LIB_PATH.exists():
        m.build()
    m.lib()
    return m


@pytest.fixture(scope="session")
def oracle():
    import oracle_py
    if not oracle_py.ORACLE_LIB.exists():
        oracle_py.build(ref=False)
    oracle_py.oracle()
    return oracle_py


@pytest.fixture(scope="session")
def gpu_ctx(icp):
    """One context on device 0 shared by the GPU tests (one process, as gpurun requires)."""
    ctx = icp.Context(0)
    yield ctx
    ctx.close()


def fnv1a(a: np.ndarray) -> str:
    h = 0xCBF29CE484222325
    for b in np.ascontiguousarray(a).tobytes():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


KAT_CASES = ["gauss", "lattice", "duplicates", "far", "single", "root_leaf"]
ENGINE_CASES = ["e1k", "e10k", "far", "relaxed", "params", "diverge", "too_few", "cancel"]


def t_rmse(a, b):
    """sqrt(mean((A - B)^2)) over the 16 entries: the north star's transform metric."""
    return float(np.sqrt(np.mean((np.asarray(a) - np.asarray(b)) ** 2)))


def engine_expected(golden_engine, golden_meta, name):
    """One engine-rule case as the reference engine ran it: inputs, params and its outputs."""
    m = golden_meta["engine_rules"][name]
    g = {k[len(name) + 1:]: golden_engine[k] for k in golden_engine.files if k.startswith(name + "_")}
    hist = g["history"].reshape(-1, 22)
    return m, g, hist
