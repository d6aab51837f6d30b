"""The C++ drop-in facade (include/icp_engine.hpp) compiles against libicp_hip.so (CPU) and runs
the reference's call shapes — ICPEngine::registerPointClouds, Octree::findNearest, ICP() —
on the GPU."""
import json
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _build(tmp_path):
    exe = tmp_path / "facade_demo"
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-I", str(ROOT / "include"), "-I", "/opt/rocm/include",
           "-D__HIP_PLATFORM_AMD__", str(ROOT / "tests" / "cpp" / "facade_demo.cpp"), "-o", str(exe),
           "-L", str(ROOT / "iterativeclosestpoint_amd"), "-licp_hip",
           f"-Wl,-rpath,{ROOT / 'iterativeclosestpoint_amd'}"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_facade_compiles(icp, tmp_path):
    assert _build(tmp_path).exists()


@pytest.mark.gpu
def test_facade_runs_on_gpu(icp, tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["success"] and out["many_ok"] and out["nn"] == 123
