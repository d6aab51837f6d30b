"""The reference-typed adapter (include/icp_ref_adapter.hpp) and the reference's own ICPEngine class
implemented on it (integration/icpengine_hip.cpp): the drop-in on the caller's types, no copy of
the clouds (VERDICT r03 missing #1; icpengine.h:13-44, :60-75; pointcloud.h:30-65;
registrationservice.cpp:204-212).

  * mirror types (tests/cpp/ref_adapter_mirror.cpp): structs laid out as the reference's, with an
    Eigen-style column-major Matrix4d; compiled here (CPU), run on the GPU against the plain facade
    (bit for bit: history, transforms, final R/t, the moved source in place) and with a stop;
  * the reference's real headers (oracle/Makefile refadapter: core/icpengine.h + pointcloud.cpp where
    they lie, moc, Qt 5.9.7 of the image, the vendored Eigen) driven as RegistrationService drives
    them: the empty-source path on the CPU, and on the GPU the same results as the mirror build
    (same generator and seed) and a stop() from the third iterationCompleted signal.
"""
import json
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REF_ENGINE = ROOT / "oracle" / "_ref" / "ref_adapter_engine"
CANCELLED = "用户取消"
EMPTY = "点云数据为空"
SUCCESS = "配准成功"


def _build_mirror(tmp_path):
    exe = tmp_path / "ref_adapter_mirror"
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", "-I", str(ROOT / "include"), "-I",
           "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", str(ROOT / "tests" / "cpp" / "ref_adapter_mirror.cpp"),
           "-o", str(exe), "-L", str(ROOT / "iterativeclosestpoint_amd"), "-licp_hip",
           f"-Wl,-rpath,{ROOT / 'iterativeclosestpoint_amd'}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def _run(exe, *args):
    r = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=300,
                       env={"QT_QPA_PLATFORM": "offscreen", "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["stderr"] = r.stderr
    return out


def _ref_engine():
    if not REF_ENGINE.exists():
        if not Path("/root/reference/PointCloudRegistration/core/icpengine.h").exists():
            pytest.skip("reference headers absent and oracle/_ref/ref_adapter_engine not built")
        subprocess.run(["make", "-C", str(ROOT / "oracle"), "refadapter"], check=True, capture_output=True)
    return REF_ENGINE


def test_mirror_adapter_empty_source(icp, tmp_path):
    out = _run(_build_mirror(tmp_path), "empty")
    assert out["finished"] == 1 and out["success"] == 0 and out["message"] == EMPTY
    assert out["started"] == 0 and out["iterations"] == 0 and out["progress"] == 0


def test_reference_engine_empty_source(icp):
    out = _run(_ref_engine(), "empty")
    assert out["finished"] == 1 and out["success"] == 0 and out["message"] == EMPTY
    assert out["started"] == 0 and out["iterations"] == 0


@pytest.mark.gpu
def test_mirror_adapter_matches_facade(icp, tmp_path):
    out = _run(_build_mirror(tmp_path))
    assert out["rc"] == 0 and out["success"] == 1 and out["result_success"] == 1 and out["message"] == SUCCESS
    assert out["same_as_facade"] == 1 and out["in_place"] == 1, out["stderr"]
    assert out["started"] == 1 and out["finished"] == 1
    assert out["iterations"] == out["history"] == out["total_iterations"] == out["progress"] >= 2


@pytest.mark.gpu
def test_mirror_adapter_stop(icp, tmp_path):
    out = _run(_build_mirror(tmp_path), "stop")
    assert out["rc"] == -10  # ICP_ENGINE_CANCELLED (icp_engine.h)
    assert out["iterations"] == 3 and out["finished"] == 1 and out["success"] == 0 and out["message"] == CANCELLED


@pytest.mark.gpu
def test_reference_engine_on_gpu_equals_mirror(icp, tmp_path):
    ref = _run(_ref_engine())
    mir = _run(_build_mirror(tmp_path))
    assert ref["success"] == 1 and ref["message"] == SUCCESS and ref["started"] == 1 and ref["finished"] == 1
    assert ref["iterations"] == ref["total_iterations"] == mir["total_iterations"]
    for key in ("final_R", "final_t", "transforms", "checksum"):
        assert ref[key] == mir[key], key  # same clouds, same library: bit for bit


@pytest.mark.gpu
def test_reference_engine_stop_signal(icp):
    out = _run(_ref_engine(), "stop")
    assert out["iterations"] == 3 and out["finished"] == 1 and out["success"] == 0 and out["message"] == CANCELLED
