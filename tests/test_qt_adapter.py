"""The Qt signal adapter (include/icp_engine_qt.h; the reference's ICPEngine signals,
icpengine.h:69-74) builds with the image's Qt 5.9.7 moc against libicp_hip.so; without a GPU an
empty source gives finished(false) and nothing else (icpengine.cpp:27-32), and on the GPU a
registration emits started once, iterationCompleted and progressUpdated once per iteration record
and finished(true) once, with the same transforms as the plain facade."""
import json
import os
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
QT = Path("/opt/conda")
QTINC = [f"-I{QT / 'include' / 'qt'}", f"-I{QT / 'include' / 'qt' / 'QtCore'}"]

pytestmark = pytest.mark.skipif(not (QT / "bin" / "moc").exists() or not (QT / "lib" / "libQt5Core.so.5").exists(),
                                reason="no Qt 5 (moc, libQt5Core) in this image")


def _qtlib(tmp_path):
    """Qt's libraries and their conda dependencies as symlinks, without conda's libstdc++ and
    libgcc_s (the system g++ runtime must win), as oracle/Makefile's refqt recipe does."""
    d = tmp_path / "qtlib"
    d.mkdir()
    core = QT / "lib" / "libQt5Core.so.5"
    out = subprocess.run(["ldd", str(core)], capture_output=True, text=True, check=True).stdout
    libs = {core}
    for line in out.splitlines():
        parts = line.split("=>")
        if len(parts) == 2 and str(QT) in parts[1]:
            libs.add(Path(parts[1].split()[0]))
    for lib in libs:
        if "libstdc++" in lib.name or "libgcc_s" in lib.name:
            continue
        (d / lib.name).symlink_to(os.path.realpath(lib))
    return d


def _build(tmp_path):
    moc = tmp_path / "moc_icp_engine_qt.cpp"
    subprocess.run([str(QT / "bin" / "moc"), *QTINC, f"-I{ROOT / 'include'}", str(ROOT / "include" / "icp_engine_qt.h"),
                    "-o", str(moc)], check=True, capture_output=True, text=True)
    qtlib = _qtlib(tmp_path)
    exe = tmp_path / "qt_adapter_demo"
    cmd = ["g++", "-std=c++17", "-O2", "-fPIC", "-Wall", "-I", str(ROOT / "include"), "-I", "/opt/rocm/include",
           "-D__HIP_PLATFORM_AMD__", *QTINC, str(ROOT / "tests" / "cpp" / "qt_adapter_demo.cpp"), str(moc),
           "-o", str(exe), "-L", str(ROOT / "iterativeclosestpoint_amd"), "-licp_hip",
           f"-Wl,-rpath,{ROOT / 'iterativeclosestpoint_amd'}", f"-L{qtlib}", "-l:libQt5Core.so.5",
           f"-Wl,-rpath,{qtlib}", f"-Wl,-rpath-link,{qtlib}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def _run(exe, *args):
    r = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=300,
                       env={**os.environ, "QT_QPA_PLATFORM": "offscreen"})
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_qt_adapter_builds_and_reports_empty_input(icp, tmp_path):
    out = _run(_build(tmp_path), "empty")
    # icpengine.cpp:31-33: an empty cloud finishes with failure before started()
    assert out == {**out, "started": 0, "progress": 0, "iterations": 0, "finished": 1, "success": 0}
    assert out["message_len"] > 0


@pytest.mark.gpu
def test_qt_adapter_signals_on_gpu(icp, tmp_path):
    out = _run(_build(tmp_path))
    assert out["success"] == 1 and out["finished"] == 1 and out["started"] == 1
    assert out["iterations"] == out["history"] > 0
    assert out["progress"] == out["iterations"] and 1 <= out["last_progress"] <= 30
    assert out["log"] > 0
    assert out["same_as_facade"] == 1
