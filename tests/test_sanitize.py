"""Sanitizer builds of the host-side code (SURVEY §5 "ASan/UBSan CPU builds of the host lib"; VERDICT
r03 missing #2): iterativeclosestpoint_amd/csrc/Makefile targets `asan` (AddressSanitizer +
UndefinedBehaviorSanitizer, no recovery) and `tsan` (ThreadSanitizer) build tests/cpp/host_sanitize.cpp
with the product's own host sources — the LAS readers/writers, the host octree builder, the host
kd query order, the 3x3 SVD / best fit, the session's decisions (session_step.h) and the
multi-device context's driver threads + in-process exchange (group_sync.h, N = 2, 3, 8 members,
1200 jobs with injected member failures). The LAS readers run on the golden files, on every
truncation of their headers and records, and on garbage. CPU only; no HIP call is made."""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "iterativeclosestpoint_amd" / "csrc"
SAN = ROOT / "build" / "sanitize"


def _las_inputs(tmp_path):
    g = np.load(ROOT / "tests" / "golden" / "las_report.npz")
    c = np.load(ROOT / "tests" / "golden" / "core_las.npz")
    files = []
    for name, blob in (("cli", g["las_file"].tobytes()), ("core", c["core_file"].tobytes()),
                       ("stale", c["core_file_stale"].tobytes())):
        for cut in sorted({len(blob), 0, 1, 4, 96, 226, 227, 240, len(blob) // 2, len(blob) - 1, len(blob) - 17}):
            if 0 <= cut <= len(blob):
                f = tmp_path / f"{name}_{cut}.las"
                f.write_bytes(blob[:cut])
                files.append(f)
        # a header whose offset/record length/count point past the end of the file
        bad = bytearray(blob[:400])
        bad[96:100] = (10 ** 9).to_bytes(4, "little")
        (tmp_path / f"{name}_badoff.las").write_bytes(bytes(bad))
        files.append(tmp_path / f"{name}_badoff.las")
    rng = np.random.default_rng(5)
    junk = tmp_path / "junk.las"
    junk.write_bytes(b"LASF" + rng.integers(0, 256, 4000, dtype=np.uint8).tobytes())
    files.append(junk)
    files.append(tmp_path / "missing.las")
    return [str(f) for f in files]


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_code_under_sanitizer(kind, tmp_path):
    r = subprocess.run(["make", "-C", str(CSRC), kind], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    exe = SAN / f"host_{kind}"
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    env["TSAN_OPTIONS"] = "halt_on_error=1:second_deadlock_stack=1"
    run = subprocess.run([str(exe), *_las_inputs(tmp_path)], capture_output=True, text=True, timeout=600, env=env)
    report = run.stdout[-2000:] + run.stderr[-6000:]
    assert run.returncode == 0, report
    assert "ERROR: AddressSanitizer" not in run.stderr and "runtime error" not in run.stderr, report
    assert "WARNING: ThreadSanitizer" not in run.stderr, report
    assert run.stdout.strip().splitlines()[-1] == "ok", report
