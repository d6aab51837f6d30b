"""The C-ABI library loads and exports every function declared in include/*.h (no GPU calls)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
DECL = re.compile(r"^[A-Za-z_][\w\s\*]*?\b(icp_\w+)\s*\(", re.M)


def declared_functions():
    names = set()
    for h in sorted((ROOT / "include").glob("*.h")):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        for m in DECL.finditer(text):
            if not text[m.start():m.end()].lstrip().startswith(("typedef", "#")):
                names.add(m.group(1))
    return sorted(names)


def test_headers_declare_functions():
    names = declared_functions()
    assert "icp_hip_iterate" in names and "icp_engine_register" in names and "icp_octree_build" in names
    assert len(names) >= 30


@pytest.mark.parametrize("name", declared_functions())
def test_symbol_exported(icp, name):
    lib = ctypes.CDLL(str(icp.LIB_PATH))
    assert hasattr(lib, name), f"{name} declared in include/ but not exported"


def test_binding_covers_headers(icp):
    from iterativeclosestpoint_amd._lib import SIGNATURES
    assert set(declared_functions()) <= set(SIGNATURES), set(declared_functions()) - set(SIGNATURES)


def test_no_gpu_fails_loudly(icp):
    """Without a GPU the device path refuses (no CPU fallback exists)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(icp.IcpError):
        icp.Context(0)


def test_create_multi_rejects_bad_arguments_without_a_gpu(icp):
    """icp_hip_create_multi validates its device list and transport before touching a device."""
    import ctypes as C
    L = icp.lib()
    h = C.c_void_p()
    two = (C.c_int32 * 2)(0, 0)
    assert L.icp_hip_create_multi(C.byref(h), 2, two, None, icp.XPORT_RCCL) == -1  # RCCL: distinct GPUs
    assert L.icp_hip_create_multi(C.byref(h), 2, two, None, 7) == -1              # unknown transport
    assert L.icp_hip_create_multi(C.byref(h), 0, two, None, icp.XPORT_AUTO) == -1  # empty list
    assert not h.value


def test_create_ex_validates_config_without_a_gpu(icp):
    """icp_hip_create_ex checks the config (version, ranges, the no_warmup switch) before any
    device call: a struct of another header version or an out-of-range field is EINVAL."""
    import ctypes as C
    L = icp.lib()
    h = C.c_void_p()
    cfg = icp.config()
    assert cfg.no_warmup == 0 and cfg.config_version == 3
    assert icp.HipConfig.config_version.offset == 0  # the version word first: checked before the copy
    for field, bad in (("no_warmup", 2), ("ball_mode", 3), ("wide_pass", 3), ("peer_timeout_ms", -1), ("scan_groups", 3),
                       ("config_version", 2), ("config_version", 0)):
        c = icp.config()
        setattr(c, field, bad)
        assert L.icp_hip_create_ex(C.byref(h), 0, C.byref(c)) == icp.EINVAL, field
        assert not h.value
        msg = L.icp_hip_last_error().decode()
        assert (field if field != "config_version" else "config_version") in msg, msg


def test_create_ex_rejects_nonzero_reserved_words(icp):
    """Later header versions carve fields out of `reserved`: a nonzero word is refused, not ignored."""
    import ctypes as C
    L = icp.lib()
    h = C.c_void_p()
    for k in range(3):
        c = icp.config()
        c.reserved[k] = 1
        assert L.icp_hip_create_ex(C.byref(h), 0, C.byref(c)) == icp.EINVAL
        assert not h.value
        assert "reserved" in L.icp_hip_last_error().decode()
