"""oracle_py — TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU oracle.

  libicp_oracle.so   plain-C restatement of the reference path (icp_oracle.c)
  _ref/libicp_ref.so the reference itself (icp_registration.cpp + vendored Eigen), built here
                     by `make -C oracle ref` where /root/reference exists; git-ignored

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module,
and only as the checker / the CPU baseline — never as the product path.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
ORACLE_LIB = ORACLE_DIR / "libicp_oracle.so"
REF_LIB = ORACLE_DIR / "_ref" / "libicp_ref.so"
REF_BENCH = ORACLE_DIR / "_ref" / "ref_bench"
REF_ENGINE_LIB = ORACLE_DIR / "_ref" / "libicp_ref_engine.so"
REF_CORE_SRC = Path("/root/reference/PointCloudRegistration/core/icpengine.cpp")
QT_MOC = Path("/opt/conda/bin/moc")
REFERENCE_SRC = Path("/root/reference/icp_registration.cpp")

SEM_ENGINE = 0
SEM_CLI = 1
DBL_MAX = np.finfo(np.float64).max

_P = C.c_void_p


class OrcParams(C.Structure):
    _fields_ = [("max_iterations", C.c_int32), ("tolerance", C.c_double), ("sigma_multiplier", C.c_double),
                ("octree_max_points", C.c_int32), ("octree_max_depth", C.c_int32), ("semantics", C.c_int32)]


class OrcIter(C.Structure):
    _fields_ = [("iteration", C.c_int32), ("rmse", C.c_double), ("valid", C.c_int32), ("outliers", C.c_int32),
                ("mean", C.c_double), ("std", C.c_double), ("threshold", C.c_double),
                ("T_inc", C.c_double * 16), ("T_cum", C.c_double * 16), ("rotation_deg", C.c_double),
                ("translation", C.c_double), ("has_transform", C.c_int32)]


class OrcResult(C.Structure):
    _fields_ = [("success", C.c_int32), ("status", C.c_int32), ("total_iterations", C.c_int32),
                ("final_rmse", C.c_double), ("final_R", C.c_double * 9), ("final_t", C.c_double * 3),
                ("n_history", C.c_int32)]


def build(ref: bool = True) -> None:
    subprocess.run(["make", "-C", str(ORACLE_DIR), "all"], check=True, capture_output=True)
    if ref and REFERENCE_SRC.exists():
        subprocess.run(["make", "-C", str(ORACLE_DIR), "ref"], check=True, capture_output=True)
    if ref and REF_CORE_SRC.exists() and QT_MOC.exists():
        subprocess.run(["make", "-C", str(ORACLE_DIR), "refqt"], check=True, capture_output=True)
        # the reference's ICPEngine class on libicp_hip.so (integration/icpengine_hip.cpp): needs the
        # product library, which __graft_entry__.build() compiles first
        if (ORACLE_DIR.parent / "iterativeclosestpoint_amd" / "libicp_hip.so").exists():
            subprocess.run(["make", "-C", str(ORACLE_DIR), "refadapter"], check=True, capture_output=True)


_O = None
_R = None


def oracle() -> C.CDLL:
    global _O
    if _O is None:
        if not ORACLE_LIB.exists():
            build(ref=False)
        L = C.CDLL(str(ORACLE_LIB))
        L.orc_octree_build.restype = _P
        L.orc_octree_build.argtypes = [_P, C.c_int64, C.c_int, C.c_int]
        L.orc_octree_free.argtypes = [_P]
        L.orc_octree_shape.argtypes = [_P, _P, _P, _P]
        L.orc_octree_dump.restype = C.c_int64
        L.orc_octree_dump.argtypes = [_P, _P, _P, _P, _P, _P, _P]
        L.orc_find_nearest.restype = C.c_int32
        L.orc_find_nearest.argtypes = [_P, _P, C.c_double, _P, _P]
        L.orc_nn_batch.argtypes = [_P, _P, C.c_int64, C.c_double, _P, _P, _P, _P]
        L.orc_jacobi_svd3.argtypes = [_P, _P, _P, _P]
        L.orc_best_fit.argtypes = [_P, _P, C.c_int64, _P]
        L.orc_transform.argtypes = [_P, _P, C.c_int64]
        L.orc_set_threads.argtypes = [C.c_int]
        L.orc_get_threads.restype = C.c_int
        L.orc_icp.restype = C.c_int
        L.orc_icp.argtypes = [C.POINTER(OrcParams), _P, C.c_int64, _P, C.c_int64, C.POINTER(OrcResult),
                              C.POINTER(OrcIter), C.c_int32]
        _O = L
    return _O


def set_threads(n: int) -> None:
    """OpenMP threads of the oracle's NN loop (per-query results are independent of it)."""
    oracle().orc_set_threads(int(n))


def get_threads() -> int:
    return int(oracle().orc_get_threads())


def reference_available() -> bool:
    return REF_LIB.exists()


def reference() -> C.CDLL:
    global _R
    if _R is None:
        if not REF_LIB.exists():
            raise FileNotFoundError(f"{REF_LIB} not built (needs /root/reference; `make -C oracle ref`)")
        L = C.CDLL(str(REF_LIB))
        L.ref_octree_build.restype = _P
        L.ref_octree_build.argtypes = [_P, C.c_int64, C.c_int, C.c_int]
        L.ref_octree_free.argtypes = [_P]
        L.ref_nn_batch.argtypes = [_P, _P, C.c_int64, _P]
        L.ref_distance.restype = C.c_double
        L.ref_distance.argtypes = [_P, _P]
        L.ref_icp_cli.argtypes = [_P, C.c_int64, _P, C.c_int64, C.c_int, C.c_double, _P, _P, _P, C.c_int, _P]
        L.ref_best_fit_transform.argtypes = [_P, _P, C.c_int64, _P]
        L.ref_jacobi_svd3.argtypes = [_P, C.c_int, _P, _P, _P]
        L.ref_transform.argtypes = [_P, _P, C.c_int64]
        L.ref_mat4_mul.argtypes = [_P, _P, _P]
        _R = L
    return _R


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _aos(a):
    return np.ascontiguousarray(np.asarray(a, np.float64).reshape(-1, 3))


class OracleTree:
    def __init__(self, xyz, max_points=10, max_depth=20):
        self.xyz = _aos(xyz)
        self.h = oracle().orc_octree_build(_p(self.xyz), self.xyz.shape[0], max_points, max_depth)

    def __del__(self):
        if getattr(self, "h", None):
            oracle().orc_octree_free(self.h)
            self.h = None

    def shape(self):
        a, b, c = C.c_int64(), C.c_int64(), C.c_int32()
        oracle().orc_octree_shape(self.h, C.byref(a), C.byref(b), C.byref(c))
        return a.value, b.value, c.value

    def dump(self):
        nn, nl, _ = self.shape()
        depth = np.empty(nn, np.int32)
        octant = np.empty(nn, np.int32)
        box = np.empty((nn, 6))
        leaf = np.empty(nn, np.int32)
        npts = np.empty(nn, np.int32)
        idx = np.empty(max(1, self.xyz.shape[0]), np.int32)
        k = oracle().orc_octree_dump(self.h, _p(depth), _p(octant), _p(box), _p(leaf), _p(npts), _p(idx))
        assert k == nn
        return {"depth": depth, "octant": octant, "box": box, "is_leaf": leaf, "npts": npts,
                "leaf_idx": idx[: int(npts.sum())]}

    def nn(self, q, init_best=DBL_MAX, count=False):
        q = _aos(q)
        idx = np.empty(q.shape[0], np.int32)
        d = np.empty(q.shape[0])
        v, s = C.c_int64(0), C.c_int64(0)
        oracle().orc_nn_batch(self.h, _p(q), q.shape[0], init_best, _p(idx), _p(d), C.byref(v), C.byref(s))
        if count:
            return idx, d, v.value, s.value
        return idx, d


def icp(src, tgt, semantics=SEM_ENGINE, max_iterations=50, tolerance=1e-6, sigma=3.0, max_points=10,
        max_depth=20):
    src = _aos(src).copy()
    tgt = _aos(tgt)
    p = OrcParams(max_iterations, tolerance, sigma, max_points, max_depth, semantics)
    res = OrcResult()
    cap = max(1, max_iterations + 1)
    hist = (OrcIter * cap)()
    rc = oracle().orc_icp(C.byref(p), _p(src), src.shape[0], _p(tgt), tgt.shape[0], C.byref(res), hist, cap)
    return rc, res, [hist[k] for k in range(res.n_history)], src


def svd3(H):
    H = np.ascontiguousarray(H, np.float64).reshape(9)
    U, S, V = np.empty(9), np.empty(3), np.empty(9)
    oracle().orc_jacobi_svd3(_p(H), _p(U), _p(S), _p(V))
    return U.reshape(3, 3), S, V.reshape(3, 3)


def best_fit(a, b):
    a, b = _aos(a), _aos(b)
    T = np.empty(16)
    oracle().orc_best_fit(_p(a), _p(b), a.shape[0], _p(T))
    return T.reshape(4, 4)


def transform(T, xyz):
    xyz = _aos(xyz).copy()
    T = np.ascontiguousarray(T, np.float64).reshape(16)
    oracle().orc_transform(_p(T), _p(xyz), xyz.shape[0])
    return xyz


# ---- the reference itself (fixture generation in this container only) ----

class RefTree:
    def __init__(self, xyz, max_points=10, max_depth=20):
        self.xyz = _aos(xyz)
        self.h = reference().ref_octree_build(_p(self.xyz), self.xyz.shape[0], max_points, max_depth)

    def __del__(self):
        if getattr(self, "h", None):
            reference().ref_octree_free(self.h)
            self.h = None

    def nn(self, q):
        q = _aos(q)
        idx = np.empty(q.shape[0], np.int32)
        reference().ref_nn_batch(self.h, _p(q), q.shape[0], _p(idx))
        return idx


def ref_icp_cli(src, tgt, max_iterations=20, tolerance=1e-2):
    src = _aos(src).copy()
    tgt = _aos(tgt)
    R, t = np.empty(9), np.empty(3)
    cap = max(1, max_iterations)
    tc = np.zeros((cap, 16))
    n = C.c_int(0)
    reference().ref_icp_cli(_p(src), src.shape[0], _p(tgt), tgt.shape[0], max_iterations, tolerance, _p(R), _p(t),
                            _p(tc), cap, C.byref(n))
    return R.reshape(3, 3), t, tc[: n.value].reshape(-1, 4, 4), src


def ref_svd3(H, dynamic=False):
    H = np.ascontiguousarray(H, np.float64).reshape(9)
    U, S, V = np.empty(9), np.empty(3), np.empty(9)
    reference().ref_jacobi_svd3(_p(H), 1 if dynamic else 0, _p(U), _p(S), _p(V))
    return U.reshape(3, 3), S, V.reshape(3, 3)


def ref_best_fit(a, b):
    a, b = _aos(a), _aos(b)
    T = np.empty(16)
    reference().ref_best_fit_transform(_p(a), _p(b), a.shape[0], _p(T))
    return T.reshape(4, 4)


def ref_transform(T, xyz):
    xyz = _aos(xyz).copy()
    T = np.ascontiguousarray(T, np.float64).reshape(16)
    reference().ref_transform(_p(T), _p(xyz), xyz.shape[0])
    return xyz


def ref_mat4_mul(A, B):
    A = np.ascontiguousarray(A, np.float64).reshape(16)
    B = np.ascontiguousarray(B, np.float64).reshape(16)
    Cm = np.empty(16)
    reference().ref_mat4_mul(_p(A), _p(B), _p(Cm))
    return Cm.reshape(4, 4)


def ref_read_las(path, cap=10_000_000):
    L = reference()
    L.ref_read_las.restype = C.c_int64
    L.ref_read_las.argtypes = [C.c_char_p, _P, C.c_int64, _P]
    xyz = np.empty((cap, 3))
    so = np.empty(6)
    n = L.ref_read_las(str(path).encode(), _p(xyz), cap, _p(so))
    return (None, None) if n < 0 else (xyz[:n].copy(), so)


def ref_save_las(path, xyz, scale, offset):
    L = reference()
    L.ref_save_las.argtypes = [C.c_char_p, _P, C.c_int64, _P, _P]
    xyz = _aos(xyz)
    sc = np.ascontiguousarray(scale, np.float64)
    of = np.ascontiguousarray(offset, np.float64)
    L.ref_save_las(str(path).encode(), _p(xyz), xyz.shape[0], _p(sc), _p(of))


def ref_save_transformation(path, R, t, transforms):
    L = reference()
    L.ref_save_transformation.argtypes = [C.c_char_p, _P, _P, _P, C.c_int]
    R = np.ascontiguousarray(R, np.float64).reshape(9)
    t = np.ascontiguousarray(t, np.float64).reshape(3)
    T = np.ascontiguousarray(transforms, np.float64).reshape(-1, 16)
    L.ref_save_transformation(str(path).encode(), _p(R), _p(t), _p(T), T.shape[0])


# ---- the reference's core engine + LAS I/O (Qt build, fixture generation in this container only)

REC_DOUBLES = 22  # iteration, rmse, valid, outliers, T_cum (16, row-major), rotation, translation
_E = None


def ref_engine_available() -> bool:
    return REF_ENGINE_LIB.exists()


def ref_engine() -> C.CDLL:
    global _E
    if _E is None:
        if not REF_ENGINE_LIB.exists():
            raise FileNotFoundError(f"{REF_ENGINE_LIB} not built (needs /root/reference and conda Qt; "
                                    "`make -C oracle refqt`)")
        L = C.CDLL(str(REF_ENGINE_LIB))
        L.refeng_register.restype = C.c_int
        L.refeng_register.argtypes = [_P, C.c_int64, _P, C.c_int64, C.c_int, C.c_double, C.c_double, C.c_int,
                                      C.c_int, C.c_int, _P, _P, _P, _P, _P, _P, C.c_int32, _P, _P, C.c_int32]
        L.refeng_read_las.restype = C.c_int64
        L.refeng_read_las.argtypes = [C.c_char_p, C.c_int64, _P, C.c_int64]
        L.refeng_write_las.restype = C.c_int
        L.refeng_write_las.argtypes = [C.c_char_p, _P, C.c_int64, _P]
        _E = L
    return _E


def ref_engine_register(src, tgt, max_iterations=50, tolerance=1e-6, sigma=3.0, max_points=10, max_depth=20,
                        stop_at=-1):
    """ICPEngine::setParameters + registerPointClouds of the real core/icpengine.cpp. Returns a dict:
    finished (1 ok / 0 failed / -1 no signal), message, total_iterations, final_rmse, final_R,
    final_t, history (k x 22), source_out."""
    src = _aos(src)
    tgt = _aos(tgt)
    out = np.empty_like(src)
    ti, fr, nh = C.c_int32(), C.c_double(), C.c_int32()
    R, t = np.empty(9), np.empty(3)
    cap = max(1, max_iterations + 1)
    hist = np.zeros((cap, REC_DOUBLES))
    msg = C.create_string_buffer(256)
    rc = ref_engine().refeng_register(_p(src), src.shape[0], _p(tgt), tgt.shape[0], max_iterations, tolerance, sigma,
                                      max_points, max_depth, stop_at, _p(out), C.byref(ti), C.byref(fr), _p(R),
                                      _p(t), _p(hist), cap, C.byref(nh), msg, 256)
    return {"finished": rc, "message": msg.value.decode("utf-8", errors="replace"),
            "total_iterations": ti.value, "final_rmse": fr.value, "final_R": R.reshape(3, 3), "final_t": t,
            "history": hist[: nh.value].copy(), "source_out": out}


def ref_core_read_las(path, max_points=0, cap=20_000_000):
    xyz = np.empty((cap, 3))
    n = ref_engine().refeng_read_las(str(path).encode(), max_points, _p(xyz), cap)
    return None if n < 0 else xyz[:n].copy()


def ref_core_write_las(path, xyz, bounds=None):
    """LASIO::writeLAS; bounds = (minX, maxX, minY, maxY, minZ, maxZ) as the caller's PointCloud
    holds them (None: computeBounds())."""
    xyz = _aos(xyz)
    b = None if bounds is None else np.ascontiguousarray(bounds, np.float64)
    return bool(ref_engine().refeng_write_las(str(path).encode(), _p(xyz), xyz.shape[0],
                                              None if b is None else _p(b)))
