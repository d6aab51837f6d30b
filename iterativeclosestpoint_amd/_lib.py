"""ctypes binding of libicp_hip.so (harness only; the product is the C-ABI library)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
LIB_PATH = Path(os.environ.get("ICP_HIP_LIB", PKG_DIR / "libicp_hip.so"))  # override: A/B of builds

RULES_ENGINE = 0
RULES_CLI = 1
FLAG_NO_EARLY_STOP = 1
SEARCH_CERTIFIED = 0
SEARCH_REFERENCE = 1
BUILD_AUTO = 0
BUILD_HOST = 1
XPORT_AUTO = 0
XPORT_RCCL = 1
XPORT_HOST = 2
XPORT_CALLBACK = 3
# icp_hip.h error codes (IcpError.code)
OK, EINVAL, ENOMEM, EDEVICE, ERCCL, ENOTREADY, EEXCHANGE = 0, -1, -2, -3, -4, -5, -6
DBG_SLOTS = 40
# icp_hip.h ICP_DBG_* slot names
DBG_NAMES = {0: "waves", 1: "overflow_waves", 2: "not_joined", 3: "not_covered", 4: "scanned_points",
             8: "fp64_scan_waves", 9: "staged_points", 10: "scan_pairs", 11: "scan_rounds",
             12: "cache_hits", 13: "cache_stores",
             5: "walk_batches", 6: "no_guess", 7: "candidates", 14: "ball_overflow", 15: "ball_points",
             21: "start_nodes", 20: "winner_prev_waves", 22: "winner_prev", 23: "winner_lanes",
             18: "prev_cert_waves", 19: "prev_cert_lanes", 16: "halves", 17: "reused_entries",
             24: "walk_moved", 25: "walk_loose", 26: "group_points", 27: "bb_queries", 28: "bb_steps",
             29: "lane_handed", 30: "fz_recompute", 31: "fz_band", 32: "wide_waves", 33: "wide_segments",
             34: "wide_stack", 35: "wide_undecided", 36: "wide_points", 37: "bb_overflow", 38: "lane_exact"}

_P = C.c_void_p
_D = C.POINTER(C.c_double)
_I32 = C.POINTER(C.c_int32)


class IcpError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"icp error {code}: {msg}")
        self.code = code


class IterStats(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("mean", C.c_double), ("std", C.c_double), ("threshold", C.c_double),
        ("valid", C.c_int64), ("rmse", C.c_double), ("sum_d2", C.c_double), ("min_d", C.c_double),
        ("max_d", C.c_double), ("n_bad", C.c_int64), ("centroid_src", C.c_double * 3),
        ("centroid_tgt", C.c_double * 3), ("H", C.c_double * 9), ("n_fallback", C.c_int64),
        ("n_lane_search", C.c_int64), ("n_ball_search", C.c_int64),
    ]

    def as_dict(self) -> dict:
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            out[name] = list(v) if not isinstance(v, (int, float)) else v
        return out


class HipConfig(C.Structure):
    """icp_hip_config (include/icp_hip.h): explicit search options of a context."""
    _fields_ = [
        ("config_version", C.c_uint32), ("search", C.c_int32), ("scan32", C.c_int32), ("cell_starts", C.c_int32),
        ("octree_builder", C.c_int32), ("join_factor", C.c_double), ("debug_counters", C.c_int32),
        ("xcd_blocks", C.c_int32), ("scan_groups", C.c_int32), ("candidate_cache", C.c_int32),
        ("candidate_margin", C.c_int32), ("certify_prev", C.c_int32), ("query_order", C.c_int32),
        ("overflow_halves", C.c_int32), ("device_loop", C.c_int32), ("timing_stride", C.c_int32),
        ("candidate_loose", C.c_int32), ("candidate_lead", C.c_int32), ("fused_cull", C.c_int32),
        ("peer_timeout_ms", C.c_int32), ("no_warmup", C.c_int32), ("ball_mode", C.c_int32), ("wide_pass", C.c_int32), ("reserved", C.c_int32 * 3),
    ]


class Params(C.Structure):
    _fields_ = [
        ("max_iterations", C.c_int32), ("tolerance", C.c_double), ("sigma_multiplier", C.c_double),
        ("octree_max_points", C.c_int32), ("octree_max_depth", C.c_int32), ("rules", C.c_int32),
        ("flags", C.c_int32),
    ]


class IterationRecord(C.Structure):
    _fields_ = [
        ("iteration", C.c_int32), ("rmse", C.c_double), ("valid_points", C.c_int32),
        ("outlier_points", C.c_int32), ("transform", C.c_double * 16),
        ("rotation_angle_deg", C.c_double), ("translation_distance", C.c_double),
        ("has_transform", C.c_int32), ("mean", C.c_double), ("std", C.c_double),
        ("threshold", C.c_double), ("increment", C.c_double * 16),
    ]


class Result(C.Structure):
    _fields_ = [
        ("success", C.c_int32), ("status", C.c_int32), ("total_iterations", C.c_int32),
        ("final_rmse", C.c_double), ("final_R", C.c_double * 9), ("final_t", C.c_double * 3),
        ("n_history", C.c_int32), ("message", C.c_char * 160),
    ]


ITER_CB = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(IterationRecord))
PROGRESS_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.c_double)
LOG_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_char_p)


class Hooks(C.Structure):
    _fields_ = [
        ("user", C.c_void_p), ("on_iteration", ITER_CB), ("on_progress", PROGRESS_CB),
        ("on_log", LOG_CB), ("stop_flag", C.POINTER(C.c_int32)),
    ]


class OctreeInfo(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_int64), ("n_leaves", C.c_int64), ("n_points", C.c_int64),
        ("max_depth", C.c_int32), ("max_inner_depth", C.c_int32), ("pos_of_orig0", C.c_int32),
    ]


class LasHeader(C.Structure):
    _fields_ = [
        ("offset_to_points", C.c_uint32), ("num_points", C.c_uint32), ("record_length", C.c_uint16),
        ("scale", C.c_double * 3), ("offset", C.c_double * 3), ("max", C.c_double * 3), ("min", C.c_double * 3),
    ]


class SynthSpec(C.Structure):
    _fields_ = [
        ("sigma", C.c_double * 3), ("yaw_deg", C.c_double), ("pitch_deg", C.c_double),
        ("roll_deg", C.c_double), ("t", C.c_double * 3), ("noise_sigma", C.c_double),
        ("outlier_fraction", C.c_double), ("seed_target", C.c_uint64), ("seed_source", C.c_uint64),
    ]


class SceneSpec(C.Structure):
    _fields_ = [
        ("site_radius", C.c_double), ("scanner_height", C.c_double), ("n_walls", C.c_int32),
        ("wall_height", C.c_double), ("terrain_amp", C.c_double), ("elev_min_deg", C.c_double),
        ("elev_max_deg", C.c_double), ("range_noise", C.c_double), ("quantum", C.c_double),
        ("yaw_deg", C.c_double), ("pitch_deg", C.c_double), ("roll_deg", C.c_double), ("t", C.c_double * 3),
        ("outlier_fraction", C.c_double), ("seed_target", C.c_uint64), ("seed_source", C.c_uint64),
    ]


_EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int32, C.POINTER(C.c_double))

# (name, restype, argtypes) for every exported symbol; also the list the ABI test checks
SIGNATURES = {
    # icp_hip.h
    "icp_hip_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "icp_hip_config_default": (None, [C.POINTER(HipConfig)]),
    "icp_hip_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_int]),
    "icp_hip_create_ex": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.POINTER(HipConfig)]),
    "icp_hip_create_multi": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, _I32, C.POINTER(HipConfig), C.c_int]),
    "icp_hip_ctx_devices": (C.c_int, [_P, _I32, _I32, C.c_int32, _I32]),
    "icp_hip_debug_counters": (C.c_int, [_P, _P]),
    "icp_hip_destroy": (None, [_P]),
    "icp_hip_get_unique_id": (C.c_int, [C.c_char_p]),
    "icp_hip_comm_init": (C.c_int, [_P, C.c_int, C.c_int, C.c_char_p]),
    "icp_hip_comm_init_host": (C.c_int, [_P, C.c_int, C.c_int, C.c_void_p, _P]),
    "icp_hip_set_target": (C.c_int, [_P, _P, C.c_int64, C.c_int, C.c_int, C.c_int]),
    "icp_hip_set_source": (C.c_int, [_P, _P, C.c_int64]),
    "icp_hip_iterate": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_double, C.POINTER(IterStats)]),
    "icp_hip_apply": (C.c_int, [_P, _P]),
    "icp_hip_get_source": (C.c_int, [_P, _P]),
    "icp_hip_get_correspondences": (C.c_int, [_P, _P, _P]),
    "icp_hip_nn": (C.c_int, [_P, _P, C.c_int64, _P, _P]),
    "icp_hip_traversal_counts": (C.c_int, [_P, _D, _D]),
    "icp_hip_target_info": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64), _I32, _I32]),
    "icp_hip_last_timing": (C.c_int, [_P, _D, _D]),
    "icp_hip_last_cull_path": (C.c_int, [_P, _I32]),
    "icp_hip_timings": (C.c_int, [_P, C.c_int, _P, _P]),
    "icp_hip_exchange_timings": (C.c_int, [_P, C.c_int, _P]),
    "icp_hip_comm_info": (C.c_int, [_P, C.c_int, _I32, _I32, _I32, _I32]),
    "icp_hip_target_build_info": (C.c_int, [_P, _I32, _D]),
    "icp_hip_copy_target": (C.c_int, [_P, _P, _P, _P, _P, _P, _P]),
    "icp_hip_target_separation": (C.c_int, [_P, _P]),
    "icp_hip_synchronize": (C.c_int, [_P]),
    "icp_hip_comm_abort": (C.c_int, [_P]),
    "icp_hip_debug_inject_failure": (C.c_int, [_P, C.c_int, C.c_int]),
    "icp_hip_last_error": (C.c_char_p, []),
    # icp_engine.h
    "icp_params_default": (None, [C.POINTER(Params)]),
    "icp_engine_register": (C.c_int, [C.POINTER(Params), _P, C.c_int64, _P, C.c_int64, C.c_int,
                                      C.POINTER(Result), C.POINTER(IterationRecord), C.c_int32,
                                      C.POINTER(Hooks)]),
    "icp_engine_register_devices": (C.c_int, [C.POINTER(Params), _P, C.c_int64, _P, C.c_int64, C.c_int, _I32,
                                              C.POINTER(Result), C.POINTER(IterationRecord), C.c_int32,
                                              C.POINTER(Hooks)]),
    "icp_engine_run": (C.c_int, [_P, C.POINTER(Params), C.POINTER(Result), C.POINTER(IterationRecord),
                                 C.c_int32, C.POINTER(Hooks)]),
    "icp_session_create": (C.c_int, [_P, C.POINTER(Params), C.POINTER(Hooks), C.POINTER(C.c_void_p)]),
    "icp_session_step": (C.c_int, [_P, C.POINTER(IterationRecord), _I32, _I32]),
    "icp_session_step_n": (C.c_int, [_P, C.c_int32, _I32, _I32]),
    "icp_session_step_n_timed": (C.c_int, [_P, C.c_int32, _I32, _I32, _P]),
    "icp_session_finish": (C.c_int, [_P, C.POINTER(Result)]),
    "icp_session_transform": (None, [_P, _P]),
    "icp_session_destroy": (None, [_P]),
    "icp_cli_icp": (C.c_int, [_P, C.c_int64, _P, C.c_int64, C.c_int, C.c_double, _P, _P, _P, C.c_int32,
                              _I32, C.c_int]),
    "icp_cli_icp_devices": (C.c_int, [_P, C.c_int64, _P, C.c_int64, C.c_int, C.c_double, _P, _P, _P, C.c_int32,
                                      _I32, C.c_int, _I32]),
    "icp_jacobi_svd3": (None, [_P, _P, _P, _P]),
    "icp_best_fit_transform": (None, [_P, _P, C.c_int64, _P]),
    "icp_best_fit_from_stats": (None, [C.POINTER(IterStats), _P]),
    "icp_mat4_mul": (None, [_P, _P, _P]),
    # icp_host.h
    "icp_octree_build": (C.c_void_p, [_P, C.c_int64, C.c_int, C.c_int]),
    "icp_octree_free": (None, [_P]),
    "icp_octree_get_info": (None, [_P, C.POINTER(OctreeInfo)]),
    "icp_octree_copy_nodes": (None, [_P, _P, _P, _P, _P]),
    "icp_octree_copy_points": (None, [_P, _P, _P]),
    "icp_moments_from_values": (None, [_P, C.c_int64, _P]),
    "icp_moments_merge": (None, [_P, C.c_int32, _P]),
    "icp_cov_from_pairs": (None, [_P, _P, _P, C.c_int64, C.c_double, _P]),
    "icp_cov_merge": (None, [_P, C.c_int32, _P]),
    "icp_cull_threshold": (C.c_double, [C.c_double, C.c_double, C.c_double, C.c_int, C.c_int]),
    "icp_synth_default": (None, [C.POINTER(SynthSpec)]),
    "icp_synth_pair": (C.c_int, [C.POINTER(SynthSpec), C.c_int64, C.c_int64, _P, _P, _P]),
    "icp_source_shard_order": (C.c_int, [_P, C.c_int64, _P]),
    "icp_scene_default": (None, [C.POINTER(SceneSpec)]),
    "icp_synth_scene": (C.c_int, [C.POINTER(SceneSpec), C.c_int64, C.c_int64, _P, _P, _P]),
    # icp_las.h
    "icp_las_read_header": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(LasHeader)]),
    "icp_las_read": (C.c_int64, [C.c_char_p, C.c_int, C.c_int64, _P, C.POINTER(LasHeader)]),
    "icp_las_write_core": (C.c_int, [C.c_char_p, _P, C.c_int64]),
    "icp_las_write_core_bounds": (C.c_int, [C.c_char_p, _P, C.c_int64, _P]),
    "icp_las_write_cli": (C.c_int, [C.c_char_p, _P, C.c_int64, _P, _P]),
    "icp_write_transform_report": (C.c_int, [C.c_char_p, _P, _P, _P, C.c_int32]),
}

_LIB = None


def build(verbose: bool = False) -> None:
    """Compile libicp_hip.so in-tree for gfx950 (hipcc; no GPU needed)."""
    jobs = str(min(16, os.cpu_count() or 4))
    r = subprocess.run(["make", "-j", jobs, "-C", str(PKG_DIR / "csrc")], capture_output=True, text=True)
    if verbose or r.returncode != 0:
        print(r.stdout[-4000:], r.stderr[-4000:])
    if r.returncode != 0:
        raise RuntimeError("building libicp_hip.so failed")


def lib() -> C.CDLL:
    """Load libicp_hip.so; raises if it is missing (there is no fallback path)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} not built: run `make -C iterativeclosestpoint_amd/csrc` "
                          "or __graft_entry__.build() (no CPU fallback exists)")
    L = C.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        if "ICP_HIP_LIB" in os.environ and not hasattr(L, name):
            continue  # an older build under A/B: it lacks the newer entry points
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _aos(a) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    if a.ndim != 2 or a.shape[1] != 3:
        raise ValueError("expected an (n, 3) float64 array")
    return a


def _check(rc: int) -> None:
    if rc != 0:
        raise IcpError(rc, lib().icp_hip_last_error().decode(errors="replace"))


def params_default(**kw) -> Params:
    p = Params()
    lib().icp_params_default(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def config(**kw) -> HipConfig:
    """icp_hip_config with the library defaults, then the given fields."""
    c = HipConfig()
    lib().icp_hip_config_default(C.byref(c))
    for k, v in kw.items():
        if not hasattr(c, k):
            raise KeyError(f"icp_hip_config has no field {k!r}")
        setattr(c, k, v)
    return c


class Context:
    """One GPU context (icp_hip_ctx) — see include/icp_hip.h. `cfg` is an icp_hip_config (or a
    dict of its fields); None = the library defaults."""

    def __init__(self, device: int = 0, cfg=None, devices=None, transport: int = XPORT_AUTO):
        """devices = a list of HIP ordinals: one context over all of them (icp_hip_create_multi)."""
        self._h = C.c_void_p()
        if isinstance(cfg, dict):
            cfg = config(**cfg)
        if devices is not None:
            ids = (C.c_int32 * len(devices))(*devices)
            _check(lib().icp_hip_create_multi(C.byref(self._h), len(devices), ids,
                                              None if cfg is None else C.byref(cfg), transport))
        elif cfg is None:
            _check(lib().icp_hip_create(C.byref(self._h), device))
        else:
            _check(lib().icp_hip_create_ex(C.byref(self._h), device, C.byref(cfg)))
        self.n_src = 0

    def close(self):
        if self._h:
            lib().icp_hip_destroy(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def devices(self):
        """(device ids, transport) of this context (ICP_XPORT_*)."""
        n, tr = C.c_int32(), C.c_int32()
        ids = (C.c_int32 * 64)()
        _check(lib().icp_hip_ctx_devices(self._h, C.byref(n), ids, 64, C.byref(tr)))
        return [ids[k] for k in range(n.value)], tr.value

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        _check(lib().icp_hip_get_unique_id(buf))
        return buf.raw

    def comm_init(self, nranks: int, rank: int, uid: bytes):
        _check(lib().icp_hip_comm_init(self._h, nranks, rank, C.c_char_p(bytes(uid))))

    def comm_init_host(self, nranks: int, rank: int, exchange):
        """Multi-rank with the all-gathers done by `exchange(local) -> (nranks, count) array`
        (rank order) instead of RCCL (icp_hip_comm_init_host): rehearses several ranks on one GPU."""
        def _cb(_user, local, count, gathered):
            try:
                loc = np.ctypeslib.as_array(local, shape=(count,)).copy()
                out = np.ascontiguousarray(exchange(loc), dtype=np.float64).reshape(-1)
                if out.shape[0] != nranks * count:
                    return 1
                C.memmove(gathered, out.ctypes.data, out.nbytes)
                return 0
            except Exception:
                return 1
        new_cb = _EXCHANGE_FN(_cb)
        # the previous callback may still run on the context's exchange thread (abandoned at the
        # deadline) until icp_hip_comm_init_host joins it: its thunk stays alive for the whole
        # call, and for the context's life (retired callbacks are kept until close)
        if getattr(self, "_xcb", None) is not None:
            self._xcb_retired = getattr(self, "_xcb_retired", []) + [self._xcb]
        rc = lib().icp_hip_comm_init_host(self._h, nranks, rank, C.cast(new_cb, C.c_void_p), None)
        self._xcb = new_cb  # kept alive as long as the context
        _check(rc)

    def set_target(self, xyz, max_points=10, max_depth=20, rules=RULES_ENGINE):
        xyz = _aos(xyz)
        _check(lib().icp_hip_set_target(self._h, _ptr(xyz), xyz.shape[0], max_points, max_depth, rules))
        self._n_tgt = xyz.shape[0]

    def set_source(self, xyz):
        xyz = _aos(xyz)
        _check(lib().icp_hip_set_source(self._h, _ptr(xyz), xyz.shape[0]))
        self.n_src = xyz.shape[0]

    def iterate(self, T_apply=None, iteration=0, rules=RULES_ENGINE, sigma=3.0) -> IterStats:
        st = IterStats()
        T = None if T_apply is None else np.ascontiguousarray(T_apply, dtype=np.float64).reshape(16)
        _check(lib().icp_hip_iterate(self._h, _ptr(T), iteration, rules, sigma, C.byref(st)))
        return st

    def apply(self, T):
        T = np.ascontiguousarray(T, dtype=np.float64).reshape(16)
        _check(lib().icp_hip_apply(self._h, _ptr(T)))

    def get_source(self) -> np.ndarray:
        out = np.empty((self.n_src, 3), np.float64)
        _check(lib().icp_hip_get_source(self._h, _ptr(out)))
        return out

    def get_correspondences(self):
        idx = np.empty(self.n_src, np.int32)
        d = np.empty(self.n_src, np.float64)
        _check(lib().icp_hip_get_correspondences(self._h, _ptr(idx), _ptr(d)))
        return idx, d

    def nn(self, q):
        q = _aos(q)
        idx = np.empty(q.shape[0], np.int32)
        d = np.empty(q.shape[0], np.float64)
        _check(lib().icp_hip_nn(self._h, _ptr(q), q.shape[0], _ptr(idx), _ptr(d)))
        return idx, d

    def traversal_counts(self):
        a, b = C.c_double(), C.c_double()
        _check(lib().icp_hip_traversal_counts(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def target_info(self):
        nn_, nl = C.c_int64(), C.c_int64()
        md, lv = C.c_int32(), C.c_int32()
        _check(lib().icp_hip_target_info(self._h, C.byref(nn_), C.byref(nl), C.byref(md), C.byref(lv)))
        return {"n_nodes": nn_.value, "n_leaves": nl.value, "max_depth": md.value, "stack_levels": lv.value}

    def target_build_info(self):
        """(built on the device?, set_target milliseconds on the context stream)."""
        od, ms = C.c_int32(), C.c_double()
        _check(lib().icp_hip_target_build_info(self._h, C.byref(od), C.byref(ms)))
        return bool(od.value), ms.value

    def copy_target(self) -> dict:
        """The resident octree, in the layout of octree_build() (host builder)."""
        info = self.target_info()
        nn_ = info["n_nodes"]
        npts = self._n_tgt
        box = np.empty((nn_, 6))
        first = np.empty(nn_, np.int32)
        meta = np.empty(nn_, np.uint32)
        depth = np.empty(nn_, np.int32)
        pts = np.empty((npts, 3))
        orig = np.empty(npts, np.int32)
        _check(lib().icp_hip_copy_target(self._h, _ptr(box), _ptr(first), _ptr(meta), _ptr(depth), _ptr(pts),
                                         _ptr(orig)))
        return {"box": box, "first": first, "meta": meta, "depth": depth, "pts": pts, "orig": orig,
                "n_leaves": info["n_leaves"], "max_depth": info["max_depth"]}

    def target_separation(self) -> np.ndarray:
        """Per target point (caller's order): lower bound of its distance to every other point."""
        out = np.empty(self._n_tgt, np.float32)
        _check(lib().icp_hip_target_separation(self._h, _ptr(out)))
        return out

    def last_timing(self):
        a, b = C.c_double(), C.c_double()
        _check(lib().icp_hip_last_timing(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def last_cull_path(self) -> int:
        """1: the last iterate's covariance sums came from the wave search's records + the band
        pairs; 0: a full cull pass (icp_hip_last_cull_path)."""
        f = C.c_int32()
        _check(lib().icp_hip_last_cull_path(self._h, C.byref(f)))
        return f.value

    def timings(self, k: int):
        """(search kernel ms, iterate device ms) of each of the last k iterates, oldest first."""
        a, b = np.zeros(k), np.zeros(k)
        _check(lib().icp_hip_timings(self._h, k, _ptr(a), _ptr(b)))
        return a, b

    def exchange_timings(self, k: int):
        """ms of the two record all-gathers of each of the last k iterates (NaN: not timed)."""
        a = np.zeros(k)
        _check(lib().icp_hip_exchange_timings(self._h, k, _ptr(a)))
        return a

    def comm_info(self, member: int = 0) -> dict:
        """The communicator of member `member` as RCCL reports it (icp_hip_comm_info)."""
        n, r, d, t = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
        _check(lib().icp_hip_comm_info(self._h, member, C.byref(n), C.byref(r), C.byref(d), C.byref(t)))
        return {"count": n.value, "rank": r.value, "device": d.value, "transport": t.value}

    def synchronize(self):
        _check(lib().icp_hip_synchronize(self._h))

    def comm_abort(self):
        """Abort this rank's RCCL communicator (icp_hip_comm_abort)."""
        _check(lib().icp_hip_comm_abort(self._h))

    def inject_failure(self, member: int = 0, where: int = 1):
        """Testing hook: member's next iterate fails before its first record exchange."""
        _check(lib().icp_hip_debug_inject_failure(self._h, member, where))

    def debug_counters(self) -> dict:
        """The wave search's diagnostic counters of the last iterate (needs debug_counters=1)."""
        out = np.zeros(DBG_SLOTS, np.uint64)
        _check(lib().icp_hip_debug_counters(self._h, _ptr(out)))
        return {name: int(out[k]) for k, name in DBG_NAMES.items()}

    def session(self, params: Params) -> "Session":
        return Session(self, params)

    def run(self, params: Params, history_cap: int = 1024):
        res = Result()
        hist = (IterationRecord * max(1, history_cap))()
        rc = lib().icp_engine_run(self._h, C.byref(params), C.byref(res), hist, history_cap, None)
        return rc, res, [hist[k] for k in range(res.n_history)]


class Session:
    """Steppable ICP loop on a context (icp_session_*): one step = one reference loop body."""

    def __init__(self, ctx: Context, params: Params):
        self._ctx = ctx  # keep alive
        self._h = C.c_void_p()
        _check(lib().icp_session_create(ctx.handle, C.byref(params), None, C.byref(self._h)))
        self.done = False

    def step(self):
        rec = IterationRecord()
        produced, done = C.c_int32(0), C.c_int32(0)
        rc = lib().icp_session_step(self._h, C.byref(rec), C.byref(produced), C.byref(done))
        self.done = bool(done.value)
        _check(rc)
        return rec if produced.value else None

    def step_n(self, k: int) -> int:
        """Up to k steps in one native call (no records); returns the steps taken."""
        if not hasattr(lib(), "icp_session_step_n"):  # an older build under A/B
            taken = 0
            while taken < k and not self.done:
                self.step()
                taken += 1
            return taken
        n, done = C.c_int32(0), C.c_int32(0)
        rc = lib().icp_session_step_n(self._h, k, C.byref(n), C.byref(done))
        self.done = bool(done.value)
        _check(rc)
        return n.value

    def step_n_timed(self, k: int) -> np.ndarray:
        """Up to k steps in one native call; returns each step's host wall time (ms)."""
        ms = np.zeros(max(1, k))
        n, done = C.c_int32(0), C.c_int32(0)
        rc = lib().icp_session_step_n_timed(self._h, k, C.byref(n), C.byref(done), _ptr(ms))
        self.done = bool(done.value)
        _check(rc)
        return ms[: n.value]

    def transform(self) -> np.ndarray:
        T = np.empty(16)
        lib().icp_session_transform(self._h, _ptr(T))
        return T.reshape(4, 4)

    def finish(self):
        res = Result()
        rc = lib().icp_session_finish(self._h, C.byref(res))
        return rc, res

    def close(self):
        if self._h:
            lib().icp_session_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def engine_register(params: Params, src, tgt, device: int = -1, history_cap: int = 1024, stop_flag=None,
                    on_log=None, on_progress=None, stop_at: int = -1, devices=None):
    """ICPEngine::registerPointClouds drop-in. Returns (rc, result, history, src_out).
    stop_at >= 0 raises the stop flag from the progress hook of that iteration (the reference's
    cross-thread ICPEngine::stop(), checked at the next iteration, icpengine.cpp:160)."""
    src = _aos(src).copy()
    tgt = _aos(tgt)
    res = Result()
    hist = (IterationRecord * max(1, history_cap))()
    hooks = None
    keep = []
    if stop_at >= 0 and stop_flag is None:
        stop_flag = C.c_int32(0)
    if stop_flag is not None or on_log is not None or on_progress is not None:
        hooks = Hooks()
        if stop_flag is not None:
            hooks.stop_flag = C.cast(C.addressof(stop_flag), C.POINTER(C.c_int32))
        if on_log is not None:
            cb = LOG_CB(lambda u, m: on_log(m.decode(errors="replace")))
            keep.append(cb)
            hooks.on_log = cb
        if on_progress is not None or stop_at >= 0:
            def _progress(_u, it, total, rmse):
                if on_progress is not None:
                    on_progress(it, total, rmse)
                if stop_at >= 0 and it == stop_at:
                    stop_flag.value = 1
            pcb = PROGRESS_CB(_progress)
            keep.append(pcb)
            hooks.on_progress = pcb
    devs = [device] if devices is None else list(devices)
    ids = (C.c_int32 * len(devs))(*devs)
    rc = lib().icp_engine_register_devices(C.byref(params), _ptr(src), src.shape[0], _ptr(tgt), tgt.shape[0],
                                           len(devs), ids, C.byref(res), hist, history_cap,
                                           C.byref(hooks) if hooks else None)
    return rc, res, [hist[k] for k in range(res.n_history)], src


def cli_icp(src, tgt, max_iterations=20, tolerance=1e-2, device: int = -1, devices=None):
    """ICP() of icp_registration.cpp drop-in. Returns (R, t, transforms, src_out)."""
    src = _aos(src).copy()
    tgt = _aos(tgt)
    R = np.zeros(9)
    t = np.zeros(3)
    cap = max(1, max_iterations)
    tr = np.zeros((cap, 16))
    n = C.c_int32()
    devs = [device] if devices is None else list(devices)
    ids = (C.c_int32 * len(devs))(*devs)
    _check(lib().icp_cli_icp_devices(_ptr(src), src.shape[0], _ptr(tgt), tgt.shape[0], max_iterations, tolerance,
                                     _ptr(R), _ptr(t), _ptr(tr), cap, C.byref(n), len(devs), ids))
    return R.reshape(3, 3), t, tr[: n.value].reshape(-1, 4, 4), src


def source_shard_order(xyz: np.ndarray) -> np.ndarray:
    """Permutation whose contiguous ranges are spatially compact (icp_source_shard_order): rank r
    of W takes xyz[order[lo:hi]] for its balanced contiguous range."""
    xyz = np.ascontiguousarray(xyz, dtype=np.float64)
    order = np.empty(len(xyz), np.int32)
    rc = lib().icp_source_shard_order(_ptr(xyz), len(xyz), _ptr(order))
    if rc != 0:
        raise IcpError(rc, lib().icp_hip_last_error().decode())
    return order


def synth_pair(n_tgt: int, n_src: int | None = None, **overrides):
    spec = SynthSpec()
    lib().icp_synth_default(C.byref(spec))
    for k, v in overrides.items():
        if k in ("sigma", "t"):
            getattr(spec, k)[:] = list(v)
        else:
            setattr(spec, k, v)
    n_src = n_tgt if n_src is None else n_src
    tgt = np.empty((n_tgt, 3))
    src = np.empty((n_src, 3))
    T = np.empty(16)
    _check(lib().icp_synth_pair(C.byref(spec), n_tgt, n_src, _ptr(tgt), _ptr(src), _ptr(T)))
    return tgt, src, T.reshape(4, 4)


def synth_scene(n_tgt: int, n_src: int | None = None, **overrides):
    """A LiDAR-like scene pair (icp_synth_scene, include/icp_host.h): ground + walls scanned from
    two poses, 1 mm grid. Returns (target, source, T_true)."""
    spec = SceneSpec()
    lib().icp_scene_default(C.byref(spec))
    for k, v in overrides.items():
        if k == "t":
            spec.t[:] = list(v)
        else:
            setattr(spec, k, v)
    n_src = n_tgt if n_src is None else n_src
    tgt = np.empty((n_tgt, 3))
    src = np.empty((n_src, 3))
    T = np.empty(16)
    _check(lib().icp_synth_scene(C.byref(spec), n_tgt, n_src, _ptr(tgt), _ptr(src), _ptr(T)))
    return tgt, src, T.reshape(4, 4)


def octree_build(xyz, max_points=10, max_depth=20) -> dict:
    """Host linear-octree build (the exact arrays the device path uploads)."""
    xyz = _aos(xyz)
    h = lib().icp_octree_build(_ptr(xyz), xyz.shape[0], max_points, max_depth)
    if not h:
        raise IcpError(-1, lib().icp_hip_last_error().decode())
    try:
        info = OctreeInfo()
        lib().icp_octree_get_info(h, C.byref(info))
        nn_ = info.n_nodes
        box = np.empty((nn_, 6))
        first = np.empty(nn_, np.int32)
        meta = np.empty(nn_, np.uint32)
        depth = np.empty(nn_, np.int32)
        lib().icp_octree_copy_nodes(h, _ptr(box), _ptr(first), _ptr(meta), _ptr(depth))
        pts = np.empty((info.n_points, 3))
        orig = np.empty(info.n_points, np.int32)
        lib().icp_octree_copy_points(h, _ptr(pts), _ptr(orig))
    finally:
        lib().icp_octree_free(h)
    return {"box": box, "first": first, "meta": meta, "depth": depth, "pts": pts, "orig": orig,
            "n_leaves": info.n_leaves, "max_depth": info.max_depth, "max_inner_depth": info.max_inner_depth,
            "pos_of_orig0": info.pos_of_orig0}


def jacobi_svd3(H):
    H = np.ascontiguousarray(H, np.float64).reshape(9)
    U, S, V = np.empty(9), np.empty(3), np.empty(9)
    lib().icp_jacobi_svd3(_ptr(H), _ptr(U), _ptr(S), _ptr(V))
    return U.reshape(3, 3), S, V.reshape(3, 3)


def best_fit_transform(a, b):
    a, b = _aos(a), _aos(b)
    T = np.empty(16)
    lib().icp_best_fit_transform(_ptr(a), _ptr(b), a.shape[0], _ptr(T))
    return T.reshape(4, 4)


def best_fit_from_stats(st: IterStats):
    T = np.empty(16)
    lib().icp_best_fit_from_stats(C.byref(st), _ptr(T))
    return T.reshape(4, 4)


def moments_from_values(d):
    d = np.ascontiguousarray(d, np.float64)
    out = np.empty(8)
    lib().icp_moments_from_values(_ptr(d), d.shape[0], _ptr(out))
    return out


def moments_merge(parts):
    parts = np.ascontiguousarray(parts, np.float64).reshape(-1, 8)
    out = np.empty(8)
    lib().icp_moments_merge(_ptr(parts), parts.shape[0], _ptr(out))
    return out


def cov_from_pairs(a, b, d, thr):
    a, b = _aos(a), _aos(b)
    d = np.ascontiguousarray(d, np.float64)
    out = np.empty(20)
    lib().icp_cov_from_pairs(_ptr(a), _ptr(b), _ptr(d), d.shape[0], thr, _ptr(out))
    return out


def cov_merge(parts):
    parts = np.ascontiguousarray(parts, np.float64).reshape(-1, 20)
    out = np.empty(20)
    lib().icp_cov_merge(_ptr(parts), parts.shape[0], _ptr(out))
    return out


def cull_threshold(mean, sd, k_sigma, iteration, engine_rules):
    return lib().icp_cull_threshold(mean, sd, k_sigma, iteration, engine_rules)


LAS_CORE = 0
LAS_CLI = 1


def las_read(path, rules=LAS_CLI, max_points=0):
    """Read a LAS 1.2 file (core LASIO::readLAS or CLI readLASFile rules). Returns (xyz, header)."""
    hdr = LasHeader()
    bpath = str(path).encode()
    rc = lib().icp_las_read_header(bpath, rules, C.byref(hdr))
    if rc != 0:
        raise IcpError(rc, f"cannot read LAS header of {path}")
    n = hdr.num_points if max_points <= 0 or rules == LAS_CLI else min(hdr.num_points, max_points)
    xyz = np.empty((max(n, 1), 3))
    got = lib().icp_las_read(bpath, rules, max_points, _ptr(xyz), C.byref(hdr))
    if got < 0:
        raise IcpError(int(got), f"cannot read LAS points of {path}")
    return xyz[:got], hdr


def las_write_core(path, xyz, bounds=None):
    """LASIO::writeLAS. bounds = the caller's PointCloud (minX, maxX, minY, maxY, minZ, maxZ) as they
    stand; None = computeBounds() of xyz."""
    xyz = _aos(xyz)
    if bounds is None:
        rc = lib().icp_las_write_core(str(path).encode(), _ptr(xyz), xyz.shape[0])
    else:
        b = np.ascontiguousarray(bounds, np.float64)
        rc = lib().icp_las_write_core_bounds(str(path).encode(), _ptr(xyz), xyz.shape[0], _ptr(b))
    if rc != 0:
        raise IcpError(rc, f"cannot write {path}")


def las_write_cli(path, xyz, scale=(0.001, 0.001, 0.001), offset=(0.0, 0.0, 0.0)):
    xyz = _aos(xyz)
    sc = np.ascontiguousarray(scale, np.float64)
    of = np.ascontiguousarray(offset, np.float64)
    rc = lib().icp_las_write_cli(str(path).encode(), _ptr(xyz), xyz.shape[0], _ptr(sc), _ptr(of))
    if rc != 0:
        raise IcpError(rc, f"cannot write {path}")


def write_transform_report(path, R, t, transforms=None):
    R = np.ascontiguousarray(R, np.float64).reshape(9)
    t = np.ascontiguousarray(t, np.float64).reshape(3)
    if transforms is None or len(transforms) == 0:
        T, n = None, 0
    else:
        T = np.ascontiguousarray(transforms, np.float64).reshape(-1, 16)
        n = T.shape[0]
    rc = lib().icp_write_transform_report(str(path).encode(), _ptr(R), _ptr(t), _ptr(T), n)
    if rc != 0:
        raise IcpError(rc, f"cannot write {path}")
