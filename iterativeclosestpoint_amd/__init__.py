"""iterativeclosestpoint_amd — MI355X-native ICP correspondence-and-alignment path.

The product is the C-ABI shared library ``libicp_hip.so`` (HIP kernels for gfx950 + C++ host
driver, declared in ``include/icp_hip.h``, ``include/icp_engine.h``, ``include/icp_host.h``, ``include/icp_las.h``).
This package is only the Python harness binding of that library (ctypes), used by the tests
and ``bench.py``. There is no CPU fallback: if the library is missing the import of
``lib()`` raises, and every device call fails loudly when no GPU is present.
"""
from ._lib import (  # noqa: F401
    LIB_PATH,
    IcpError,
    Context,
    HipConfig,
    config,
    lib,
    build,
    params_default,
    engine_register,
    cli_icp,
    source_shard_order,
    synth_pair,
    octree_build,
    jacobi_svd3,
    best_fit_transform,
    best_fit_from_stats,
    moments_from_values,
    moments_merge,
    cov_from_pairs,
    cov_merge,
    cull_threshold,
    las_read,
    las_write_core,
    las_write_cli,
    write_transform_report,
    LAS_CORE,
    LAS_CLI,
    RULES_ENGINE,
    RULES_CLI,
    FLAG_NO_EARLY_STOP,
    SEARCH_CERTIFIED,
    SEARCH_REFERENCE,
    BUILD_AUTO,
    BUILD_HOST,
    XPORT_AUTO,
    XPORT_RCCL,
    XPORT_HOST,
    XPORT_CALLBACK,
    DBG_NAMES,
)
