"""The process warm-up of icp_hip_create_ex (icp_ctx.hip warm_kernels; icp_hip_config.no_warmup):
a private 3-iterate registration that loads the kernels before the first real iterate. It must
be invisible to the caller: the thread's last error message survives it, a context with a new set
of search options (a new warm-up) and one without the warm-up give the same results as any other."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(icp, cfg, tgt, src):
    with icp.Context(0, cfg) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        T, stats = None, []
        for it in range(3):
            st = ctx.iterate(T, it, icp.RULES_ENGINE, 3.0)
            stats.append((st.valid, st.rmse, tuple(st.H)))
            T = icp.best_fit_from_stats(st)
        idx, d = ctx.get_correspondences()
    return stats, idx, d


def test_warmup_is_invisible(icp):
    tgt, src, _ = icp.synth_pair(50_000, yaw_deg=3.0)
    L = icp.lib()
    # an error left by an earlier call survives a context creation that warms a new option set
    with pytest.raises(icp.IcpError):
        icp.Context(0, icp.config(scan_groups=3))
    msg = L.icp_hip_last_error().decode()
    assert "scan_groups" in msg
    with icp.Context(0, icp.config(scan_groups=2, join_factor=3.0)):
        assert L.icp_hip_last_error().decode() == msg
    a = _run(icp, icp.config(scan_groups=2), tgt, src)   # warmed (the option set above)
    b = _run(icp, icp.config(scan_groups=2, no_warmup=1), tgt, src)
    c = _run(icp, icp.config(), tgt, src)               # the default set (warmed by an earlier test or now)
    assert a[0] == b[0]
    for k in (1, 2):
        np.testing.assert_array_equal(a[k], b[k])
        np.testing.assert_array_equal(a[k], c[k])
