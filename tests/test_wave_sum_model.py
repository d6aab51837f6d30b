"""A lane-level model of the wave search's record reduction (iterativeclosestpoint_amd/csrc/
wave_stats.h wave_sum16) on the CPU: the gfx950 permlane swaps as the header documents them, the
XOR-swizzled LDS stage, the quarter adds. Checks that every lane ends with the full 64-lane sum of
the value it owns (lane & 15) and that the four lanes owning a value agree bit for bit. With
integer-valued terms the sums are exact, so any lane routed twice or dropped shows up.
(The GPU parity of the sums themselves: tests/test_gpu_fused_cull.py.)
"""
import numpy as np


def swap32(x, y):
    # v_permlane32_swap: x' = [x lanes 0-31, y lanes 0-31], y' = [x lanes 32-63, y lanes 32-63]
    return np.concatenate([x[:32], y[:32]]), np.concatenate([x[32:], y[32:]])


def swap16(x, y):
    # v_permlane16_swap: x' = rows [x0, y0, x2, y2], y' = rows [x1, y1, x3, y3]
    r = lambda a, k: a[16 * k:16 * k + 16]  # noqa: E731
    return (np.concatenate([r(x, 0), r(y, 0), r(x, 2), r(y, 2)]),
            np.concatenate([r(x, 1), r(y, 1), r(x, 3), r(y, 3)]))


def wave_sum16(c):
    """c: 16 x 64 array (value k of lane l at c[k, l]); returns the 64 lanes' results."""
    c = [c[k].copy() for k in range(16)]
    for k in range(8):
        c[k], c[k + 8] = swap32(c[k], c[k + 8])
        c[k] = c[k] + c[k + 8]
    for k in range(4):
        c[k], c[k + 4] = swap16(c[k], c[k + 4])
        c[k] = c[k] + c[k + 4]
    lds = np.full(256, np.nan)
    lanes = np.arange(64)
    for j in range(4):
        lds[64 * j + (lanes ^ (4 * j + (lanes >> 4)))] = c[j]
    v, q = lanes & 15, lanes >> 4
    vr, vj = v >> 2, v & 3
    key = 4 * vj + vr
    s0 = 16 * vr + 4 * q
    g = lds[64 * vj + (s0 ^ key)]
    for i in range(1, 4):
        g = g + lds[64 * vj + ((s0 + i) ^ key)]
    h = g.copy()
    g, h = swap32(g, h)
    g = g + h
    h = g.copy()
    g, h = swap16(g, h)
    return g + h


def test_every_lane_gets_the_full_sum_of_its_value():
    rng = np.random.default_rng(3)
    for _ in range(20):
        c = rng.integers(-2 ** 20, 2 ** 20, size=(16, 64)).astype(np.float64)
        out = wave_sum16(c)
        want = c.sum(axis=1)
        np.testing.assert_array_equal(out, want[np.arange(64) & 15])


def test_each_term_counted_once():
    # one-hot terms: lane l's value k = 2^(k) * (l + 1) exactly representable, sums exact
    c = np.zeros((16, 64))
    for k in range(16):
        for lane in range(64):
            c[k, lane] = float(lane + 1) * (1 << k)
    out = wave_sum16(c)
    for lane in range(64):
        assert out[lane] == 2080.0 * (1 << (lane & 15))  # sum of 1..64 = 2080


def test_lds_layout_is_a_permutation_and_spreads_banks():
    lanes = np.arange(64)
    for j in range(4):
        idx = lanes ^ (4 * j + (lanes >> 4))
        assert sorted(idx) == list(range(64))
    # one read step: the 64 addresses fall on 16 distinct 8-B slots mod 128 B (4 lanes each)
    v, q = lanes & 15, lanes >> 4
    vr, vj = v >> 2, v & 3
    for i in range(4):
        addr = 64 * vj + ((16 * vr + 4 * q + i) ^ (4 * vj + vr))
        slots = addr % 16
        assert np.bincount(slots, minlength=16).tolist() == [4] * 16
