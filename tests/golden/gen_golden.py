#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE ITSELF.

The reference (B1AnKAlpha/IterativeClosestPoint) ships no tests, fixtures or golden data
(SURVEY.md §4), so every vector here is produced in this container by the compiled
reference: oracle/_ref/libicp_ref.so = /root/reference/icp_registration.cpp + its vendored
Eigen 3.3.4, built by oracle/Makefile (`make -C oracle ref`), and oracle/_ref/libicp_ref_engine.so
= the core engine and LAS I/O (PointCloudRegistration/core, moc + the image's conda Qt 5.9.7,
`make -C oracle refqt`). Inputs come from the product's
deterministic generator (icp_synth_pair) or from numpy with fixed seeds, and are stored
alongside (or as hashes, for the 100k case).

Run from the repo root:  python tests/golden/gen_golden.py [--only-engine | --only-las | --only-scene]
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import oracle_py as O  # noqa: E402
import iterativeclosestpoint_amd as icp  # noqa: E402

OUT = Path(__file__).resolve().parent


def fnv1a(a: np.ndarray) -> str:
    h = 0xCBF29CE484222325
    for b in np.ascontiguousarray(a).tobytes():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


def nn_known_answers():
    """(iii) NN known-answer sets: split planes, duplicates beyond leaf capacity, ties, far queries."""
    rng = np.random.default_rng(7)
    cases = {}
    # a) Gaussian target, random + jittered-target queries
    t = rng.normal(size=(8000, 3)) * [5, 5, 1]
    q = np.concatenate([rng.normal(size=(3000, 3)) * [6, 6, 1.5], t[:1000] + rng.normal(size=(1000, 3)) * 1e-3])
    cases["gauss"] = (t, q)
    # b) integer lattice: many exact ties and points on split planes
    g = np.stack(np.meshgrid(np.arange(12), np.arange(12), np.arange(6), indexing="ij"), -1).reshape(-1, 3).astype(float)
    q = np.concatenate([g[rng.integers(0, len(g), 500)] + 0.5, rng.integers(-1, 13, size=(500, 3)).astype(float),
                        g[rng.integers(0, len(g), 200)]])
    cases["lattice"] = (g, q)
    # c) heavy duplicates: 300 copies of a few points force leaves at max depth (> max_pts)
    base = rng.normal(size=(5, 3))
    dup = np.concatenate([np.repeat(base, 300, axis=0), rng.normal(size=(2000, 3)) * 3])
    q = np.concatenate([base + 1e-9, rng.normal(size=(1000, 3)) * 3])
    cases["duplicates"] = (dup, q)
    # d) far-away queries (> 1e10): the CLI's 1e20 initial best (icp_registration.cpp:201) keeps
    #    index 0 where the engine's DBL_MAX (octree.cpp:180) finds the true nearest
    t = rng.normal(size=(2000, 3))
    q = np.concatenate([rng.normal(size=(50, 3)) * 1e11, rng.normal(size=(50, 3))])
    cases["far"] = (t, q)
    # e) tiny targets: single point, root leaf (<= 10 points)
    t = rng.normal(size=(1, 3))
    cases["single"] = (t, rng.normal(size=(20, 3)))
    t = rng.normal(size=(7, 3))
    cases["root_leaf"] = (t, rng.normal(size=(50, 3)))
    arrays = {}
    meta = {}
    for name, (t, q) in cases.items():
        t = np.ascontiguousarray(t, np.float64)
        q = np.ascontiguousarray(q, np.float64)
        ref_idx = O.RefTree(t).nn(q)  # reference CLI octree, init 1e20, (10, 20)
        arrays[f"{name}_target"] = t
        arrays[f"{name}_query"] = q
        arrays[f"{name}_idx_cli"] = ref_idx
        # residual as the reference computes it: distance(src, target[idx]) (icp_registration.cpp:506)
        d = np.array([O.reference().ref_distance(np.ascontiguousarray(q[i]).ctypes.data_as(O.C.c_void_p),
                                                 np.ascontiguousarray(t[ref_idx[i]]).ctypes.data_as(O.C.c_void_p))
                      for i in range(len(q))])
        arrays[f"{name}_dist_cli"] = d
        meta[name] = {"n_target": len(t), "n_query": len(q)}
    # max_depth / max_points variants on the Gaussian set (the GUI range, settingspage.cpp:53-76)
    t, q = cases["gauss"]
    for mp, md in [(5, 10), (100, 50), (10, 3)]:
        arrays[f"gauss_idx_cli_p{mp}_d{md}"] = O.RefTree(t, mp, md).nn(q)
    np.savez_compressed(OUT / "nn_known_answers.npz", **arrays)
    return meta


def svd_and_transform():
    rng = np.random.default_rng(11)
    Hs = [rng.normal(size=(3, 3)) for _ in range(40)]
    Hs += [np.diag(rng.normal(size=3)) for _ in range(4)]
    Hs += [np.outer(rng.normal(size=3), rng.normal(size=3)) for _ in range(4)]  # rank 1
    Hs += [np.zeros((3, 3)), np.eye(3), -np.eye(3), np.diag([1.0, 1.0, -1.0])]
    Hs += [rng.normal(size=(3, 3)) * 1e8, rng.normal(size=(3, 3)) * 1e-8]
    Hs = np.array(Hs)
    fixed = [O.ref_svd3(H, False) for H in Hs]
    dyn = [O.ref_svd3(H, True) for H in Hs]
    # best_fit_transform on point sets (icp_registration.cpp:389-440)
    A = [rng.normal(size=(n, 3)) * [5, 5, 1] + rng.normal(size=3) * 100 for n in (3, 10, 500, 5000)]
    B = []
    for a in A:
        ang = rng.uniform(-0.2, 0.2)
        R = np.array([[np.cos(ang), -np.sin(ang), 0], [np.sin(ang), np.cos(ang), 0], [0, 0, 1]])
        B.append(a @ R.T + rng.normal(size=3) + rng.normal(size=a.shape) * 1e-3)
    # reflection case: mirrored set
    a = rng.normal(size=(50, 3))
    A.append(a)
    B.append(a * [1, 1, -1])
    Tbf = [O.ref_best_fit(a, b) for a, b in zip(A, B)]
    # Eigen T * src (4xN) and T * T_cum bits
    T = np.eye(4)
    T[:3, :3] = np.linalg.qr(rng.normal(size=(3, 3)))[0]
    T[:3, 3] = rng.normal(size=3) * 10
    pts = rng.normal(size=(4000, 3)) * [50, 50, 5] + [1e5, -2e5, 30]
    tp = O.ref_transform(T, pts)
    T2 = np.eye(4)
    T2[:3, :3] = np.linalg.qr(rng.normal(size=(3, 3)))[0]
    T2[:3, 3] = rng.normal(size=3)
    mm = O.ref_mat4_mul(T, T2)
    arrays = {
        "H": Hs,
        "U_fixed": np.array([f[0] for f in fixed]), "S_fixed": np.array([f[1] for f in fixed]),
        "V_fixed": np.array([f[2] for f in fixed]),
        "U_dyn": np.array([f[0] for f in dyn]), "S_dyn": np.array([f[1] for f in dyn]),
        "V_dyn": np.array([f[2] for f in dyn]),
        "T": T, "T2": T2, "pts": pts, "T_pts": tp, "T_T2": mm,
        "T_bestfit": np.array(Tbf),
    }
    for k, (a, b) in enumerate(zip(A, B)):
        arrays[f"bf_A{k}"] = a
        arrays[f"bf_B{k}"] = b
    np.savez_compressed(OUT / "svd_transform.npz", **arrays)
    return {"n_H": len(Hs), "n_bestfit": len(A)}


def icp_cli_cases():
    """(i)/(ii): the reference CLI ICP() end to end on config-1 and 10k pairs."""
    rng = np.random.default_rng(2024)
    out = {}
    arrays = {}
    # config 1: test_icp.cpp-style random R (<= 10 deg) and t (+-2.5 m xy, +-1 m z) (test_icp.cpp:165-229)
    angle = rng.uniform() * 10.0
    yaw, pitch, roll = angle, (rng.uniform() - 0.5) * angle, (rng.uniform() - 0.5) * angle
    t = [(rng.uniform() - 0.5) * 5, (rng.uniform() - 0.5) * 5, (rng.uniform() - 0.5) * 2]
    specs = {
        "cfg1_1k": dict(n=1000, yaw_deg=yaw, pitch_deg=pitch, roll_deg=roll, t=t, iters=20, tol=1e-2),
        "g10k": dict(n=10000, yaw_deg=3.0, pitch_deg=1.0, roll_deg=-0.5, t=[0.3, -0.2, 0.05], iters=30, tol=1e-9),
    }
    for name, sp in specs.items():
        tgt, src, Ttrue = icp.synth_pair(sp["n"], yaw_deg=sp["yaw_deg"], pitch_deg=sp["pitch_deg"],
                                         roll_deg=sp["roll_deg"], t=sp["t"])
        R, tt, tcums, src_out = O.ref_icp_cli(src, tgt, sp["iters"], sp["tol"])
        idx0 = O.RefTree(tgt).nn(src)
        arrays[f"{name}_target"] = tgt
        arrays[f"{name}_source"] = src
        arrays[f"{name}_T_true"] = Ttrue
        arrays[f"{name}_R_final"] = R
        arrays[f"{name}_t_final"] = tt
        arrays[f"{name}_T_cums"] = tcums
        arrays[f"{name}_source_out"] = src_out
        arrays[f"{name}_idx_iter0"] = idx0
        out[name] = {"n": sp["n"], "iterations": sp["iters"], "tolerance": sp["tol"],
                     "n_transforms": int(len(tcums)), "synth": {k: v for k, v in sp.items() if k not in ("n",)}}
    np.savez_compressed(OUT / "icp_cli.npz", **arrays)
    return out


def nn_100k_hashes():
    """(ii) 100k Gaussian pair: inputs regenerated by icp_synth_pair; reference indices hashed."""
    tgt, src, _ = icp.synth_pair(100000)
    idx = O.RefTree(tgt).nn(src)
    tree = O.OracleTree(tgt)
    _, _, visits, scanned = tree.nn(src, count=True)
    return {"n": 100000, "target_fnv1a": fnv1a(tgt), "source_fnv1a": fnv1a(src), "idx_fnv1a": fnv1a(idx),
            "idx_sum": int(idx.astype(np.int64).sum()), "mean_node_entries": visits / len(src),
            "mean_leaf_points": scanned / len(src)}


def las_and_report():
    """(f1) LAS 1.2 writer/reader and the transformation report of the reference CLI.

    saveResultAsLAS / readLASFile / saveTransformation (icp_registration.cpp:625-815, :248-378),
    run by the compiled reference CLI. The core LASIO (core/lasio.cpp, built against the image's
    Qt 5.9.7 by oracle/Makefile's refqt target) has fixtures of its own: core_las() below."""
    import tempfile
    rng = np.random.default_rng(77)
    n = 12345  # > one 10000-record batch, ragged tail
    xyz = np.stack([rng.normal(0, 30, n) - 5.0, rng.normal(0, 20, n) + 7.0, rng.normal(0, 3, n)], 1)
    xyz[:4] = [[0.0, 0.0, 0.0], [-0.0049999, 0.0049999, -1e-9], [-123.4567891, 98.7654321, -0.0051], [1e3, -1e3, 5.0]]
    scale = np.array([0.01, 0.01, 0.005])
    offset = np.array([100.0, -50.0, 3.0])
    arrays = {"las_points": xyz, "las_scale": scale, "las_offset": offset}
    with tempfile.TemporaryDirectory() as d:
        f = Path(d) / "w.las"
        O.ref_save_las(f, xyz, scale, offset)
        blob = f.read_bytes()
        arrays["las_file"] = np.frombuffer(blob, np.uint8)
        rd, so = O.ref_read_las(f)
        arrays["las_read"] = rd
        arrays["las_read_so"] = so
        # truncated file: header claims n points, data stops mid-record in the second batch
        cut = 227 + 20 * 10007 + 7
        (Path(d) / "t.las").write_bytes(blob[:cut])
        rt, _ = O.ref_read_las(Path(d) / "t.las")
        arrays["las_trunc_cut"] = np.array([cut])
        arrays["las_trunc_read"] = rt
        # the reference rejects 0 points (readLASFile :291)
        z = bytearray(blob[:227])
        z[107:111] = (0).to_bytes(4, "little")
        (Path(d) / "z.las").write_bytes(bytes(z))
        rz, _ = O.ref_read_las(Path(d) / "z.las")
        arrays["las_zero_rejected"] = np.array([rz is None])
        # transformation report: with and without the per-iteration list
        R = np.array([[0.9961946981, -0.0871557427, 0.0], [0.0871557427, 0.9961946981, 0.0], [0.0, 0.0, 1.0]])
        R = R + rng.normal(0, 1e-7, (3, 3))
        t = np.array([0.5, -0.3, 1.0 / 3.0])
        Ts = np.stack([np.eye(4) + rng.normal(0, 1e-3, (4, 4)) for _ in range(3)])
        Ts[:, 3] = [0, 0, 0, 1]
        arrays["rep_R"], arrays["rep_t"], arrays["rep_T"] = R, t, Ts
        O.ref_save_transformation(Path(d) / "r1.txt", R, t, Ts)
        O.ref_save_transformation(Path(d) / "r0.txt", R, t, np.zeros((0, 16)))
        arrays["rep_with_iters"] = np.frombuffer((Path(d) / "r1.txt").read_bytes(), np.uint8)
        arrays["rep_final_only"] = np.frombuffer((Path(d) / "r0.txt").read_bytes(), np.uint8)
    np.savez_compressed(OUT / "las_report.npz", **arrays)
    return {"n": n, "file_bytes": len(blob), "file_fnv1a": fnv1a(arrays["las_file"]), "trunc_cut": cut}


def _divergent_pair():
    """Unstructured clouds on which the reference engine stops on 'rmse > 1.1 prev'
    (icpengine.cpp:311-314): the first such draw of a fixed-seed search."""
    rng = np.random.default_rng(1)
    for _ in range(2000):
        n = int(rng.integers(50, 400))
        tgt = rng.uniform(-1, 1, size=(n, 3)) * rng.uniform(0.2, 5, 3)
        m = int(rng.integers(20, 400))
        src = rng.uniform(-1, 1, size=(m, 3)) * rng.uniform(0.2, 5, 3) + rng.normal(size=3)
        sig = float(rng.choice([0.5, 1.0, 2.0, 3.0]))
        r = O.ref_engine_register(src, tgt, 50, 1e-6, sig)
        if r["finished"] == 1 and r["total_iterations"] < 50 and not np.isnan(r["history"][-1][20]):
            # ended early without the convergence record: the divergence break
            return src, tgt, sig
    raise RuntimeError("no divergent pair found")


def engine_cases():
    """The engine rules, run by the REAL core engine (core/icpengine.cpp + octree.cpp, moc, conda
    Qt 5.9.7: oracle/_ref/libicp_ref_engine.so). Each case pins rules the CLI fixtures cannot:
      e1k       test_icp-style 1k pair, default ICPParameters (icpengine.h:13-19)
      e10k      10k pair to convergence: the extra convergence record with T_cumulative
                (icpengine.cpp:293-303), final R/t = T_cumulative (:378-383)
      far       far source points (> 1e10): DBL_MAX initial best (octree.cpp:180)
      relaxed   near-constant residuals: the relaxed iteration-0 threshold mean + max(k std,
                0.5 mean) (icpengine.cpp:249-252) keeps every pair
      params    octreeMaxPoints 5, octreeMaxDepth 10, sigmaMultiplier 2
      diverge   'error increased' break (icpengine.cpp:311-314): success with write-back
      too_few   2 source points: finished(false) without write-back (icpengine.cpp:319-323)
      cancel    ICPEngine::stop() during iteration 3: finished(false) at the next check
                (icpengine.cpp:160-164), no write-back"""
    rng = np.random.default_rng(4242)
    cases = {}
    angle = rng.uniform() * 10.0
    cases["e1k"] = dict(synth=dict(n=1000, yaw_deg=angle, pitch_deg=(rng.uniform() - 0.5) * angle,
                                   roll_deg=(rng.uniform() - 0.5) * angle,
                                   t=[(rng.uniform() - 0.5) * 5, (rng.uniform() - 0.5) * 5, (rng.uniform() - 0.5) * 2]),
                        params=dict(max_iterations=50, tolerance=1e-6, sigma=3.0, max_points=10, max_depth=20))
    cases["e10k"] = dict(synth=dict(n=10000, yaw_deg=4.0, pitch_deg=1.5, roll_deg=-1.0, t=[0.4, -0.25, 0.08]),
                         params=dict(max_iterations=80, tolerance=1e-9, sigma=3.0, max_points=10, max_depth=20))
    t = rng.normal(size=(3000, 3)) * [4, 4, 1]
    s = np.concatenate([t[:1500] + rng.normal(size=(1500, 3)) * 0.01 + [0.05, -0.02, 0.01],
                        rng.normal(size=(4, 3)) * 3e10])
    cases["far"] = dict(src=s, tgt=t, params=dict(max_iterations=10, tolerance=1e-6, sigma=3.0, max_points=10,
                                                  max_depth=20))
    t = rng.uniform(-2, 2, size=(4000, 3))
    s = t[rng.permutation(4000)[:2000]] + [0.01, -0.004, 0.002] + rng.normal(size=(2000, 3)) * 1e-5
    cases["relaxed"] = dict(src=s, tgt=t, params=dict(max_iterations=6, tolerance=1e-6, sigma=3.0, max_points=10,
                                                      max_depth=20))
    cases["params"] = dict(synth=dict(n=6000, yaw_deg=-3.0, pitch_deg=0.5, roll_deg=2.0, t=[-0.2, 0.3, 0.1]),
                           params=dict(max_iterations=25, tolerance=1e-7, sigma=2.0, max_points=5, max_depth=10))
    s, t, sig = _divergent_pair()
    cases["diverge"] = dict(src=s, tgt=t, params=dict(max_iterations=50, tolerance=1e-6, sigma=sig, max_points=10,
                                                      max_depth=20))
    t = rng.normal(size=(100, 3))
    cases["too_few"] = dict(src=t[:2] + 0.01, tgt=t, params=dict(max_iterations=50, tolerance=1e-6, sigma=3.0,
                                                                 max_points=10, max_depth=20))
    cases["cancel"] = dict(synth=dict(n=3000, yaw_deg=5.0, pitch_deg=0.0, roll_deg=0.0, t=[0.3, 0.1, 0.0]),
                           params=dict(max_iterations=50, tolerance=1e-9, sigma=3.0, max_points=10, max_depth=20),
                           stop_at=3)
    arrays, meta = {}, {}
    for name, c in cases.items():
        if "synth" in c:
            sp = c["synth"]
            tgt, src, _ = icp.synth_pair(sp["n"], yaw_deg=sp["yaw_deg"], pitch_deg=sp["pitch_deg"],
                                         roll_deg=sp["roll_deg"], t=sp["t"])
        else:
            src, tgt = np.ascontiguousarray(c["src"]), np.ascontiguousarray(c["tgt"])
        p = c["params"]
        r = O.ref_engine_register(src, tgt, p["max_iterations"], p["tolerance"], p["sigma"], p["max_points"],
                                  p["max_depth"], c.get("stop_at", -1))
        arrays[f"{name}_source"] = src
        arrays[f"{name}_target"] = tgt
        arrays[f"{name}_history"] = r["history"]
        arrays[f"{name}_source_out"] = r["source_out"]
        arrays[f"{name}_final_R"] = r["final_R"]
        arrays[f"{name}_final_t"] = r["final_t"]
        meta[name] = {"params": p, "stop_at": c.get("stop_at", -1), "finished": r["finished"],
                      "message": r["message"], "total_iterations": r["total_iterations"],
                      "final_rmse": r["final_rmse"], "n_history": int(len(r["history"]))}
    np.savez_compressed(OUT / "engine_rules.npz", **arrays)
    return meta


def core_las():
    """The core LASIO (core/lasio.cpp, Qt build): writeLAS bytes, readLAS with and without the
    maxPoints truncation (lasio.cpp:60-63), readLAS of the CLI writer's file."""
    import tempfile
    rng = np.random.default_rng(78)
    n = 10007
    xyz = np.stack([rng.normal(0, 30, n) + 4.0e5, rng.normal(0, 20, n) + 3.2e6, rng.normal(0, 3, n) + 12.0], 1)
    xyz[:3] = [[4.0e5, 3.2e6, 12.0], [4.0e5 - 0.0004999, 3.2e6 + 0.0005001, 11.9995], [4.1e5, 3.1e6, -7.0]]
    arrays = {"core_points": xyz}
    G = np.load(OUT / "las_report.npz")
    with tempfile.TemporaryDirectory() as d:
        f = Path(d) / "core.las"
        assert O.ref_core_write_las(f, xyz)
        blob = f.read_bytes()
        arrays["core_file"] = np.frombuffer(blob, np.uint8)
        arrays["core_read"] = O.ref_core_read_las(f)
        arrays["core_read_max"] = O.ref_core_read_las(f, max_points=1234)
        # the registered source written with the bounds of the cloud as loaded (stale: the
        # service never recomputes them after registration, registrationservice.cpp:98, :156)
        moved = xyz + [0.7, -1.3, 0.25]
        stale = np.array([xyz[:, 0].min(), xyz[:, 0].max(), xyz[:, 1].min(), xyz[:, 1].max(),
                          xyz[:, 2].min(), xyz[:, 2].max()])
        h = Path(d) / "stale.las"
        assert O.ref_core_write_las(h, moved, stale)
        arrays["core_moved"] = moved
        arrays["core_stale_bounds"] = stale
        arrays["core_file_stale"] = np.frombuffer(h.read_bytes(), np.uint8)
        g = Path(d) / "cli.las"
        g.write_bytes(G["las_file"].tobytes())
        arrays["core_read_cli_file"] = O.ref_core_read_las(g)
        arrays["core_read_cli_file_max"] = O.ref_core_read_las(g, max_points=10001)
        z = bytearray(G["las_file"].tobytes()[:227])
        z[107:111] = (0).to_bytes(4, "little")
        (Path(d) / "z.las").write_bytes(bytes(z))
        rz = O.ref_core_read_las(Path(d) / "z.las")
        arrays["core_zero_points"] = np.array([-1 if rz is None else len(rz)])
    np.savez_compressed(OUT / "core_las.npz", **arrays)
    return {"n": n, "file_bytes": len(blob), "file_fnv1a": fnv1a(arrays["core_file"])}


def scene_cases():
    """A LiDAR-like surface pair (icp_synth_scene on a 3 m site: ground + walls from two scanner
    poses, ~1 cm spacing, 1 mm LAS grid, occlusion shadows, the blind disc under the scanner,
    0.2 % outliers) through the reference: the CLI octree's correspondences of the source as given
    and of the source the CLI ICP leaves (icp_registration.cpp:107-205, init 1e20), the CLI ICP's
    per-iteration cumulative transforms (:443-622), and the core engine's registration
    (core/icpengine.cpp)."""
    n, site = 30000, 3.0
    tgt, src, Ttrue = icp.synth_scene(n, site_radius=site)
    arrays = {"scene_target": tgt, "scene_source": src, "scene_T_true": Ttrue}
    ref = O.reference()

    def ref_dist(q, t, idx):
        return np.array([ref.ref_distance(np.ascontiguousarray(q[i]).ctypes.data_as(O.C.c_void_p),
                                          np.ascontiguousarray(t[idx[i]]).ctypes.data_as(O.C.c_void_p))
                         for i in range(len(q))])

    tree = O.RefTree(tgt)
    idx0 = tree.nn(src)
    arrays["scene_idx_iter0_cli"] = idx0
    arrays["scene_dist_iter0_cli"] = ref_dist(src, tgt, idx0)
    iters, tol = 20, 1e-9
    R, tt, tcums, src_out = O.ref_icp_cli(src, tgt, iters, tol)
    arrays["scene_cli_R_final"] = R
    arrays["scene_cli_t_final"] = tt
    arrays["scene_cli_T_cums"] = tcums
    arrays["scene_cli_source_out"] = src_out
    idxf = tree.nn(src_out)
    arrays["scene_idx_final_cli"] = idxf
    arrays["scene_dist_final_cli"] = ref_dist(src_out, tgt, idxf)
    eng = {"iterations": 10, "tolerance": 0.0, "sigma": 3.0}
    r = O.ref_engine_register(src, tgt, eng["iterations"], eng["tolerance"], eng["sigma"])
    arrays["scene_engine_history"] = r["history"]
    arrays["scene_engine_R"] = r["final_R"]
    arrays["scene_engine_t"] = r["final_t"]
    arrays["scene_engine_source_out"] = r["source_out"]
    np.savez_compressed(OUT / "scene_ref.npz", **arrays)
    q = np.round(tgt * 1000).astype(np.int64)
    return {"n": n, "site_radius": site, "cli_iterations": iters, "cli_tolerance": tol,
            "n_transforms": int(len(tcums)), "target_copies": int(n - len(np.unique(q, axis=0))),
            "engine": dict(eng, finished=r["finished"], total_iterations=r["total_iterations"],
                           final_rmse=r["final_rmse"], message=r["message"]),
            "inputs": "icp_synth_scene(30000, site_radius=3.0), stored in scene_ref.npz"}


def main():
    if not O.reference_available():
        O.build(ref=True)
    if "--only-scene" in sys.argv:
        meta = json.loads((OUT / "golden.json").read_text())
        meta["scene_ref"] = scene_cases()
        (OUT / "golden.json").write_text(json.dumps(meta, indent=1, sort_keys=True))
        print(json.dumps(meta["scene_ref"], indent=1))
        return
    if "--only-engine" in sys.argv:
        meta = json.loads((OUT / "golden.json").read_text())
        meta["engine_rules"] = engine_cases()
        meta["core_las"] = core_las()
        meta["engine_reference"] = ("PointCloudRegistration/core/{icpengine,octree,pointcloud,lasio}.cpp + moc, "
                                    "Qt 5.9.7 (/opt/conda), g++ -O2 -ffp-contract=off, no -march "
                                    "(oracle/_ref/libicp_ref_engine.so)")
        (OUT / "golden.json").write_text(json.dumps(meta, indent=1, sort_keys=True))
        print(json.dumps({k: meta[k] for k in ("engine_rules", "core_las")}, indent=1))
        return
    if "--only-las" in sys.argv:
        meta = json.loads((OUT / "golden.json").read_text())
        meta["las_report"] = las_and_report()
        (OUT / "golden.json").write_text(json.dumps(meta, indent=1, sort_keys=True))
        print(json.dumps(meta["las_report"], indent=1))
        return
    meta = {"generator": "tests/golden/gen_golden.py", "reference": "icp_registration.cpp + vendored Eigen 3.3.4 "
            "(oracle/_ref/libicp_ref.so, g++ -O2 -ffp-contract=off, no -march)"}
    meta["nn_known_answers"] = nn_known_answers()
    meta["svd_transform"] = svd_and_transform()
    meta["icp_cli"] = icp_cli_cases()
    meta["nn_100k"] = nn_100k_hashes()
    meta["las_report"] = las_and_report()
    meta["engine_rules"] = engine_cases()
    meta["core_las"] = core_las()
    meta["scene_ref"] = scene_cases()
    meta["engine_reference"] = ("PointCloudRegistration/core/{icpengine,octree,pointcloud,lasio}.cpp + moc, "
                                "Qt 5.9.7 (/opt/conda), g++ -O2 -ffp-contract=off, no -march "
                                "(oracle/_ref/libicp_ref_engine.so)")
    (OUT / "golden.json").write_text(json.dumps(meta, indent=1, sort_keys=True))
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
