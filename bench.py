#!/usr/bin/env python3
"""bench.py — Mcorr/s per ICP iteration on MI355X (BASELINE.json metric), config 4 by default:
10M <-> 10M synthetic clouds, source sharded over the ranks, target octree replicated.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--points 10000000]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)
    python bench.py --gpus N ...   (N > 1 without a launcher: one process drives the N GPUs,
                                    icp_hip_create_multi; the drop-in's single-process path)

A step = one full ICP iteration of the product engine (icp_session_step): fused transform of
the resident source + exact octree NN + residual + 3-sigma statistics (RCCL all-gather) + cull
+ centroid/covariance (RCCL all-gather) + host 3x3 SVD. Convergence stops are disabled
(ICP_FLAG_NO_EARLY_STOP) so exactly K iterations are timed.

Rank 0 prints ONE JSON line. `value` = the points of all ranks x K / the wall time of the K timed
iterations (max over ranks); `median` = the same rate from the median iteration of 2..K
(SURVEY.md §8d). Extra objects:
  roofline      the search kernel k_nn_wave: its compulsory HBM bytes per launch (DESIGN.md §3.1:
                64 B per query streamed + every target point (28 B) and node (56 B) once) / its
                average HIP-event duration over the timed iterations; `traffic` = PMC bytes per
                launch (rocprofv3, calibrated per access width: tools/calib_pmc.sh) of the same
                kernel source, or null; `fabric_gbs` = those bytes over this run's kernel time
                (L2 -> fabric requests, Infinity-Cache hits included: not an HBM rate).
  reference_work  SURVEY.md §8d's model of the reference DFS's work (148 + 56 V + 24 P bytes per
                correspondence): what the reference would move, not what this kernel moves.
  cpu_baseline  the REFERENCE CPU path (oracle/_ref/ref_bench: icp_registration.cpp's ICP()),
                1 thread, on a bounded sample of the same workload (rank 0, N=1 only).
  cpu_allcores  the CPU restatement (oracle/icp_oracle.c, OpenMP NN loop) on every core of this
                process's CPU set, full size, from the parity leg below.
  timed_state_parity  (N=1) the correspondences and residuals of the LAST TIMED iterate (the
                candidate-cache state the figure was measured in) against the CPU oracle's octree
                NN on the same moved source, every query: mismatch counts (bit for bit).
  registration  (N=1) a registration of the full clouds with the reference's stops on
                (ICPParameters defaults): iterations taken, wall, mean Mcorr/s over all iterates
                including the first, the first iterate's share.
  parity        (N=1) a fresh engine registration of the full clouds for --parity-iters
                iterations on the GPU and on the CPU oracle: final transform RMSE (north star:
                <= 1e-6), per-iteration valid counts, final RMSE.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "M correspondences/sec per ICP iter at 1/2/4/8 GPUs; final RMSE vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
# BASELINE.json configs by cloud size (config 3 is the LAS pair: tests/test_gpu_lasflow.py)
CONFIG_NAMES = {100_000: "config2", 1_000_000: "synthetic-1M (config 3's size; config 3 itself, the LAS flow, is tests/test_gpu_lasflow.py)", 10_000_000: "config4", 50_000_000: "config5"}
SEARCH_SOURCES = ("nn_kernels.hip", "nn_device.h", "kernels.h", "wave_stats.h")
# compulsory bytes of one k_nn_wave<true> launch
STREAM_B_PER_QUERY = 24 + 24 + 4 + 4 + 8  # source read + transformed write, previous match (guess), pos + dist
TGT_B_PER_POINT = 28  # x, y, z + original index of a leaf-ordered target point
NODE_B = 56  # box (48 B) + topology (8 B) of a node record


TIMING_STRIDE = 8
PEER_TIMEOUT_MS = 10_000


def search_source_sha1() -> str:
    """Hash of the search kernel's sources: a PMC profile counts only for the code it measured."""
    h = hashlib.sha1()
    for f in SEARCH_SOURCES:
        h.update((ROOT / "iterativeclosestpoint_amd" / "csrc" / f).read_bytes())
    return h.hexdigest()


def workload_key(args) -> str:
    """The data a PMC profile was taken on (tools/profile_bench.sh WORKLOAD): counters of one
    workload never describe another's kernel."""
    return f"{'scene' if args.scene else 'blob'}|q={float(args.quantize)}|dup={int(args.duplicates)}" + (
        "" if args.scene_outliers is None else f"|out={float(args.scene_outliers)}")


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced source shard of rank (sizes differ by at most one point)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def compulsory_bytes(n_local: int, n_total: int, n_tgt: int, n_nodes: int) -> float:
    """HBM bytes one search launch cannot avoid: its queries streamed once, and the target points
    and nodes once (a spatial shard touches about its share of them)."""
    share = n_local / max(1, n_total)
    return STREAM_B_PER_QUERY * n_local + (TGT_B_PER_POINT * n_tgt + NODE_B * n_nodes) * share


def reference_bytes_per_corr(v: float, p: float) -> float:
    # query 24 + idx 4 + residual 8 (NN pass); residual 8 (sigma pass);
    # residual 8 + query 24 + idx 4 + gather 24 (cull/covariance); transform r+w 48;
    # 56 B per node entry (48 B box + 8 B topology); 24 B per leaf point scanned.
    return 148.0 + 56.0 * v + 24.0 * p


def cpu_model() -> str:
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def cpu_threads() -> int:
    """Cores of this process's CPU share: the affinity set, capped by OMP_NUM_THREADS if set."""
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def cpu_baseline(tgt: np.ndarray, src: np.ndarray, sample: int) -> dict | None:
    """Reference ICP() iteration on `sample` source queries against the full target (1 thread)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_py  # test infrastructure: the CPU baseline leg only

    rng = np.random.default_rng(1)
    pick = np.sort(rng.choice(len(src), size=min(sample, len(src)), replace=False))
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        tf, sf = Path(td) / "target.f64", Path(td) / "source.f64"
        np.ascontiguousarray(tgt).tofile(tf)
        np.ascontiguousarray(src[pick]).tofile(sf)
        if oracle_py.REF_BENCH.exists():
            r = subprocess.run([str(oracle_py.REF_BENCH), str(tf), str(sf)], capture_output=True, text=True,
                               timeout=900)
            if r.returncode == 0 and r.stdout.strip():
                j = json.loads(r.stdout.strip().splitlines()[-1])
                return {"value": j["mcorr_per_s"], "unit": "Mcorr/s", "cores": 1, "kind": "reference",
                        "sample": f"{len(pick)} of {len(src)} source queries vs the full {len(tgt)}-point target; "
                                  f"one reference ICP() iteration (icp_registration.cpp:443-622, g++ -O2) = "
                                  f"t(ICP 2 iters) - t(ICP 1 iter) = {j['iter_s']:.2f} s; CPU {cpu_model()}"}
    # fallback: the C restatement (oracle/icp_oracle.c), same iteration difference, one thread
    oracle_py.set_threads(1)
    t0 = time.perf_counter()
    oracle_py.icp(src[pick], tgt, oracle_py.SEM_CLI, 1, 1e-300)
    t1 = time.perf_counter()
    oracle_py.icp(src[pick], tgt, oracle_py.SEM_CLI, 2, 1e-300)
    t2 = time.perf_counter()
    it = (t2 - t1) - (t1 - t0)
    return {"value": len(pick) / it / 1e6, "unit": "Mcorr/s", "cores": 1, "kind": "port",
            "sample": f"{len(pick)} of {len(src)} queries vs full target, oracle/icp_oracle.c, CPU {cpu_model()}"}


def timed_state_parity(tgt: np.ndarray, q: np.ndarray, idx: np.ndarray, d: np.ndarray, iterate: int) -> dict:
    """The correspondences and residuals of the LAST TIMED iterate (candidate cache state and all)
    against the CPU oracle's octree NN on the same moved source, every query (OpenMP)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_py  # test infrastructure: the checker only

    cores = cpu_threads()
    oracle_py.set_threads(cores)
    t0 = time.perf_counter()
    oidx, od = oracle_py.OracleTree(tgt).nn(q, init_best=oracle_py.DBL_MAX)
    return {"iterate": iterate, "checked": int(len(q)),
            "idx_mismatch": int(np.count_nonzero(idx != oidx)),
            "dist_mismatch": int(np.count_nonzero(d.view(np.uint64) != od.view(np.uint64))),
            "checker": f"oracle/icp_oracle.c octree NN (octree.cpp:128-184), {cores} threads, "
                       f"{time.perf_counter() - t0:.1f} s"}


def registration_leg(icp, ctx, src: np.ndarray) -> dict:
    """A real registration of the full clouds with the reference's stops on (ICPParameters defaults:
    50 iterations, tolerance 1e-6, 3x no improvement, divergence; icpengine.cpp:287-323): what one
    registration costs end to end on the resident target, first iterate included."""
    ctx.set_source(src)
    p = icp.params_default()
    sess = ctx.session(p)
    ms = sess.step_n_timed(p.max_iterations + 1)
    rc, res = sess.finish()
    sess.close()
    n = len(src)
    total = float(np.sum(ms))
    status = {0: "max_iterations", 1: "converged", 2: "diverged", 3: "too_few", 4: "cancelled"}.get(res.status, "?")
    return {"iterations": len(ms), "status": status, "wall_ms": round(total, 3),
            "mean_value": round(n * len(ms) / total / 1e3, 3), "unit": "Mcorr/s",
            "first_iteration_ms": round(float(ms[0]), 4), "first_iteration_share": round(float(ms[0]) / total, 4),
            "final_rmse": res.final_rmse,
            "note": "ICPParameters defaults (icpengine.h:13-19) with the reference's stops on; wall = sum of "
                    "the steps (set_source excluded); mean_value = n x iterations / wall"}


def parity_leg(icp, ctx, tgt: np.ndarray, src: np.ndarray, iters: int) -> tuple[dict, dict]:
    """A fresh engine registration (tolerance 0: exactly `iters` iterations) of the full clouds on
    the GPU and on the CPU oracle (OpenMP over all cores of this process). Returns the parity
    record and the all-core CPU throughput (per-iteration time = (ICP time - octree build) / iters)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_py  # test infrastructure: the checker and the CPU baseline leg only

    ctx.set_source(src)
    sess = ctx.session(icp.params_default(max_iterations=iters, tolerance=0.0))
    g_valid, g_rmse = [], []
    while not sess.done:
        rec = sess.step()
        if rec is not None:
            g_valid.append(int(rec.valid_points))
            g_rmse.append(float(rec.rmse))
    rc, res = sess.finish()
    sess.close()
    Tg = np.eye(4)
    Tg[:3, :3] = np.array(res.final_R).reshape(3, 3)
    Tg[:3, 3] = res.final_t

    cores = cpu_threads()
    oracle_py.set_threads(cores)
    t0 = time.perf_counter()
    oracle_py.OracleTree(tgt)  # the octree build inside ICP, timed alone (single-threaded)
    t_build = time.perf_counter() - t0
    t0 = time.perf_counter()
    orc, ores, ohist, _ = oracle_py.icp(src, tgt, oracle_py.SEM_ENGINE, iters, 0.0)
    t_icp = time.perf_counter() - t0
    To = np.eye(4)
    To[:3, :3] = np.array(ores.final_R).reshape(3, 3)
    To[:3, 3] = ores.final_t
    o_valid = [int(h.valid) for h in ohist if h.has_transform]
    o_rmse = [float(h.rmse) for h in ohist if h.has_transform]
    rel = [abs(a - b) / max(abs(b), 1e-300) for a, b in zip(g_rmse, o_rmse)]
    parity = {
        "iterations": iters,
        "final_transform_rmse_vs_cpu": float(np.sqrt(np.mean((Tg - To) ** 2))),
        "tolerance": 1e-6,
        "iterations_equal": res.total_iterations == ores.total_iterations,
        "valid_counts_equal": g_valid == o_valid,
        "final_rmse_gpu": res.final_rmse, "final_rmse_cpu": ores.final_rmse,
        "rmse_max_rel_diff": max(rel) if rel else None,
        "checker": "oracle/icp_oracle.c engine rules (pinned to core/icpengine.cpp by tests/golden/engine_rules.npz)",
    }
    per_iter = max(1e-9, (t_icp - t_build) / iters)
    allcores = {"value": round(len(src) / per_iter / 1e6, 4), "unit": "Mcorr/s", "cores": cores, "kind": "port",
                "sample": f"full {len(src)}<->{len(tgt)} engine ICP, {iters} iterations: ({t_icp:.1f} s - "
                          f"{t_build:.1f} s octree build) / {iters}; OpenMP NN loop, CPU {cpu_model()}"}
    return parity, allcores


class stdout_to_stderr:
    """RCCL prints a version banner on file descriptor 1 when a communicator is created; the bench
    contract is ONE JSON line on stdout, so native writes go to stderr while RCCL initialises."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        import ctypes
        ctypes.CDLL(None).fflush(None)  # C stdio buffers too, before fd 1 is restored
        os.dup2(self.saved, 1)
        os.close(self.saved)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--points", type=int, default=10_000_000, help="points per cloud (config 4: 10M)")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000)
    ap.add_argument("--parity-iters", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the CPU checks (the timed state's correspondences and the fresh registration)")
    ap.add_argument("--no-registration", action="store_true", help="skip the stops-on registration leg")
    ap.add_argument("--prewarm-ms", type=float, default=0.0,
                    help="diagnostic: keep the GPU busy with a matrix loop this long before the warmup steps")
    ap.add_argument("--exchange", choices=("rccl", "host"), default="rccl",
                    help="per-iteration all-gathers: RCCL (default), or over torch.distributed gloo "
                         "through the host (rehearsal of N ranks on one GPU; RCCL refuses that)")
    ap.add_argument("--rccl-self", action="store_true",
                    help="one rank: run the iterations over a 1-rank RCCL communicator (the multi-rank "
                         "path: ncclAllGather + rank-order device merges) instead of the plain path")
    ap.add_argument("--quantize", type=float, default=0.0,
                    help="round both clouds to this grid (LAS 1.2 stores int32 x scale: 0.001 emulates "
                         "config 3's 1 mm grid, with its exact ties and duplicates)")
    ap.add_argument("--duplicates", type=int, default=1,
                    help="every target point repeated this many times (an exact tie for every query: the "
                         "certified search's fp64 rescan gives copies of the winner the lowest slot, "
                         "as the reference's leaf order does)")
    ap.add_argument("--scene", action="store_true",
                    help="a LiDAR-like scene pair (icp_synth_scene: ground + walls scanned from two poses, "
                         "range-dependent density, 1 mm grid) instead of config 4's Gaussian blob")
    ap.add_argument("--scene-outliers", type=float, default=None,
                    help="--scene: the source's outlier fraction (default the generator's 0.002)")
    ap.add_argument("--config", action="append", default=[], metavar="KEY=VALUE",
                    help="icp_hip_config field for the context (A/B of search options), repeatable")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "traffic_latest.json"),
                    help="PMC-derived bytes per search launch (written by tools/pmc_traffic.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    import iterativeclosestpoint_amd as icp

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        with stdout_to_stderr():  # gloo prints "[Gloo] Rank r is connected to ..." on fd 1
            dist.init_process_group("gloo", rank=rank, world_size=world)
            dist.barrier()
    n_dev = max(1, torch.cuda.device_count())
    device = local_rank % n_dev  # ranks > GPUs only in host-exchange rehearsals
    # --gpus N > 1 without a launcher: one process drives all N devices (icp_hip_create_multi:
    # a driver thread per device, RCCL from ncclCommInitAll; devices repeat only in a rehearsal on
    # fewer GPUs, which then uses the in-process host gather)
    group = world == 1 and args.gpus > 1
    shards = args.gpus if group else world
    gpus_used = min(shards, n_dev)
    shared_gpu = shards > gpus_used
    torch.cuda.set_device(device)

    n = args.points
    t_setup = time.perf_counter()
    scene_kw = {} if args.scene_outliers is None else {"outlier_fraction": args.scene_outliers}
    tgt, src, T_true = icp.synth_scene(n, **scene_kw) if args.scene else icp.synth_pair(n)
    if args.duplicates > 1:
        tgt = np.repeat(tgt[: n // args.duplicates + 1], args.duplicates, axis=0)[:n]
    if args.quantize > 0:
        tgt = np.round(tgt / args.quantize) * args.quantize
        src = np.round(src / args.quantize) * args.quantize
    lo, hi = shard_range(n, rank, world)
    # the search kernel is timed (HIP events on its dispatch and the next kernel's) on every 8th
    # iterate: an event on a dispatch packet delays the next kernel by ~3-5 us (25 samples of 200)
    kv = {"timing_stride": str(TIMING_STRIDE)}
    if shards > 1:
        # a stalled or dead peer ends the run with ICP_HIP_ERCCL instead of a hang (per iterate;
        # the first iterate of a 10M scene shard takes ~0.1 s)
        kv["peer_timeout_ms"] = str(PEER_TIMEOUT_MS)
    kv.update(dict(c.split("=", 1) for c in args.config))
    conf = icp.config(**{k: (float(v) if "." in v else int(v)) for k, v in kv.items()})
    ctx = icp.Context(devices=[k % n_dev for k in range(args.gpus)], cfg=conf) if group else icp.Context(device, conf)
    t_synth = time.perf_counter() - t_setup
    t1 = time.perf_counter()
    ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
    t_target = time.perf_counter() - t1
    t1 = time.perf_counter()
    # spatial shards: contiguous ranges of the kd order (a contiguous range of the shuffled cloud
    # would thin each rank's queries `world` times; see icp_host.h icp_source_shard_order)
    ctx.set_source(src[icp.source_shard_order(src)[lo:hi]] if world > 1 else src)
    if world > 1 and args.exchange == "host":
        def exchange(local):
            t = torch.from_numpy(local)
            out = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(out, t)
            return torch.stack(out).numpy()
        ctx.comm_init_host(world, rank, exchange)
    elif world > 1:
        with stdout_to_stderr():
            uid = [icp.Context.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        with stdout_to_stderr():
            ctx.comm_init(world, rank, uid[0])
    elif args.rccl_self:
        with stdout_to_stderr():
            ctx.comm_init(1, 0, icp.Context.unique_id())
    t_source = time.perf_counter() - t1
    setup_s = time.perf_counter() - t_setup
    build_on_dev, build_ms = ctx.target_build_info()

    params = icp.params_default(max_iterations=args.warmup + args.steps + 1, tolerance=1e-6,
                                flags=icp.FLAG_NO_EARLY_STOP)
    sess = ctx.session(params)
    if args.prewarm_ms > 0:
        a_ = torch.randn(4096, 4096, device=f"cuda:{device}")
        t_w = time.perf_counter()
        while (time.perf_counter() - t_w) * 1e3 < args.prewarm_ms:
            for _ in range(8):
                a_ = torch.tanh(a_ @ a_)
            torch.cuda.synchronize()
        del a_
    # warmup; the first iteration (no previous residuals: the guess is a descent) is reported alone
    first_ms = sess.step_n_timed(1)
    first_nn_ms, _ = ctx.timings(1)
    if args.warmup > 1:
        sess.step_n_timed(args.warmup - 1)
    ctx.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    step_ms = sess.step_n_timed(args.steps)  # the engine's own loop, K iterations (no early stop)
    ctx.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    assert len(step_ms) == args.steps, f"only {len(step_ms)} of {args.steps} iterations ran"
    med_ms = float(np.median(step_ms[1:] if len(step_ms) > 1 else step_ms))
    if world > 1:
        t = torch.tensor([elapsed, med_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, med_ms = float(t[0].item()), float(t[1].item())
    # HIP events of the timed iterates (read after the timed region)
    nn_ms, it_ms = ctx.timings(min(args.steps, 256))
    comm = None
    if shards > 1 or args.rccl_self:
        # what RCCL itself reports (ncclCommCount / ncclCommUserRank / ncclCommCuDevice) for every
        # rank, and each rank's exchange time (events around the two all-gathers, timed iterates)
        xms = ctx.exchange_timings(min(args.steps, 256))
        xms = xms[np.isfinite(xms)]
        mine = [dict(ctx.comm_info(m), hip_device=dev, pid=os.getpid(),
                     exchange_ms_mean=None if len(xms) == 0 else round(float(np.mean(xms)), 4),
                     exchange_ms_max=None if len(xms) == 0 else round(float(np.max(xms)), 4),
                     exchange_samples=int(len(xms)))
                for m, dev in ((k, d) for k, d in enumerate(ctx.devices()[0] if group else [device]))]
        if world > 1:
            allr = [None] * world
            dist.all_gather_object(allr, mine)
            mine = [r for per in allr for r in per]
        comm = {"ranks": mine, "rccl_count_ok": all(r["count"] == shards for r in mine),
                "rank_set_ok": sorted(r["rank"] for r in mine) == list(range(shards)),
                "peer_timeout_ms": int(conf.peer_timeout_ms),
                "note": "count/rank/device: RCCL's own view (icp_hip_comm_info); exchange_ms: the two per-iteration "
                        "record all-gathers (HIP events on the compute stream, includes waiting for the slowest "
                        "peer; host clock for the host exchange), timed iterates (every 8th) of the timed region"}
    # untimed: the state the last timed iterate left (its queries = the moved source, and its
    # correspondences/residuals), checked against the CPU oracle below
    timed_q = timed_idx = timed_d = None
    if rank == 0 and world == 1 and not args.no_parity:
        timed_q = ctx.get_source()
        timed_idx, timed_d = ctx.get_correspondences()
    # untimed: how the last timed state splits over the search paths (same queries, same guess)
    probe = ctx.iterate(None, 1, icp.RULES_ENGINE, 3.0)
    rc, res = sess.finish()
    sess.close()
    # v, p of the reference DFS on this rank's queries (untimed; COUNT build of the parity kernel)
    v_mean, p_mean = ctx.traversal_counts() if rank == 0 else (None, None)

    info = ctx.target_info()
    n_local = n // shards if group else hi - lo  # per device
    nn_ms, it_ms = nn_ms[np.isfinite(nn_ms)], it_ms[np.isfinite(it_ms)]  # the timed iterates
    nn_avg_s = float(np.mean(nn_ms)) / 1e3
    need = compulsory_bytes(n_local, n, n, info["n_nodes"])
    achieved = need / nn_avg_s / 1e9
    traffic = valu = None
    tj = Path(args.traffic_json)
    if tj.exists():
        try:
            tr = json.loads(tj.read_text())
            # only a profile of this exact kernel source and workload counts (a profile written before
            # the workload key existed is of config 4's blob)
            if (tr.get("n") == n and tr.get("world") == shards and tr.get("search_src_sha1") == search_source_sha1()
                    and tr.get("workload", "blob|q=0.0|dup=1") == workload_key(args)):
                traffic = tr.get("bytes_per_launch")
                if tr.get("valu_issue_frac") is not None:
                    # the bound that binds the search kernel: VALU issue (SQ counters of the same
                    # profile): SQ_INSTS_VALU x 4 cycles per wave64 instruction on a 16-lane SIMD
                    # over 1024 SIMDs x the kernel's cycles (GRBM_GUI_ACTIVE / 8 XCDs)
                    valu = {"insts_per_wave": round(tr["valu_per_wave"], 1),
                            "salu_per_wave": None if tr.get("salu_per_wave") is None else round(tr["salu_per_wave"], 1),
                            "issue_frac": round(tr["valu_issue_frac"], 4),
                            "active_frac": None if tr.get("valu_active_frac") is None else round(tr["valu_active_frac"], 4),
                            "kernel_cycles": round(tr["kernel_cycles"]),
                            "peak": "1 wave64 VALU instruction per 4 cycles per SIMD, 1024 SIMDs",
                            "source": "rocprofv3 --pmc SQ_* of this kernel source, the driver's window "
                                      "(profiles/traffic_latest.json)"}
        except Exception:
            traffic = valu = None

    value = n * args.steps / elapsed / 1e6

    cpu = allcores = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(tgt, src, args.cpu_sample)
        except Exception as e:  # keep the bench line even if the baseline cannot run
            cpu = {"value": None, "unit": "Mcorr/s", "cores": 1, "kind": "reference", "sample": f"failed: {e}"}
    timed_parity = None
    if timed_q is not None:
        try:
            timed_parity = timed_state_parity(tgt, timed_q, timed_idx, timed_d, args.warmup + args.steps)
        except Exception as e:
            timed_parity = {"error": str(e)}
        del timed_q, timed_idx, timed_d
    registration = None
    if rank == 0 and world == 1 and not args.no_registration:
        try:
            registration = registration_leg(icp, ctx, src)
        except Exception as e:
            registration = {"error": str(e)}
    if rank == 0 and world == 1 and not args.no_parity and args.parity_iters > 0:
        try:
            parity, allcores = parity_leg(icp, ctx, tgt, src, args.parity_iters)
        except Exception as e:
            parity = {"error": str(e)}

    if rank == 0:
        nq = max(1, n_local * (shards if group else 1))
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mcorr/s",
            "n_gpus": gpus_used,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic LiDAR-like scene (icp_synth_scene: ground + 8 walls, scanner rays uniform in "
                     "azimuth/elevation, 2 mm range noise, 1 mm grid; source = an independent scan from a moved "
                     "scanner, 0.2 % outliers)" if args.scene else
                     "synthetic (icp_synth_pair: N(0, diag(5,5,1)^2) target seed 42; source = R^T(target - t) "
                     "+ 1 mm noise, 1% outliers, shuffled, seed 43)")
                    + (f"; both clouds rounded to a {args.quantize} m grid (LAS-style)" if args.quantize > 0 else "")
                    + (f"; every target point repeated {args.duplicates}x" if args.duplicates > 1 else ""),
            "config": {
                "workload": f"{'scene' if args.scene else CONFIG_NAMES.get(n, 'custom')}: {n}<->{n} synthetic pair, full ICP iteration "
                            f"(engine rules, octree leaf 10 / depth 20), "
                            f"source sharded over {shards} rank(s) on {gpus_used} GPU(s), target octree replicated",
                "n_target": n, "n_source": n, "ranks": shards, "ranks_per_gpu": shards // gpus_used,
                "parallelism": f"spatial source shards x{shards} (kd-order ranges; "
                + (("one process, a driver thread per device, " + ("RCCL (ncclCommInitAll)" if not shared_gpu else
                                                                   "in-process host gather rehearsal"))
                   if group else ("RCCL" if args.exchange == "rccl" else "host/gloo rehearsal"))
                + " all-gather of 2 moment records per iteration)"
                + ("; 1-rank RCCL communicator (multi-rank path)" if world == 1 and args.rccl_self else ""),
                "octree_nodes": info["n_nodes"], "octree_leaves": info["n_leaves"],
            },
            "median": {"iter_ms": round(med_ms, 4), "value": round(n / med_ms / 1e3, 3),
                       "over": f"iterations 2..{args.steps} of the timed region (host wall per step, max over ranks)"},
            "first_iteration": {"ms": round(float(first_ms[0]), 4), "search_kernel_ms": round(float(first_nn_ms[0]), 4),
                                "note": "no previous matches: the guesses are a descent, its sibling leaves and the other lanes' "
                                        "points (k_nn_wave<false>), every wave walks, full cull pass; kernels loaded by the "
                                        "context's process warm-up (icp_hip_config.no_warmup)"},
            # ranks sharing one GPU (host-exchange rehearsal) contend for it: no per-rank roofline
            "roofline": None if shared_gpu else {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "valu": valu,
                "binding": None if valu is None else ("valu" if valu["issue_frac"] > achieved / HBM_PEAK_GBS else "hbm"),
                "traffic_over_algorithmic": None if traffic is None else round(traffic / need, 3),
                # the PMC bytes of the same launch over this run's kernel time: L2 -> fabric
                # requests, which include Infinity-Cache (MALL) hits, so an upper bound of the HBM
                # rate, not an HBM figure (`frac` above, compulsory bytes, is the roofline figure)
                "fabric_gbs": None if traffic is None else round(traffic / nn_avg_s / 1e9, 1),
                "kernel": "k_nn_wave<true> (fused transform + wave-cooperative certified octree NN + residual)",
                "algorithmic_bytes_per_launch": round(need), "kernel_ms_avg": round(float(np.mean(nn_ms)), 4),
                "iterate_device_ms_avg": round(float(np.mean(it_ms)), 4),
                "model": f"{STREAM_B_PER_QUERY} B/query streamed + {TGT_B_PER_POINT} B/target point + {NODE_B} B/node, each once",
            },
            "search_paths": {"queries": n_local * (shards if group else 1),
                             "wave": n_local * (shards if group else 1) - int(probe.n_ball_search),
                             "ball": int(probe.n_ball_search), "lane": int(probe.n_lane_search),
                             "exact_fallback": int(probe.n_fallback),
                             "ball_share": round(probe.n_ball_search / nq, 6),
                             "fallback_share": round(probe.n_fallback / nq, 6)},
            "reference_work": None if v_mean is None else {
                "node_entries_per_query": round(v_mean, 3), "leaf_points_per_query": round(p_mean, 3),
                "bytes_per_corr": round(reference_bytes_per_corr(v_mean, p_mean), 1),
                "note": "SURVEY.md §8d model of the reference DFS's work; the certified search does not do it"},
            "cpu_baseline": cpu,
            "cpu_allcores": allcores,
            "parity": parity,
            "timed_state_parity": timed_parity,
            "registration": registration,
            "setup_s": round(setup_s, 2),
            "setup": {"synthesis_s": round(t_synth, 3), "set_target_s": round(t_target, 3),
                      "set_source_s": round(t_source, 3),
                      "note": "host synthesis; set_target = upload + device octree build + tables; "
                              "set_source = query order + upload (+ communicator setup for N > 1)"},
            "octree_build": {"on_device": build_on_dev, "ms": round(build_ms, 2)},
            "comm": comm,
            "final_rmse": res.final_rmse,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
