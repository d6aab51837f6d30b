#!/usr/bin/env python3
"""bench.py — Mcorr/s per ICP iteration on MI355X (BASELINE.json metric), config 4 by default:
10M <-> 10M synthetic clouds, source sharded over the ranks, target octree replicated.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 10000000]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

A step = one full ICP iteration of the product engine (icp_session_step): fused transform of
the resident source + exact octree NN + residual + 3-sigma statistics (RCCL all-gather) + cull
+ centroid/covariance (RCCL all-gather) + host 3x3 SVD. Convergence stops are disabled
(ICP_FLAG_NO_EARLY_STOP) so exactly K iterations are timed.

Rank 0 prints ONE JSON line. Extra objects:
  roofline      the search kernel's algorithmic bytes per launch (SURVEY.md §8d byte model:
                148 + 56 V + 24 P bytes per correspondence, V/P = node entries / leaf points of the
                reference DFS, counted exactly by the kernel) / its average HIP-event duration.
  cpu_baseline  the REFERENCE CPU path (oracle/_ref/ref_bench: icp_registration.cpp's ICP()),
                1 thread, on a bounded sample of the same workload (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
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
CONFIG_NAMES = {100_000: "config2", 10_000_000: "config4", 50_000_000: "config5"}


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced source shard of rank (sizes differ by at most one point)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def bytes_per_corr(v: float, p: float) -> float:
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
    # fallback: the C restatement (oracle/icp_oracle.c), same iteration difference
    t0 = time.perf_counter()
    oracle_py.icp(src[pick], tgt, oracle_py.SEM_CLI, 1, 1e-300)
    t1 = time.perf_counter()
    oracle_py.icp(src[pick], tgt, oracle_py.SEM_CLI, 2, 1e-300)
    t2 = time.perf_counter()
    it = (t2 - t1) - (t1 - t0)
    return {"value": len(pick) / it / 1e6, "unit": "Mcorr/s", "cores": 1, "kind": "port",
            "sample": f"{len(pick)} of {len(src)} queries vs full target, oracle/icp_oracle.c, CPU {cpu_model()}"}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--points", type=int, default=10_000_000, help="points per cloud (config 4: 10M)")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--exchange", choices=("rccl", "host"), default="rccl",
                    help="per-iteration all-gathers: RCCL (default), or over torch.distributed gloo "
                         "through the host (rehearsal of N ranks on one GPU; RCCL refuses that)")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "traffic_latest.json"),
                    help="PMC-derived HBM bytes per search launch (written by tools/pmc_traffic.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    import iterativeclosestpoint_amd as icp

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    device = local_rank % max(1, torch.cuda.device_count())  # ranks > GPUs only in rehearsals
    torch.cuda.set_device(device)

    n = args.points
    t_setup = time.perf_counter()
    tgt, src, T_true = icp.synth_pair(n)
    lo, hi = shard_range(n, rank, world)
    ctx = icp.Context(device)
    ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
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
        uid = [icp.Context.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(world, rank, uid[0])
    setup_s = time.perf_counter() - t_setup
    build_on_dev, build_ms = ctx.target_build_info()

    params = icp.params_default(max_iterations=args.warmup + args.steps + 1, tolerance=1e-6,
                                flags=icp.FLAG_NO_EARLY_STOP)
    sess = ctx.session(params)
    for _ in range(args.warmup):
        sess.step()
    ctx.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    taken = sess.step_n(args.steps)  # the engine's own loop, K iterations (no early stop)
    ctx.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    assert taken == args.steps, f"only {taken} of {args.steps} iterations ran"
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # HIP events of the timed iterates (read after the timed region)
    nn_ms, it_ms = ctx.timings(min(args.steps, 64))
    # untimed: how the last timed state splits over the search paths (same queries, same guess)
    probe = ctx.iterate(None, 1, icp.RULES_ENGINE, 3.0)
    rc, res = sess.finish()

    # untimed: reference-DFS work of this rank's queries (the V, P of the byte model)
    v_mean, p_mean = ctx.traversal_counts()
    n_local = hi - lo
    nn_avg_s = float(np.mean(nn_ms)) / 1e3
    b_corr = bytes_per_corr(v_mean, p_mean)
    achieved = b_corr * n_local / nn_avg_s / 1e9
    traffic = None
    tj = Path(args.traffic_json)
    if tj.exists():
        try:
            tr = json.loads(tj.read_text())
            import hashlib
            kh = hashlib.sha1((ROOT / "iterativeclosestpoint_amd" / "csrc" / "kernels.hip").read_bytes()).hexdigest()
            # only a profile of this exact kernel source and workload counts
            if tr.get("n") == n and tr.get("world") == world and tr.get("kernels_hip_sha1") == kh:
                traffic = tr.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    value = n * args.steps / elapsed / 1e6

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(tgt, src, args.cpu_sample)
        except Exception as e:  # keep the bench line even if the baseline cannot run
            cpu = {"value": None, "unit": "Mcorr/s", "cores": 1, "kind": "reference", "sample": f"failed: {e}"}

    if rank == 0:
        info = ctx.target_info()
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mcorr/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (icp_synth_pair: N(0, diag(5,5,1)^2) target seed 42; source = R^T(target - t) "
                    "+ 1 mm noise, 1% outliers, shuffled, seed 43)",
            "config": {
                "workload": f"{CONFIG_NAMES.get(n, 'custom')}: {n}<->{n} synthetic pair, full ICP iteration "
                            f"(engine rules, octree leaf 10 / depth 20), "
                            f"source sharded over {world} GPU(s), target octree replicated",
                "n_target": n, "n_source": n, "parallelism": f"spatial source shards x{world} (kd-order ranges; "
                + ("RCCL" if args.exchange == "rccl" else "host/gloo") + " all-gather of 2 moment records per iteration)",
                "octree_nodes": info["n_nodes"], "octree_leaves": info["n_leaves"],
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                # the measured side: PMC HBM bytes per launch / the same launch time (the model above
                # prices every node entry as an HBM read; most are L2/MALL hits, so frac can exceed 1)
                "traffic_gbs": None if traffic is None else round(traffic / nn_avg_s / 1e9, 1),
                "traffic_frac": None if traffic is None else round(traffic / nn_avg_s / 1e9 / HBM_PEAK_GBS, 4),
                "kernel": "k_nn4 (fused transform + wave-cooperative certified octree NN + residual + block moments)",
                "bytes_per_corr": round(b_corr, 1), "node_entries_per_query": round(v_mean, 3),
                "leaf_points_per_query": round(p_mean, 3), "kernel_ms_avg": round(float(np.mean(nn_ms)), 4),
                "iterate_device_ms_avg": round(float(np.mean(it_ms)), 4),
                "exact_fallback_queries": int(probe.n_fallback),
                "lane_search_queries": int(probe.n_lane_search),
                "ball_search_queries": int(probe.n_ball_search),
            },
            "cpu_baseline": cpu,
            "setup_s": round(setup_s, 2),
            "octree_build": {"on_device": build_on_dev, "ms": round(build_ms, 2)},
            "final_rmse": res.final_rmse,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
