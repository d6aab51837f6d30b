# Rehearsal of the bench's N>1 path on a one-GPU box: N ranks share cuda:0 (bench.py maps
# local_rank % device_count) and exchange the per-iteration records over gloo (--exchange host;
# RCCL refuses two ranks on one device). Then the same workload on one rank for comparison.
set -u
mkdir -p gpurun_out
PTS=${1:-10000000}
for W in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 2951$W \
     bench.py --gpus $W --points $PTS --steps 10 --warmup 3 --no-cpu-baseline --exchange host \
     > gpurun_out/bench_${W}rank_host.json 2> gpurun_out/bench_${W}rank_host.err || { echo "W=$W failed"; grep -v "^$" gpurun_out/bench_${W}rank_host.err | tail -25; exit 1; }
  echo "W=$W"; cat gpurun_out/bench_${W}rank_host.json
done
