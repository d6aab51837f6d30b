# RCCL rehearsal on a one-GPU box: two ranks share cuda:0 (bench.py maps local_rank % device_count).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
   bench.py --gpus 2 --points 2000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err
echo "2rank rc=$?"; cat gpurun_out/bench_2rank.json; grep -v "^$" gpurun_out/bench_2rank.err | tail -25
