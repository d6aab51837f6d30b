set -u
mkdir -p gpurun_out
bash tools/sq_profile.sh "3"
echo "=== 2 ranks on one GPU (RCCL rehearsal) ==="
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
   bench.py --gpus 2 --n 2000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err
echo "2rank rc=$?"; cat gpurun_out/bench_2rank.json; grep -v "^$" gpurun_out/bench_2rank.err | tail -5
timeout -k 10 300 python bench.py --n 2000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_1rank_2m.json 2>/dev/null
echo "1rank rc=$?"; cat gpurun_out/bench_1rank_2m.json
