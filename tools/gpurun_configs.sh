# GPU: bench lines for the other BASELINE configs on one GPU (the driver's bench is config 4):
# config 2 (100k), config 3's size on a 1 mm LAS grid (1M, ties and duplicates), config 5 (50M).
set -u
mkdir -p gpurun_out/configs
timeout -k 10 300 python3 bench.py --points 100000 --steps 200 --cpu-sample 100000 > gpurun_out/configs/config2.json 2> gpurun_out/configs/config2.err || exit 1
timeout -k 10 300 python3 bench.py --points 1000000 --steps 200 --quantize 0.001 --cpu-sample 200000 > gpurun_out/configs/config3_grid.json 2> gpurun_out/configs/config3_grid.err || exit 1
timeout -k 10 600 python3 bench.py --points 50000000 --steps 50 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/configs/config5.json 2> gpurun_out/configs/config5.err || exit 1
for f in gpurun_out/configs/*.json; do python3 -c "
import json,sys; j=json.load(open(sys.argv[1])); p=j.get('parity') or {}; r=j['roofline'] or {}
print(sys.argv[1], j['value'], 'median', j['median']['value'], 'knn', r.get('kernel_ms_avg'), 'paths', j['search_paths'], 'T_rmse', p.get('final_transform_rmse_vs_cpu'), 'cpu', (j.get('cpu_baseline') or {}).get('value'), (j.get('cpu_allcores') or {}).get('value'))" $f; done
