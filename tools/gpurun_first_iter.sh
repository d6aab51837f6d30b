set -u
timeout -k 10 300 python3 tools/counter_probe.py 10000000 3 2>/dev/null > gpurun_out/fi_counters.jsonl || exit 1
cat gpurun_out/fi_counters.jsonl
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fi_pytest.log 2>&1 || { tail -30 gpurun_out/fi_pytest.log; exit 1; }
tail -1 gpurun_out/fi_pytest.log
bash tools/gpurun_ab.sh fi "" 2 iterativeclosestpoint_amd/libicp_hip_base.so cur || exit 1
for f in gpurun_out/ab_fi.*.json; do python3 -c "import json,sys; j=json.load(open(sys.argv[1])); print(sys.argv[1], j['first_iteration'])" $f; done
