set -u
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/counter_probe.py 10000000 8 > gpurun_out/counters.jsonl 2>gpurun_out/counters.err || exit 1
tail -2 gpurun_out/counters.jsonl
ICP_HIP_LIB=$PWD/iterativeclosestpoint_amd/libicp_hip_clk.so timeout -k 10 300 python3 tools/phase_probe.py > gpurun_out/phase.txt 2>&1 || exit 1
cat gpurun_out/phase.txt
bash tools/sq_wave.sh cur
