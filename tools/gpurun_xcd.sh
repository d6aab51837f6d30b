# GPU: XCD block renumbering A/B (timing + L2/fetch counters) and the per-phase clock probe.
set -u
mkdir -p gpurun_out
bash tools/gpurun_ab.sh xcd "" 2 cur:xcd_blocks=0 cur:xcd_blocks=64 cur:xcd_blocks=256 cur:xcd_blocks=1024 || exit 1
export TMPDIR=/tmp
for x in 0 256; do
  for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $set | cut -c1-5)
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OLDPWD/gpurun_out/xcd${x}/p_${tag} -o p -- \
      python3 $OLDPWD/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-parity --config xcd_blocks=$x > /dev/null 2>&1) || { echo "pmc fail $x $set"; exit 1; }
  done
  python3 tools/sq_summary.py gpurun_out/xcd${x} "k_nn_wave<true" | sed "s/^/xcd=$x /"
done
ICP_HIP_LIB=$PWD/iterativeclosestpoint_amd/libicp_hip_clk.so timeout -k 10 300 python3 tools/phase_probe.py || exit 1
