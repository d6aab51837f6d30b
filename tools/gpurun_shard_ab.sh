# GPU: per-rank iteration cost at 1/W of 10M for two library builds, interleaved (same box).
# usage (gpurun): bash tools/gpurun_shard_ab.sh LIB_A LIB_B [WORLDS]
set -u
W=${3:-1,8}
for r in 1 2; do
  for L in "$1" "$2"; do
    echo "== $L"
    ICP_HIP_LIB=$PWD/$L timeout -k 10 300 python3 tools/shard_probe.py $W 2>/dev/null | grep world || exit 1
  done
done
