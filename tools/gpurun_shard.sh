# GPU: per-rank iteration cost at 1/W of 10M (plain and over a 1-rank RCCL communicator), and a
# kernel trace of the W=8 shard over RCCL (per-kernel times and gaps of one iteration).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/shard_probe.py 1,2,4,8 || exit 1
RCCL=1 timeout -k 10 300 python3 tools/shard_probe.py 1,8 || exit 1
export TMPDIR=/tmp
(cd /tmp && RCCL=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OLDPWD/gpurun_out/shard_trace -o t -- python3 $OLDPWD/tools/shard_probe.py 8 > /dev/null 2>&1) || exit 1
python3 tools/timeline.py gpurun_out/shard_trace
