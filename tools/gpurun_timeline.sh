# GPU: rocprofv3 kernel trace of a short bench; per-kernel medians and the timeline of the last
# timed iteration (start offsets and idle gaps between kernels).
# usage: bash tools/gpurun_timeline.sh [bench args...]
set -u
mkdir -p gpurun_out/tl
rm -rf gpurun_out/tl/*
export TMPDIR=/tmp
REPO=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/tl -o tl -- \
  python3 $REPO/bench.py --no-cpu-baseline --steps 6 --warmup 2 "$@" > $REPO/gpurun_out/tl/bench.json 2> $REPO/gpurun_out/tl/err.log || exit $?
cd $REPO
python3 tools/timeline.py gpurun_out/tl
