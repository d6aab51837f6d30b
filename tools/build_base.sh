#!/bin/bash
# Build the library of a git revision (default HEAD) next to the working one, for same-box A/B
# runs (ICP_HIP_LIB=iterativeclosestpoint_amd/libicp_hip_<tag>.so). Runs here, not on the GPU box.
# usage: bash tools/build_base.sh [REV] [TAG]
set -eu
REV=${1:-HEAD}
TAG=${2:-base}
D=$(mktemp -d /tmp/icp_base.XXXXXX)
git archive "$REV" | tar -x -C "$D"
make -s -C "$D/iterativeclosestpoint_amd/csrc" -j8 ../libicp_hip.so
cp "$D/iterativeclosestpoint_amd/libicp_hip.so" "iterativeclosestpoint_amd/libicp_hip_$TAG.so"
rm -rf "$D"
echo "built iterativeclosestpoint_amd/libicp_hip_$TAG.so from $REV"
