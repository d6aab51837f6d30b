#!/bin/bash
# Build the working tree's library as iterativeclosestpoint_amd/libicp_hip_<tag>.so (same-box A/B of
# uncommitted variants and diagnostic builds: ICP_HIP_LIB selects it). Runs here, not on the GPU box.
# usage: bash tools/build_variant.sh TAG ["-DDEFINE=1 ..."]
#   e.g. build_variant.sh clk "-DICP_PHASE_CLOCKS=1"
set -eu
TAG=$1
EXTRA=${2:-}
make -s -C iterativeclosestpoint_amd/csrc -j8 BUILD="../../build/obj_$TAG" OUT="../libicp_hip_$TAG.so" EXTRA="$EXTRA" "../libicp_hip_$TAG.so"
echo "built iterativeclosestpoint_amd/libicp_hip_$TAG.so from the working tree ${EXTRA:+($EXTRA)}"
