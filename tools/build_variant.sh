#!/bin/bash
# Build the working tree's library and keep a copy as iterativeclosestpoint_amd/libicp_hip_<tag>.so
# (same-box A/B of uncommitted variants: ICP_HIP_LIB selects it). Runs here, not on the GPU box.
# usage: bash tools/build_variant.sh TAG
set -eu
TAG=$1
make -s -C iterativeclosestpoint_amd/csrc -j8 ../libicp_hip.so
cp iterativeclosestpoint_amd/libicp_hip.so "iterativeclosestpoint_amd/libicp_hip_$TAG.so"
echo "built iterativeclosestpoint_amd/libicp_hip_$TAG.so from the working tree"
