#!/bin/bash
set -u
bash tools/sq_nn4.sh > gpurun_out/sq_base.txt 2>&1 || { echo fail; cat gpurun_out/sq_base.txt; exit 1; }
cat gpurun_out/sq_base.txt
