#!/bin/bash
# Round 6 final record, part 2 (GPU box): the C1, C2, C3, C5 bench lines with
# their CPU baselines (tools/bench_configs.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final6
CONFIGS="C1 C2 C3 C5" bash tools/bench_configs.sh > gpurun_out/final6/configs.txt 2>&1 || { cat gpurun_out/final6/configs.txt; exit 1; }
cp gpurun_out/configs/bench_*.json gpurun_out/final6/
cat gpurun_out/final6/configs.txt
