#!/bin/bash
# Round 6 (GPU box): tests/test_gpu_box_pair.py (incl. the low-residual box-walk
# cases against the oracle), printing the cases' timings.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06k
mkdir -p $out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread --durations=8 \
    tests/test_gpu_box_pair.py > $out/box_tests.txt 2>&1 || { grep -E "^E |FAILED|Error" $out/box_tests.txt | head -40; tail -5 $out/box_tests.txt; exit 1; }
grep -E "low_residual|passed|failed" $out/box_tests.txt | tail -8
