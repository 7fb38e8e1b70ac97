#!/bin/bash
# Round 6 (GPU box): the thin-box cases of tests/test_gpu_box_pair.py.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06o
mkdir -p $out
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread \
    tests/test_gpu_box_pair.py -k thin > $out/thin.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" $out/thin.txt | head -30; exit $rc
