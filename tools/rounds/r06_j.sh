#!/bin/bash
# Round 6 (GPU box): the C4 full-size tests (box walks bitwise the dual path,
# partitions vs the oracle).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06j
mkdir -p $out
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread \
    tests/test_gpu_fullsize.py -k c4 > $out/c4_fullsize.txt 2>&1 || { tail -40 $out/c4_fullsize.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $out/c4_fullsize.txt
