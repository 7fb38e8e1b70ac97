#!/bin/bash
# Round 6 (GPU box): the whole tests/test_gpu_box_pair.py at the final tree.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06q
mkdir -p $out
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread \
    tests/test_gpu_box_pair.py > $out/box_tests.txt 2>&1
rc=$?; tail -3 $out/box_tests.txt; grep -E "FAILED|^E " $out/box_tests.txt | head -20; exit $rc
