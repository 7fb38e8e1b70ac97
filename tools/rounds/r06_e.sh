#!/bin/bash
# Round 6 (GPU box): box-walk + stencil tests at the 128-plane walk defaults,
# the C5 full-size parity test with its printed envelope, then the graph_min
# capture patterns 5, 4, 3 (last: a crash ends the call).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06e
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_box_pair.py tests/test_gpu_stencil.py > $out/tests.txt 2>&1 || { tail -40 $out/tests.txt; exit 1; }
tail -2 $out/tests.txt
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread \
    tests/test_gpu_fullsize.py -k c5 > $out/c5_fullsize.txt 2>&1 || { tail -40 $out/c5_fullsize.txt; exit 1; }
grep -E "residual max|passed|failed" $out/c5_fullsize.txt
for p in 5 4 3; do
  timeout -k 10 60 ./tools/micro/graph_min $p > $out/graph_min$p.txt 2>&1
  rc=$?; echo "exit $rc" >> $out/graph_min$p.txt; tail -3 $out/graph_min$p.txt
  [ $rc -ne 0 ] && exit 0
done
