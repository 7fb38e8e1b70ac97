#!/bin/bash
# Round 6 (GPU box): same-box C4 A/B of the library against the one whose
# products-only whole-line pair walks two plane steps per trip
# (KR_ST2B_UNROLL=1), then graph_min patterns 6, 7 (last: a crash ends the call).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06f
mkdir -p $out
LIBS="parallel-krylov_amd/libkrylov_amd.so parallel-krylov_amd/libkrylov_amd_unroll.so" bash tools/lib_ab.sh > $out/ab.txt 2>&1 || { cat $out/ab.txt; exit 1; }
cat $out/ab.txt
for p in 6 7; do
  timeout -k 10 60 ./tools/micro/graph_min $p > $out/graph_min$p.txt 2>&1
  rc=$?; echo "exit $rc" >> $out/graph_min$p.txt; tail -3 $out/graph_min$p.txt
  [ $rc -ne 0 ] && exit 0
done
