#!/bin/bash
# Round 6 (GPU box): rocprof trace + PMC passes of C4 at the box walks, SQ issue
# counters of the same run, the C2 stream-ceiling micro, then ONE capture-crash
# bisection variant of tools/micro/graph_cost (last: a crash ends the call).
#   GMODE=<mode> GNSPMV=<n>: the graph_cost variant (S = 2 shards)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06b
bash tools/profile.sh r06b/C4 > gpurun_out/r06b/C4_prof.txt 2>&1 || { tail -20 gpurun_out/r06b/C4_prof.txt; exit 1; }
tail -12 gpurun_out/r06b/C4/summary.txt
bash tools/sq_profile.sh r06b/sq > gpurun_out/r06b/sq.txt 2>&1 || { tail -20 gpurun_out/r06b/sq.txt; exit 1; }
cat gpurun_out/r06b/sq/sq_summary.txt
timeout -k 10 120 ./tools/micro/c2_stream > gpurun_out/r06b/c2_stream.txt 2>&1 || exit $?
cat gpurun_out/r06b/c2_stream.txt
g=gpurun_out/r06b/graph_s2_m${GMODE:-4}_n${GNSPMV:-9}.txt
timeout -k 10 60 ./tools/micro/graph_cost 2 ${GNSPMV:-9} 200 64 ${GMODE:-4} > $g 2>&1
echo "exit $?" >> $g
tail -6 $g
