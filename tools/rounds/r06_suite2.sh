#!/bin/bash
# Round 6 (GPU box): the whole GPU suite + smoke at the final tree, then the SQ
# issue counters of the final C4 kernels (tools/sq_profile.sh).
set -o pipefail
export TMPDIR=/tmp
TAG=r06l bash tools/rounds/r06_suite.sh || exit $?
bash tools/sq_profile.sh r06l/sq > gpurun_out/r06l/sq.txt 2>&1 || { tail -20 gpurun_out/r06l/sq.txt; exit 1; }
grep -E "spmv2x2|spmv_step" gpurun_out/r06l/sq/sq_summary.txt
