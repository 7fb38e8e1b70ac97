#!/bin/bash
# Round 6 (GPU box): the whole GPU suite and smoke at the current tree.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r06i}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    > $out/pytest_gpu_full.txt 2>&1
rc=$?; tail -3 $out/pytest_gpu_full.txt; grep FAILED $out/pytest_gpu_full.txt | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit $?
cat $out/smoke.txt
