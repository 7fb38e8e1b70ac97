#!/bin/bash
# Round 6 re-entry check (GPU box): the whole GPU suite, smoke, the default bench line.
# Everything under gpurun_out/r06a/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06a
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    > gpurun_out/r06a/pytest_gpu_full.txt 2>&1
rc=$?; tail -3 gpurun_out/r06a/pytest_gpu_full.txt; grep FAILED gpurun_out/r06a/pytest_gpu_full.txt | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06a/smoke.txt 2>&1 || exit $?
cat gpurun_out/r06a/smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/r06a/bench.log 2>&1 || exit $?
grep "^{" gpurun_out/r06a/bench.log | tail -1 > gpurun_out/r06a/bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/r06a/bench.json')); c=d.get('csr') or {}
print('C4', d['value'], d['ms_per_step'], d['roofline'], 'csr', c.get('value'), c.get('frac'), 'parity', (d.get('parity') or {}).get('ok'))"
