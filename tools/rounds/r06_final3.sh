#!/bin/bash
# Round 6 final record, part 3 (GPU box), after the DPP neighbours (r06v-r06y): rocprofv3 kernel trace + PMC passes
# of C4 (tools/profile.sh), then the default bench line (C4 with its CPU
# baseline, full-size parity and the plain-CSR sub-record).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final6c
bash tools/profile.sh final6c/C4 > gpurun_out/final6c/C4_prof.txt 2>&1 || { tail -20 gpurun_out/final6c/C4_prof.txt; exit 1; }
tail -14 gpurun_out/final6c/C4/summary.txt
timeout -k 10 600 python bench.py > gpurun_out/final6c/bench_C4.log 2>&1 || exit $?
grep "^{" gpurun_out/final6c/bench_C4.log | tail -1 > gpurun_out/final6c/bench_C4.json
python3 -c "
import json; d=json.load(open('gpurun_out/final6c/bench_C4.json')); c=d['csr']; r=d['roofline']
print('C4', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['avg_ms'], 'csr', c['value'], c['frac'], c['avg_ms'], 'parity', (d.get('parity') or {}).get('ok'), 'cpu', d['cpu_baseline']['value'])
for k, v in d['kernels'].items(): print(' ', k, v['avg_ms'], v['gbs'])"
