#!/bin/bash
# Round-5 final record (GPU box): rocprof + PMC passes of C4 plain CSR, C4 and C5, the
# C1/C2/C3/C5 bench lines with their CPU baselines, the C4 headline line.
# Everything under gpurun_out/final2/.
set -o pipefail
mkdir -p gpurun_out/final2
KR_MASK=0 KR_VDICT=0 KR_STENCIL=0 bash tools/profile.sh final2/C4_csr > gpurun_out/final2/C4_csr_prof.txt 2>&1 || exit $?
bash tools/profile.sh final2/C4 > gpurun_out/final2/C4_prof.txt 2>&1 || exit $?
bash tools/profile.sh final2/C5 --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-csr > gpurun_out/final2/C5_prof.txt 2>&1 || exit $?
bash tools/bench_configs.sh > gpurun_out/final2/configs.txt 2>&1 || exit $?
timeout -k 10 900 python bench.py > gpurun_out/final2/C4.log 2>&1 || exit $?
grep "^{" gpurun_out/final2/C4.log | tail -1 > gpurun_out/final2/bench_C4.json
cp gpurun_out/configs/bench_*.json gpurun_out/final2/
cat gpurun_out/final2/configs.txt
python3 -c "
import json; d=json.load(open('gpurun_out/final2/bench_C4.json')); c=d['csr']
print('C4', d['value'], d['roofline']['frac'], 'csr', c['value'], c['frac'], c['avg_ms'], 'parity', (d.get('parity') or {}).get('ok'))"
