# Round-end bench lines: the default (C4, CPU baseline, CSR sub-run) and
# C1-C3, C5 with their CPU baselines, into gpurun_out/final/.
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 600 python bench.py > gpurun_out/final/bench_C4.log 2>&1 || exit $?
grep "^{" gpurun_out/final/bench_C4.log | tail -1 > gpurun_out/final/bench_C4.json
python -c "
import json; d=json.load(open('gpurun_out/final/bench_C4.json'))
print('C4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'), d['parity']['ok'], d['cpu_baseline']['value'], d['csr']['value'])"
CONFIGS="C1 C2 C3 C5" bash tools/bench_configs.sh || exit $?
cp gpurun_out/configs/bench_C*.json gpurun_out/final/
