# Round-end check of the final tree: the whole GPU suite, smoke, the default
# bench line (C4) and the C3 / C5 lines with their CPU baselines.
export TMPDIR=/tmp
mkdir -p gpurun_out/final3
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/final3/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/final3/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/final3/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final3/smoke.txt 2>&1 || { cat gpurun_out/final3/smoke.txt; exit 1; }
tail -2 gpurun_out/final3/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/final3/bench_C4.log 2>&1 || exit $?
grep "^{" gpurun_out/final3/bench_C4.log | tail -1 > gpurun_out/final3/bench_C4.json
CONFIGS="C3 C5" bash tools/bench_configs.sh || exit $?
cp gpurun_out/configs/bench_C3.json gpurun_out/configs/bench_C5.json gpurun_out/final3/
for c in C3 C4 C5; do python -c "
import json; d=json.load(open('gpurun_out/final3/bench_$c.json')); r=d['roofline']
print('$c', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['bytes_per_launch'], r.get('traffic'), (d.get('parity') or {}).get('ok'), d['cpu_baseline']['value'])"; done
