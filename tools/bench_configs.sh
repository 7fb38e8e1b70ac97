# bench.py lines of C1..C5 on one box (each with its CPU baseline and, where
# the sample is the config's own system, the parity field; no CSR sub-run;
# NOCPU=1 skips the CPU leg), written to gpurun_out/configs/bench_<C>.json
mkdir -p gpurun_out/configs
for cfg in ${CONFIGS:-C1 C2 C3 C5}; do
  case $cfg in C1) st=2000; wu=200;; C2|C3) st=200; wu=20;; *) st=10; wu=2;; esac
  timeout -k 10 900 python bench.py --config $cfg --steps $st --warmup $wu ${NOCPU:+--no-cpu-baseline} --no-csr > gpurun_out/configs/$cfg.log 2>&1 || exit $?
  grep "^{" gpurun_out/configs/$cfg.log | tail -1 > gpurun_out/configs/bench_$cfg.json
  python -c "
import json; d=json.load(open('gpurun_out/configs/bench_$cfg.json'))
p=d.get('parity') or {}; c=d.get('cpu_baseline') or {}
print('$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], 'cpu', c.get('value'), 'parity', p.get('ok'), p.get('entries'), p.get('max_rel'))"
done
