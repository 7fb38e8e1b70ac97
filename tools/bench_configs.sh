# bench.py lines of C1..C5 on one box (no CPU baseline, no CSR sub-run),
# written to gpurun_out/configs/bench_<C>.json
mkdir -p gpurun_out/configs
for cfg in ${CONFIGS:-C1 C2 C3 C5}; do
  case $cfg in C1) st=2000; wu=200;; C2|C3) st=200; wu=20;; *) st=10; wu=2;; esac
  timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup $wu --no-cpu-baseline --no-csr > gpurun_out/configs/$cfg.log 2>&1 || exit $?
  grep "^{" gpurun_out/configs/$cfg.log | tail -1 > gpurun_out/configs/bench_$cfg.json
  python -c "
import json; d=json.load(open('gpurun_out/configs/bench_$cfg.json'))
print('$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
done
