#!/bin/bash
mkdir -p gpurun_out
for v in 0 1 2; do
  KR_EW_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider -k "update or dot" > gpurun_out/ewt_$v.log 2>&1; echo "ew $v tests: $(tail -1 gpurun_out/ewt_$v.log)"
  KR_EW_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ewb_$v.log 2>&1 || exit $?
  python3 -c "
import json; r=json.loads(open('gpurun_out/ewb_$v.log').read().strip().splitlines()[-1]); print('ew $v', r['value'], {k:(v['avg_ms'],v['gbs']) for k,v in r['kernels'].items() if 'update' in k})"
done
