#!/bin/bash
# A/B of kernel variants: parity of the kernels under each, then the bench.
# Usage: VARIANTS="0 1" bash tools/ab.sh [bench args]
mkdir -p gpurun_out
export TMPDIR=/tmp
args=${@:---steps 10 --warmup 2 --no-cpu-baseline}
for v in ${VARIANTS:-0 1}; do
  KR_SPMV_VARIANT=$v timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider > gpurun_out/ab_test_$v.log 2>&1
  rc=$?; echo "variant $v kernels rc=$rc $(tail -1 gpurun_out/ab_test_$v.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for v in ${VARIANTS:-0 1}; do
  KR_SPMV_VARIANT=$v timeout -k 10 600 python bench.py $args > gpurun_out/ab_bench_$v.log 2>&1 || exit $?
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
rec = json.loads(open(f"gpurun_out/ab_bench_{v}.log").read().strip().splitlines()[-1])
ks = " ".join(f"{k}={d['avg_ms']:.3f}ms/{d['gbs']:.0f}GB/s" for k, d in rec["kernels"].items())
print(f"variant {v}: {rec['value']} it/s  {ks}")
PY
done
