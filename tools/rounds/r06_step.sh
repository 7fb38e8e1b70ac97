#!/bin/bash
# Round 6: the box step walks (triple + pairs) -- GPU tests, then C4 A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out/r06t
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_box_pair.py > gpurun_out/r06t/tests.txt 2>&1 || { tail -40 gpurun_out/r06t/tests.txt; exit 1; }
tail -2 gpurun_out/r06t/tests.txt
for rep in 1 2; do
  for env in "KR_STEP2=1" "KR_STEP3=0" "KR_STEP2=0"; do
    env $env timeout -k 10 200 python bench.py --config C4 --steps 8 --warmup 2 --no-cpu-baseline \
        --no-csr --profile-every 1 > gpurun_out/r06t/c4_${env}_$rep.json 2> /dev/null || exit $?
    python - gpurun_out/r06t/c4_${env}_$rep.json "$env" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[2]:11s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
