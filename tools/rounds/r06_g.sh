#!/bin/bash
# Round 6 (GPU box): the box step pair + head (spmv_step2h) -- box-walk tests,
# then a same-box C4 A/B against the step pair + head launch (KR_STEP2H=0).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06g
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_box_pair.py > $out/box_tests.txt 2>&1 || { tail -60 $out/box_tests.txt; exit 1; }
tail -2 $out/box_tests.txt
for rep in 1 2; do
  for env in "KR_STEP2H=1" "KR_STEP2H=0"; do
    env $env timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-csr \
        --profile-every 1 > $out/c4_${env}_$rep.json 2> $out/c4_${env}_$rep.err || exit $?
    python - $out/c4_${env}_$rep.json "$env" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[2]:12s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
