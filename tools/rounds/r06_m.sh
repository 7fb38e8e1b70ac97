#!/bin/bash
# Round 6 (GPU box): C4 A/B of the box pairs' x segments at the final build:
# whole lines (default) against halves, for the storing and products-only pairs.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06m
mkdir -p $out
for rep in 1 2; do
  for env in "KR_NONE=1" "KR_ST2B_XS=2" "KR_ST2B_XS_PO=2" "KR_ST2B_XS=2 KR_ST2B_XS_PO=2"; do
    tag=$(echo $env | tr ' =' '_-')
    env $env timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-csr \
        --profile-every 1 > $out/c4_${tag}_$rep.json 2> $out/c4_${tag}_$rep.err || exit $?
    python - $out/c4_${tag}_$rep.json "$env" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[2]:30s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
