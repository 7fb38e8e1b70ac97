#!/bin/bash
# Round 6 (GPU box): box-pair GPU tests at the whole-line (XS = 1) no-halo build,
# then a same-box C4 A/B over the storing pair's x segments (KR_ST2B_XS) and the
# step walks' plane segments (KR_STEP2_Z), then ONE graph_cost capture variant
# (GMODE / GNSPMV; last: a crash ends the call).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06c
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_box_pair.py > $out/box_tests.txt 2>&1 || { tail -40 $out/box_tests.txt; exit 1; }
tail -2 $out/box_tests.txt
for rep in 1 2; do
  for env in "KR_ST2B_XS=4" "KR_ST2B_XS=1" "KR_STEP2_Z=8" "KR_STEP2_Z=32"; do
    env $env timeout -k 10 200 python bench.py --config C4 --steps 8 --warmup 2 --no-cpu-baseline \
        --no-csr --profile-every 1 > $out/c4_${env}_$rep.json 2> $out/c4_${env}_$rep.err || exit $?
    python - $out/c4_${env}_$rep.json "$env" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[2]:14s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
g=$out/graph_s2_m${GMODE:-8}_n${GNSPMV:-9}.txt
timeout -k 10 60 ./tools/micro/graph_cost 2 ${GNSPMV:-9} 200 64 ${GMODE:-8} > $g 2>&1
echo "exit $?" >> $g
tail -6 $g
