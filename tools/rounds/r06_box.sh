#!/bin/bash
# Round 6: the box fused basis pair (KR_ST2=3) -- its GPU tests, then a
# same-box A/B of C4 against the dual launches (KR_ST2=0).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_box_pair.py > gpurun_out/r06/box_tests.txt 2>&1 || { tail -30 gpurun_out/r06/box_tests.txt; exit 1; }
tail -3 gpurun_out/r06/box_tests.txt
for rep in 1 2; do
  for st2 in 0 3; do
    KR_ST2=$st2 timeout -k 10 240 python bench.py --config C4 --steps 8 --warmup 2 --no-cpu-baseline \
        --no-csr --profile-every 1 > gpurun_out/r06/c4_st2_${st2}_$rep.json 2> gpurun_out/r06/c4_st2_${st2}_$rep.err || exit $?
    python - gpurun_out/r06/c4_st2_${st2}_$rep.json $st2 <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"KR_ST2={sys.argv[2]} {d['value']:8.2f} it/s parity={d.get('parity', {}).get('ok')} | {ks}", flush=True)
PY
  done
done
