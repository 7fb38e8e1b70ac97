#!/bin/bash
# Round 6 (GPU box): DPP +-1 operands also in the products-only pair's level 2
# (KR_ST2B_DPP=11) and the step triple's level 2 (KR_STEP_DPP=30), one build
# (libkrylov_amd_v.so), against the library: the box pair tests on it, then
# four alternating reps of C4 (16 steps), events per kernel.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06ac
mkdir -p $out
v=$(realpath parallel-krylov_amd/libkrylov_amd_v.so)
KRYLOV_AMD_LIB=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_box_pair.py > $out/pytest_v.txt 2>&1 || { tail -30 $out/pytest_v.txt; exit 1; }
tail -1 $out/pytest_v.txt
for rep in 1 2 3 4; do
  for t in lib v; do
    lib=$(realpath parallel-krylov_amd/libkrylov_amd.so)
    [ $t = v ] && lib=$v
    KRYLOV_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps 16 --warmup 2 \
        --no-cpu-baseline --no-csr --profile-every 1 > $out/${t}_$rep.json 2> $out/${t}_$rep.err || exit $?
    python - $out/${t}_$rep.json $t <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[2]:4s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
