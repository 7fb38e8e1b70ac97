#!/bin/bash
# Round 6 (GPU box): the box pairs' +-1 operands. The pair tests on the DPP
# variant (KR_ST2B_DPP=1: own-row values by wave_shr / wave_shl, the wave's
# edge rows from LDS), then C4 same-box A/B, twice: the library, the ablation
# ab4 (the +-1 operands from the own rows: wrong results, the LDS reads'
# price) and the DPP variant; events per kernel.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06u
mkdir -p $out
dpp=$(realpath parallel-krylov_amd/libkrylov_amd_dpp.so)
KRYLOV_AMD_LIB=$dpp timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_box_pair.py > $out/pytest_dpp.txt 2>&1 || { tail -30 $out/pytest_dpp.txt; exit 1; }
tail -2 $out/pytest_dpp.txt
for rep in 1 2; do
  for v in lib ab4 dpp; do
    lib=parallel-krylov_amd/libkrylov_amd.so
    [ $v = ab4 ] && lib=parallel-krylov_amd/libkrylov_amd_ab4.so
    [ $v = dpp ] && lib=parallel-krylov_amd/libkrylov_amd_dpp.so
    KRYLOV_AMD_LIB=$(realpath $lib) timeout -k 10 200 python bench.py --steps 8 --warmup 2 \
        --no-cpu-baseline --no-csr --profile-every 1 > $out/${v}_$rep.json 2> $out/${v}_$rep.err || exit $?
    python - $out/${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[2]:4s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
