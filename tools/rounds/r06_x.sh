#!/bin/bash
# Round 6 (GPU box): DPP +-1 operands in the step walks (KR_STEP_DPP bits: 0/1
# the step pair's level 1/2, 2/3/4 the step pair + head's level 1/2/3). The
# pair tests on the all-DPP build (31), then C4 same-box A/B, two reps: the
# library (0), 3, 28, 31; events per kernel.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06x
mkdir -p $out
KRYLOV_AMD_LIB=$(realpath parallel-krylov_amd/libkrylov_amd_dpp31.so) timeout -k 10 400 python -u -m pytest -x -q \
    --timeout 200 --timeout-method thread -m gpu tests/test_gpu_box_pair.py > $out/pytest_dpp31.txt 2>&1 \
    || { tail -30 $out/pytest_dpp31.txt; exit 1; }
tail -2 $out/pytest_dpp31.txt
for rep in 1 2; do
  for v in 0 3 28 31; do
    lib=parallel-krylov_amd/libkrylov_amd.so
    [ $v != 0 ] && lib=parallel-krylov_amd/libkrylov_amd_dpp$v.so
    KRYLOV_AMD_LIB=$(realpath $lib) timeout -k 10 200 python bench.py --steps 8 --warmup 2 \
        --no-cpu-baseline --no-csr --profile-every 1 > $out/sdpp${v}_$rep.json 2> $out/sdpp${v}_$rep.err || exit $?
    python - $out/sdpp${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"sdpp{sys.argv[2]:3s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
