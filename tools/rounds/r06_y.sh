#!/bin/bash
# Round 6 (GPU box): the step pair + head walk with DPP +-1 operands (KR_STEP_DPP=28)
# against the library (0), four alternating reps, C4 events per kernel.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06y
mkdir -p $out
for rep in 1 2 3 4; do
  for v in 0 28; do
    lib=parallel-krylov_amd/libkrylov_amd.so
    [ $v != 0 ] && lib=parallel-krylov_amd/libkrylov_amd_dpp$v.so
    KRYLOV_AMD_LIB=$(realpath $lib) timeout -k 10 200 python bench.py --steps 16 --warmup 2 \
        --no-cpu-baseline --no-csr --profile-every 1 > $out/sdpp${v}_$rep.json 2> $out/sdpp${v}_$rep.err || exit $?
    python - $out/sdpp${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"sdpp{sys.argv[2]:3s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
