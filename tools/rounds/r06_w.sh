#!/bin/bash
# Round 6 (GPU box): the box pairs' DPP +-1 operands per level (KR_ST2B_DPP
# bits: 0/1 the storing pair's level 1/2, 2/3 the products-only pair's).
# C4 same-box A/B, two reps: the library (3), 1, 2, 7, 11; events per kernel.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06w
mkdir -p $out
for rep in 1 2; do
  for v in 3 1 2 7 11; do
    lib=parallel-krylov_amd/libkrylov_amd.so
    [ $v != 3 ] && lib=parallel-krylov_amd/libkrylov_amd_dpp$v.so
    KRYLOV_AMD_LIB=$(realpath $lib) timeout -k 10 200 python bench.py --steps 8 --warmup 2 \
        --no-cpu-baseline --no-csr --profile-every 1 > $out/dpp${v}_$rep.json 2> $out/dpp${v}_$rep.err || exit $?
    python - $out/dpp${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv2x2"))
print(f"dpp{sys.argv[2]:3s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
