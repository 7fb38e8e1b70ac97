#!/bin/bash
# Round 6 (GPU box): cost split of the box pairs by timing-only ablation builds
# (tools/micro/pair_ab_build.sh, KR_ST2B_AB bits; wrong results, never the
# library): the library, then each ablation, twice, C4 with events per kernel.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06p
mkdir -p $out
for rep in 1 2; do
  for ab in 0 $ABS; do
    lib=parallel-krylov_amd/libkrylov_amd.so
    [ $ab != 0 ] && lib=parallel-krylov_amd/libkrylov_amd_ab$ab.so
    KRYLOV_AMD_LIB=$(realpath $lib) timeout -k 10 200 python bench.py --steps 6 --warmup 2 \
        --no-cpu-baseline --no-csr --profile-every 1 > $out/ab${ab}_$rep.json 2> $out/ab${ab}_$rep.err || exit $?
    python - $out/ab${ab}_$rep.json $ab <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv2x2"))
print(f"ab={sys.argv[2]:3s} {ks}", flush=True)
PY
  done
done
