#!/bin/bash
# Same-box A/B of timing-only box-pair builds (tools/micro/pair_ab_build.sh),
# C4 with KR_ST2=3: the pair kernels' times per variant.
export TMPDIR=/tmp
mkdir -p gpurun_out/r06ab
for rep in 1 2; do
  for ab in $ABS; do
    KR_ST2=3 KRYLOV_AMD_LIB=$(realpath parallel-krylov_amd/libkrylov_amd_ab$ab.so) timeout -k 10 200 \
        python bench.py --config C4 --steps 6 --warmup 2 --no-cpu-baseline --no-csr --profile-every 1 \
        > gpurun_out/r06ab/ab${ab}_$rep.json 2> gpurun_out/r06ab/ab${ab}_$rep.err || exit $?
    python - gpurun_out/r06ab/ab${ab}_$rep.json $ab <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv2"))
print(f"ab={sys.argv[2]:3s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
