#!/bin/bash
# Round 6 (GPU box): the walks' result stores, non-temporal or plain
# (KR_WALK_NT bit 0: the storing pair's, bit 1: the step walks'). C4, three
# alternating reps of the library (3), 2 (pair stores plain), 1 (step walks'
# stores plain); events per kernel.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06af
mkdir -p $out
for rep in 1 2 3; do
  for v in 3 2 1; do
    lib=parallel-krylov_amd/libkrylov_amd.so
    [ $v != 3 ] && lib=parallel-krylov_amd/libkrylov_amd_dpp$v.so
    KRYLOV_AMD_LIB=$(realpath $lib) timeout -k 10 200 python bench.py --steps 16 --warmup 2 \
        --no-cpu-baseline --no-csr --profile-every 1 > $out/nt${v}_$rep.json 2> $out/nt${v}_$rep.err || exit $?
    python - $out/nt${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"nt{sys.argv[2]} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
