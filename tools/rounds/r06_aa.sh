#!/bin/bash
# Round 6 (GPU box): the stencil walk reads only the outer row of a +-1 NEAR slot (the inner one is the lane's own other row).
# The stencil parity tests on the library, then a same-box A/B against the
# library built without it (KR_ST_AB=16: right results, timing only):
# one rank's 512^2 x 64-plane slab on the dual path (KR_BOX=0), C4 on the dual
# path, and C2 (CG, 256^3), twice each.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06aa
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_stencil.py > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -2 $out/pytest.txt
run() {  # tag, then env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-csr \
      --profile-every 1 $BARGS > $out/$tag.json 2> $out/$tag.err || exit $?
  python - $out/$tag.json "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[2]:16s} {d['value']:10.2f} {d['unit']} | {ks}", flush=True)
PY
}
off=$(realpath parallel-krylov_amd/libkrylov_amd_near0.so)
for rep in 1 2; do
  BARGS="--nz 64 --steps 40 --warmup 4" run slab_new_$rep KR_BOX=0
  BARGS="--nz 64 --steps 40 --warmup 4" run slab_off_$rep KR_BOX=0 KRYLOV_AMD_LIB=$off
  BARGS="--steps 8 --warmup 2" run c4d_new_$rep KR_BOX=0
  BARGS="--steps 8 --warmup 2" run c4d_off_$rep KR_BOX=0 KRYLOV_AMD_LIB=$off
  BARGS="--config C2 --steps 64 --warmup 8" run c2_new_$rep KR_NONE=1
  BARGS="--config C2 --steps 64 --warmup 8" run c2_off_$rep KRYLOV_AMD_LIB=$off
done
