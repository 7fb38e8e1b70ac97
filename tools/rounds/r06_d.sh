#!/bin/bash
# Round 6 (GPU box): same-box C4 A/B of the library at a78acfe (round-6 re-entry)
# against the current one, the walk-segment knobs, the 8-GPU per-rank slab
# ceilings, then ONE graph_cost capture variant (last: a crash ends the call).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06d
mkdir -p $out
run() {  # tag, then env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-csr \
      --profile-every 1 $BARGS > $out/$tag.json 2> $out/$tag.err || exit $?
  python - $out/$tag.json "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[2]:16s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
}
base=$(realpath parallel-krylov_amd/libkrylov_amd_r06base.so)
for rep in 1 2; do
  run base_$rep KRYLOV_AMD_LIB=$base
  run new_$rep KR_NONE=1
  run stepz4_$rep KR_STEP2_Z=4
  run pairz4_$rep KR_ST2B_Z=4
  run pairz16_$rep KR_ST2B_Z=16
done
# one rank's 512^2 x 64-plane slab of the 8-GPU run: the box walks (a whole box)
# and the dual path (KR_BOX=0: what a rank whose slab borders halos runs)
BARGS="--nz 64 --steps 40 --warmup 4" run slab_box KR_NONE=1
BARGS="--nz 64 --steps 40 --warmup 4" run slab_duals KR_BOX=0
BARGS="--steps 8 --warmup 2" run c4_duals KR_BOX=0
g=$out/graph_s2_m${GMODE:-56}_n${GNSPMV:-1}.txt
timeout -k 10 60 ./tools/micro/graph_cost 2 ${GNSPMV:-1} 200 64 ${GMODE:-56} > $g 2>&1
echo "exit $?" >> $g
tail -6 $g
