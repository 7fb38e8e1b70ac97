#!/bin/bash
# Round 6 (GPU box): the vector allocations' low address bits. The step walks'
# per-process bimodal times (e.g. the step triple 1.62 or 1.78 ms, r06ac) ask
# whether vectors streamed together collide in their low address bits;
# KR_VEC_STAGGER starts vector i at i x S bytes into its allocation. C4, four
# alternating reps of S = 0, 135168 (33 x 4 KiB), 1052672 (1 MiB + 4 KiB).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06ad
mkdir -p $out
for rep in 1 2 3 4; do
  for S in 0 135168 1052672; do
    KR_VEC_STAGGER=$S timeout -k 10 200 python bench.py --steps 16 --warmup 2 \
        --no-cpu-baseline --no-csr --profile-every 1 > $out/s${S}_$rep.json 2> $out/s${S}_$rep.err || exit $?
    python - $out/s${S}_$rep.json $S <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"S={sys.argv[2]:8s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
