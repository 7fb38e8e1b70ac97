#!/bin/bash
# A/B of the symmetric DIA walk on one box: C5 (and C3) bench lines under
# KR_* settings given as "NAME=VALUE[,NAME=VALUE]" words ("base" = defaults).
# Usage: CONFIG=C5 bash tools/diaw_ab.sh base KR_DIA_WALK=0 KR_DIAW_GRID=4096 ...
cfg=${CONFIG:-C5}
st=${STEPS:-6}
mkdir -p gpurun_out/diaw
for v in "$@"; do
  env_args=()
  if [ "$v" != "base" ]; then IFS=',' read -ra kv <<< "$v"; env_args=("${kv[@]}"); fi
  tag=$(echo "$cfg_$v" | tr '=,' '__')
  timeout -k 10 300 env "${env_args[@]}" python bench.py --config $cfg --steps $st --warmup 2 \
      --no-cpu-baseline --no-csr --profile-every 1 > gpurun_out/diaw/${cfg}_$tag.json 2> gpurun_out/diaw/${cfg}_$tag.err || exit $?
  python - "$cfg" "$v" "gpurun_out/diaw/${cfg}_$tag.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[1]} {sys.argv[2]:28s} {d['value']:9.2f} it/s | {ks}", flush=True)
PY
done
