#!/bin/bash
# A/B of environment knobs on the bench. Usage:
#   SETTINGS="KR_SLAB=0 base A=1,B=2" bash tools/env_ab.sh [bench args]
# ("base" = no extra variable). Prints one line per setting.
mkdir -p gpurun_out
export TMPDIR=/tmp
args=${@:---steps 10 --warmup 2 --no-cpu-baseline}
# The first bench on a fresh box runs a few % slow (clocks / page-in): one
# untimed run first, so the first setting is not penalised.
timeout -k 10 600 python bench.py $args --no-profile > gpurun_out/envab_warm.log 2>&1 || exit $?
for set in ${SETTINGS:-base}; do
  tag=${set//[^A-Za-z0-9]/_}
  if [ "$set" = base ]; then
    timeout -k 10 600 python bench.py $args > gpurun_out/envab_$tag.log 2>&1 || exit $?
  else
    timeout -k 10 600 env ${set//,/ } python bench.py $args > gpurun_out/envab_$tag.log 2>&1 || exit $?
  fi
  python - "$tag" "$set" <<'PY'
import json, sys
tag, setting = sys.argv[1], sys.argv[2]
rec = json.loads(open(f"gpurun_out/envab_{tag}.log").read().strip().splitlines()[-1])
ks = " ".join(f"{k}={d['avg_ms']:.3f}ms/{d['gbs']:.0f}" for k, d in rec["kernels"].items())
print(f"{setting}: {rec['value']} it/s  {ks}", flush=True)
PY
done
