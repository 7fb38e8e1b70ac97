#!/bin/bash
# One bench line per BASELINE config (single GPU).
mkdir -p gpurun_out
for c in ${CONFIGS:-C1 C2 C3 C5}; do
  timeout -k 10 600 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/cfg_$c.log 2>&1 || { echo "$c failed rc=$?"; tail -5 gpurun_out/cfg_$c.log; exit 1; }
  python - "$c" <<'PY'
import json, sys
c = sys.argv[1]
rec = json.loads(open(f"gpurun_out/cfg_{c}.log").read().strip().splitlines()[-1])
ks = " ".join(f"{k}={d['avg_ms']:.3f}ms/{d['gbs']:.0f}GB/s" for k, d in rec["kernels"].items())
print(f"{c}: {rec['value']} it/s ms/step={rec['ms_per_step']} | {ks}")
PY
done
