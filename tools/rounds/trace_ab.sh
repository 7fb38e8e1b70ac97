#!/bin/bash
# Kernel-trace A/B (GPU box): per-kernel average durations of one short C4
# bench run per setting (no PMC). Usage:
#   SETTINGS="base KR_STENCIL_DEPTH=2" bash tools/trace_ab.sh [bench args...]
args=${@:---steps 10 --warmup 2 --no-cpu-baseline --no-csr}
mkdir -p gpurun_out/trace_ab
export TMPDIR=/tmp
for s in ${SETTINGS:-base}; do
  d=gpurun_out/trace_ab/$s
  mkdir -p $d
  if [ "$s" = base ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py $args > $d/bench.log 2>&1 || exit $?
  else
    export "$s"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py $args > $d/bench.log 2>&1 || exit $?
    unset "${s%%=*}"
  fi
  echo "== $s $(grep -o '"value": [0-9.]*' $d/bench.log | head -1)"
  f=$(find $d -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'EOF'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "stencil" in n or "spmv" in n:
        print(f'{n[:60]:60s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1e6:8.3f} ms')
EOF
done
