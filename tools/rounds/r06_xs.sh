#!/bin/bash
# Round 6: the x-segmented box pair -- its GPU tests, then C4 over KR_ST2B_XS.
export TMPDIR=/tmp
mkdir -p gpurun_out/r06x
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_box_pair.py > gpurun_out/r06x/box_tests.txt 2>&1 || { tail -40 gpurun_out/r06x/box_tests.txt; exit 1; }
tail -2 gpurun_out/r06x/box_tests.txt
for rep in 1 2; do
for xs in 4 2 1; do
  KR_ST2B_XS=$xs timeout -k 10 200 python bench.py --config C4 --steps 8 --warmup 2 --no-cpu-baseline \
      --no-csr --profile-every 1 > gpurun_out/r06x/c4_xs${xs}_$rep.json 2> gpurun_out/r06x/c4_xs${xs}_$rep.err || exit $?
  python - gpurun_out/r06x/c4_xs${xs}_$rep.json $xs <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"XS={sys.argv[2]} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
done
done
