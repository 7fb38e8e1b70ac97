#!/bin/bash
# Round 6: stencil / pair / solver GPU tests with the box pair as the default,
# then C4 over the box pair's walk segments (KR_ST2B_Z).
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_box_pair.py tests/test_gpu_stencil.py tests/test_gpu_solvers.py \
    > gpurun_out/r06c/tests.txt 2>&1 || { tail -40 gpurun_out/r06c/tests.txt; exit 1; }
tail -2 gpurun_out/r06c/tests.txt
for z in 16 8 32 4; do
  KR_ST2B_Z=$z timeout -k 10 200 python bench.py --config C4 --steps 8 --warmup 2 --no-cpu-baseline \
      --no-csr --profile-every 1 > gpurun_out/r06c/c4_z$z.json 2> gpurun_out/r06c/c4_z$z.err || exit $?
  python - gpurun_out/r06c/c4_z$z.json $z <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv2"))
print(f"Z={sys.argv[2]:3s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
done
