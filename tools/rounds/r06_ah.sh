#!/bin/bash
# Round 6 (GPU box): longer box walks. The pair tests and C4's full-size
# box-vs-dual bitwise test with one 512-plane walk per column (KR_ST2B_Z=1,
# KR_STEP2_Z=1), then C4, three alternating reps: the defaults (4 segments:
# 128-plane walks), the pairs at 2 / 1 segments, the step walks at 2 / 1.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06ah
mkdir -p $out
KR_ST2B_Z=1 KR_STEP2_Z=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_box_pair.py "tests/test_gpu_fullsize.py::test_c4_fullsize_box_walks_bitwise_dual_path" \
    > $out/pytest_z1.txt 2>&1 || { tail -30 $out/pytest_z1.txt; exit 1; }
tail -1 $out/pytest_z1.txt
run() {  # tag, then env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-csr \
      --profile-every 1 > $out/$tag.json 2> $out/$tag.err || exit $?
  python - $out/$tag.json "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[2]:8s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
}
for rep in 1 2 3; do
  run base_$rep KR_NONE=1
  run p2_$rep KR_ST2B_Z=2
  run p1_$rep KR_ST2B_Z=1
  run s2_$rep KR_STEP2_Z=2
  run s1_$rep KR_STEP2_Z=1
done
