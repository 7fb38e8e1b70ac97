#!/bin/bash
# Round 6 (GPU box): DPP +-1 operands in the storing box pair (KR_ST2B_DPP=1,
# the new default). The pair tests and C4's full-size box-vs-dual bitwise
# test on the library, then C4 same-box A/B against the previous library
# (libkrylov_amd_r06prev.so), three times, events per kernel.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06v
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_box_pair.py "tests/test_gpu_fullsize.py::test_c4_fullsize_box_walks_bitwise_dual_path" \
    > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -2 $out/pytest.txt
for rep in 1 2 3; do
  for v in prev new; do
    lib=parallel-krylov_amd/libkrylov_amd.so
    [ $v = prev ] && lib=parallel-krylov_amd/libkrylov_amd_r06prev.so
    KRYLOV_AMD_LIB=$(realpath $lib) timeout -k 10 200 python bench.py --steps 8 --warmup 2 \
        --no-cpu-baseline --no-csr --profile-every 1 > $out/${v}_$rep.json 2> $out/${v}_$rep.err || exit $?
    python - $out/${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[2]:4s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
