#!/bin/bash
# Same-box A/B of library builds (compile-time variants, Makefile EXTRA/OUT):
#   LIBS="a.so b.so" CONFIG=C5 bash tools/lib_ab.sh
# runs bench.py on each library in turn, twice (a b a b), one line per run.
cfg=${CONFIG:-C4}
st=${STEPS:-6}
mkdir -p gpurun_out/libab
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in $LIBS; do
    tag=$(basename $lib .so)_$rep
    KRYLOV_AMD_LIB=$(realpath $lib) timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup 2 \
        --no-cpu-baseline --no-csr --profile-every 1 > gpurun_out/libab/${cfg}_$tag.json 2> gpurun_out/libab/${cfg}_$tag.err || exit $?
    python - "$cfg" "$tag" "gpurun_out/libab/${cfg}_$tag.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[1]} {sys.argv[2]:24s} {d['value']:9.2f} it/s | {ks}", flush=True)
PY
  done
done
