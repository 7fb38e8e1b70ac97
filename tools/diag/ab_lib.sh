# same-box A/B of two library builds: bash tools/diag/ab_lib.sh <lib.so> [bench args]
mkdir -p gpurun_out/ablib
alt=$1; shift
for rep in 1 2; do
  for v in base alt; do
    if [ $v = alt ]; then export KRYLOV_AMD_LIB=$alt; else unset KRYLOV_AMD_LIB; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-csr "$@" > gpurun_out/ablib/$v$rep.log 2>&1 || exit $?
    python -c "
import json; l=[x for x in open('gpurun_out/ablib/$v$rep.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$v$rep', d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items() if k.startswith('spmv')})"
  done
done
