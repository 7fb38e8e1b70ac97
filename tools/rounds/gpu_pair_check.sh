# Fused-basis-pair and ILU GPU tests, then the C4 bench with and without the pair.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_stencil.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "pair or box512 or aniso512" > gpurun_out/pytest_pair.log 2>&1
rc=$?; echo "pair rc=$rc"; tail -5 gpurun_out/pytest_pair.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_pipecg.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "ilu" > gpurun_out/pytest_ilu.log 2>&1
rc=$?; echo "ilu rc=$rc"; tail -5 gpurun_out/pytest_ilu.log
[ $rc -gt 1 ] && exit $rc
[ -n "$NO_BENCH" ] && exit 0
for st2 in 1 0; do
  KR_ST2=$st2 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-csr --profile-every 1 > gpurun_out/bench_st2_$st2.log 2>&1 || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/bench_st2_$st2.log').read().strip().splitlines()[-1])
print('ST2=$st2', d['value'], d['ms_per_step'], {k:(v['launches'],v['avg_ms']) for k,v in d['kernels'].items()})"
done
