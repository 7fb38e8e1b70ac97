mkdir -p gpurun_out/persist
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_edge.py -q -k "persistent or device_scalars or matches_reference" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/persist/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/persist/pytest.log; [ $rc -ne 0 ] && exit $rc
for e in 1 0; do
  KR_PERSIST=$e timeout -k 10 200 python bench.py --config C1 --steps 2000 --warmup 200 --no-cpu-baseline --no-csr > gpurun_out/persist/C1_$e.log 2>&1 || exit $?
  grep "^{" gpurun_out/persist/C1_$e.log | tail -1 | cut -c1-200
  python -c "
import json; d=json.loads(open('gpurun_out/persist/C1_$e.log').read().strip().splitlines()[-1]); print({k:(v['avg_ms'],v['launches']) for k,v in d['kernels'].items()})"
done
