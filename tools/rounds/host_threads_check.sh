export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_order.py tests/test_gpu_stencil.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_ms.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ms.log
[ $rc -ne 0 ] && exit $rc
for ht in 1 0; do
  KR_HOST_THREADS=$ht timeout -k 10 300 python bench.py --local-shards 8 --steps 12 --warmup 2 --no-cpu-baseline --no-csr > gpurun_out/ls8_ht$ht.log 2>&1 || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/ls8_ht$ht.log').read().strip().splitlines()[-1])
print('HT=$ht', d['value'], d['ms_per_step'], d.get('host'))"
done
bash tools/ranks_queues.sh
