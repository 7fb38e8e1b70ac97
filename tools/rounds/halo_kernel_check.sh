# Multi-shard GPU tests with the halo gather kernel, then the 8-local-shard
# bench (512^3 as 8 shards on one device) with KR_HALO_KERNEL=1 / 0:
# host enqueue and wait per outer iteration.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_order.py tests/test_gpu_stencil.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_halo.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_halo.log
[ $rc -ne 0 ] && exit $rc
for hk in 1 0 1 0; do
  KR_HALO_KERNEL=$hk timeout -k 10 300 python bench.py --local-shards 8 --steps 12 --warmup 2 --no-cpu-baseline --no-csr > gpurun_out/ls8_hk$hk.log 2>&1 || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/ls8_hk$hk.log').read().strip().splitlines()[-1])
print('HALO_KERNEL=$hk', d['value'], d['ms_per_step'], d.get('host'))"
done
