mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; grep FAILED gpurun_out/pytest_gpu.log | head; [ $rc -ne 0 ] && exit $rc
SETTINGS="base KR_EW_PREFETCH=0 base KR_EW_PREFETCH=0" bash tools/env_ab.sh --config C1 --steps 3000 --warmup 300 --no-cpu-baseline --no-csr || exit $?
SETTINGS="base KR_EW_PREFETCH=0" bash tools/env_ab.sh --config C3 --steps 200 --warmup 20 --no-cpu-baseline --no-csr
