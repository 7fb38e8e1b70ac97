mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; grep FAILED gpurun_out/pytest_gpu.log | head; [ $rc -ne 0 ] && exit $rc
SETTINGS="base KR_STENCIL_Z=8 base KR_STENCIL_Z=8" bash tools/env_ab.sh --steps 30 --warmup 3 --no-cpu-baseline --no-csr
