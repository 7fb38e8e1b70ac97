mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_order.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "dia or banded or band" > gpurun_out/symup_t.log 2>&1
rc=$?; tail -2 gpurun_out/symup_t.log; grep FAILED gpurun_out/symup_t.log | head -5; [ $rc -ne 0 ] && exit $rc
SETTINGS="base KR_DIA_SYMUP=0 KR_DIA_SYM=0 base KR_DIA_SYMUP=0" bash tools/env_ab.sh --config C3 --steps 200 --warmup 20 --no-cpu-baseline --no-csr || exit $?
SETTINGS="base KR_DIA_SYMUP=0 KR_DIA_SYM=0" bash tools/env_ab.sh --config C5 --steps 6 --warmup 2 --no-cpu-baseline --no-csr
