mkdir -p gpurun_out/diasym
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/diasym/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/diasym/pytest.log; grep FAILED gpurun_out/diasym/pytest.log | head; [ $rc -ne 0 ] && exit $rc
SETTINGS="base KR_DIA_SYM=0 base KR_DIA_SYM=0" bash tools/env_ab.sh --config C3 --steps 200 --warmup 20 --no-cpu-baseline --no-csr || exit $?
SETTINGS="base KR_DIA_SYM=0" bash tools/env_ab.sh --config C5 --steps 6 --warmup 2 --no-cpu-baseline --no-csr
