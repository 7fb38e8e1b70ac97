mkdir -p gpurun_out/kx
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/kx/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/kx/pytest.log; grep FAILED gpurun_out/kx/pytest.log | head; [ $rc -ne 0 ] && exit $rc
SETTINGS="base KR_KSKIP_XDEFER=0 base KR_KSKIP_XDEFER=0" bash tools/env_ab.sh --steps 20 --warmup 3 --no-cpu-baseline --no-csr
