mkdir -p gpurun_out/xdefer
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_edge.py tests/test_gpu_stencil.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "device_scalars or matches_reference or persistent or edge or guard or maxiter" > gpurun_out/xdefer/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/xdefer/pytest.log; grep FAILED gpurun_out/xdefer/pytest.log | head; [ $rc -ne 0 ] && exit $rc
SETTINGS="base KR_CG_XDEFER=0 base KR_CG_XDEFER=0" bash tools/env_ab.sh --config C2 --steps 300 --warmup 30 --no-cpu-baseline --no-csr || exit $?
SETTINGS="base KR_CG_XDEFER=0" bash tools/env_ab.sh --config C1 --steps 2000 --warmup 200 --no-cpu-baseline --no-csr
