mkdir -p gpurun_out/xdefer
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_rccl.py tests/test_gpu_fullsize.py tests/test_gpu_edge.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/xdefer/pytest_mrr.log 2>&1
rc=$?; tail -5 gpurun_out/xdefer/pytest_mrr.log; grep FAILED gpurun_out/xdefer/pytest_mrr.log | head; [ $rc -ne 0 ] && exit $rc
SETTINGS="base KR_MRR_XDEFER=0 base KR_MRR_XDEFER=0" bash tools/env_ab.sh --config C3 --steps 200 --warmup 20 --no-cpu-baseline --no-csr
