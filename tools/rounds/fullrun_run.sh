# DIA walk: no mask loads over the run of full row blocks (KR_DIAW_FULLRUN):
# the DIA GPU tests, then same-box A/B on C5 and C3 (a b a b).
export TMPDIR=/tmp
mkdir -p gpurun_out/fullrun
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_order.py tests/test_gpu_solvers.py \
  tests/test_gpu_fullsize.py tests/test_gpu_edge.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/fullrun/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/fullrun/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/fullrun/pytest_gpu.txt
SETTINGS="base KR_DIAW_FULLRUN=0 base KR_DIAW_FULLRUN=0" bash tools/env_ab.sh --config C5 --steps 2 --warmup 1 --no-cpu-baseline --no-csr || exit $?
SETTINGS="base KR_DIAW_FULLRUN=0 base KR_DIAW_FULLRUN=0" bash tools/env_ab.sh --config C3 --steps 20 --warmup 2 --no-cpu-baseline --no-csr || exit $?
