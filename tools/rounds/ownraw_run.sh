# DIA walk: virtual steps' own-row operands from registers: DIA tests, then
# same-box A/B against the previous library on C3 (a b a b).
export TMPDIR=/tmp
mkdir -p gpurun_out/ownraw
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_order.py tests/test_gpu_solvers.py \
  tests/test_gpu_fullsize.py tests/test_gpu_edge.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/ownraw/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/ownraw/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/ownraw/pytest_gpu.txt
LIBS="parallel-krylov_amd/libkrylov_amd.so parallel-krylov_amd/libkrylov_amd_prev.so" CONFIG=C3 STEPS=20 bash tools/lib_ab.sh || exit $?
