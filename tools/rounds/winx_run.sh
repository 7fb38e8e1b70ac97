# DIA walk: own-row epilogue operands from the LDS window (KR_DIAW_WINX):
# the GPU suite at the new default, then same-box A/B on C5 and C3.
export TMPDIR=/tmp
mkdir -p gpurun_out/winx
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/winx/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/winx/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/winx/pytest_gpu.txt
LIBS="parallel-krylov_amd/libkrylov_amd.so parallel-krylov_amd/libkrylov_amd_winx0.so" CONFIG=C5 STEPS=2 bash tools/lib_ab.sh || exit $?
LIBS="parallel-krylov_amd/libkrylov_amd.so parallel-krylov_amd/libkrylov_amd_winx0.so" CONFIG=C3 STEPS=20 bash tools/lib_ab.sh || exit $?
