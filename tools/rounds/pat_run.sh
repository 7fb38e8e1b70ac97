export TMPDIR=/tmp
mkdir -p gpurun_out/pat
timeout -k 10 900 python -u -m pytest tests/test_gpu_stencil.py tests/test_gpu_order.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pat/tests.txt 2>&1; rc=$?
tail -3 gpurun_out/pat/tests.txt
[ $rc -eq 0 ] || exit $rc
LIBS="parallel-krylov_amd/libkrylov_amd.so parallel-krylov_amd/libkrylov_amd_old.so" STEPS=20 bash tools/lib_ab.sh || exit $?
LIBS="parallel-krylov_amd/libkrylov_amd.so parallel-krylov_amd/libkrylov_amd_old.so" STEPS=200 CONFIG=C2 bash tools/lib_ab.sh
