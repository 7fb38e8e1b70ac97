# Grouped finalize: multi-shard GPU tests, then the slab / 8-local-shard bench.
export TMPDIR=/tmp
mkdir -p gpurun_out/grp
timeout -k 10 900 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_poison.py tests/test_gpu_solvers.py tests/test_pipecg.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/grp/tests.txt 2>&1; rc=$?
tail -3 gpurun_out/grp/tests.txt
[ $rc -eq 0 ] || exit $rc
bash tools/rounds/slab_run.sh
