export TMPDIR=/tmp
mkdir -p gpurun_out/ilu2
timeout -k 10 600 python -u -m pytest tests/test_pipecg.py -m gpu -x -q --timeout 300 --timeout-method thread -k ilu > gpurun_out/ilu2/tests.txt 2>&1; rc=$?
tail -3 gpurun_out/ilu2/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/ilu_c2.py 256 > gpurun_out/ilu2/c2.json 2> gpurun_out/ilu2/c2.err; rc=$?
cat gpurun_out/ilu2/c2.json
exit $rc
