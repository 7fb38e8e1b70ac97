# GPU suite, then the C3 / C5 profiles (trace + PMC passes), stopping at the first failure.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_round.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_round.log; grep FAILED gpurun_out/pytest_round.log | head; [ $rc -ne 0 ] && exit $rc
bash tools/profile.sh r02f_C3 --config C3 --steps 50 --warmup 5 --no-cpu-baseline --no-csr > /dev/null || exit $?
bash tools/profile.sh r02f_C5 --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-csr > /dev/null || exit $?
CONFIGS="C3 C5" bash tools/bench_configs.sh
