# Round-end check of the final tree: the whole GPU suite, smoke, then every
# bench line (tools/rounds/final_bench.sh: C4 default + C1-C3, C5 with CPU baselines).
export TMPDIR=/tmp
mkdir -p gpurun_out/final4
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/final4/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/final4/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/final4/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final4/smoke.txt 2>&1 || { cat gpurun_out/final4/smoke.txt; exit 1; }
tail -1 gpurun_out/final4/smoke.txt
bash tools/rounds/final_bench.sh || exit $?
cp gpurun_out/final/bench_C*.json gpurun_out/final4/
