# The whole GPU suite, then the default bench line (C4).
export TMPDIR=/tmp
mkdir -p gpurun_out/full
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/full/pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/full/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/full/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/full/bench_default.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('C4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['ok'], d['parity']['entries'], d['cpu_baseline']['value'], d['csr']['value'])"
