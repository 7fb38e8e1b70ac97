# End-of-round measurements on one box: the default bench line (C4 with the
# CPU baseline and the plain-CSR sub-run), C1-C3/C5 lines, and the C4 + C5
# rocprofv3 trace + PMC passes (tools/profile.sh).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('C4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['ok'], d['parity']['entries'], d['cpu_baseline']['value'], d['csr']['value'])"
CONFIGS="C1 C2 C3 C5" bash tools/bench_configs.sh || exit $?
bash tools/profile.sh ${TAG:-r03f}_C4 > /dev/null || exit $?
bash tools/profile.sh ${TAG:-r03f}_C5 --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-csr > /dev/null || exit $?
echo done
