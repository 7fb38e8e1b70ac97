export TMPDIR=/tmp
mkdir -p gpurun_out/ls8
for mode in 1 0 1 0; do
  KR_SHARED_STREAM=$mode timeout -k 10 300 python -u bench.py --local-shards 8 --steps 20 --warmup 3 --no-cpu-baseline --no-csr > gpurun_out/ls8/ss$mode.log 2>&1 || exit $?
  tail -1 gpurun_out/ls8/ss$mode.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('shared=$mode', d['value'], d['ms_per_step'], json.dumps(d.get('host')), d.get('parity',{}) and d['parity'].get('ok'))"
done
