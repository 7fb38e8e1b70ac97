# The 8-GPU per-rank share on one GPU (512^2 x 64-plane slab, no exchange)
# and the 512^3 system as 8 in-process shards on one GPU.
export TMPDIR=/tmp
mkdir -p gpurun_out/slab
timeout -k 10 300 python bench.py --nz 64 --steps 200 --warmup 20 --no-cpu-baseline --no-csr > gpurun_out/slab/slab64.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --local-shards 8 --steps 30 --warmup 3 --no-cpu-baseline --no-csr > gpurun_out/slab/ls8.log 2>&1 || exit $?
for f in slab64 ls8; do
  tail -1 gpurun_out/slab/$f.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], json.dumps(d.get('host')))"
done
