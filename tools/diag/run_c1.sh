# C1/C2/C3 with and without the fused scalar steps (one box)
mkdir -p gpurun_out/c1
for cfg in C1 C2 C3; do
  for f in 0 1; do
    KR_FUSE_SCALAR=$f timeout -k 10 150 python bench.py --config $cfg --steps ${STEPS:-1000} --warmup 100 --no-cpu-baseline > gpurun_out/c1/${cfg}_f$f.log 2>&1 || exit $?
    python -c "
import json
l=[x for x in open('gpurun_out/c1/${cfg}_f$f.log') if x.startswith('{')]
d=json.loads(l[-1]); print('$cfg fuse=$f', d['value'], d['ms_per_step'])"
  done
done
