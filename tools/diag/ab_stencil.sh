# A/B of the stencil walk mapping on one box: C4 cube and the 8-GPU slab
mkdir -p gpurun_out/ab
run() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-csr $BARGS > gpurun_out/ab/$name.log 2>&1 || return $?
  python -c "
import json; l=[x for x in open('gpurun_out/ab/$name.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$name', d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items() if k.startswith('spmv')})"
}
for rep in 1 2; do
  BARGS=""
  run cube_pm$rep KR_STENCIL_PM=1 || exit 1
  run cube_plane$rep KR_STENCIL_PM=0 || exit 1
  BARGS="--nz 64"
  run slab_pm$rep KR_STENCIL_PM=1 || exit 1
  run slab_plane$rep KR_STENCIL_PM=0 || exit 1
done
