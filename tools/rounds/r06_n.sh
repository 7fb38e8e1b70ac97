#!/bin/bash
# Round 6 (GPU box), final tree: the 8-GPU layout on one GPU -- the 512^3 system
# as 8 in-process shards (the single-process multi-GPU family's layout), one
# rank's 64-plane slab (duals: what a rank runs; box: as its own box), and the
# driver's N = 4 launch rehearsed at full size (4 ranks sharing the GPU).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06n
mkdir -p $out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py $BARGS --no-cpu-baseline --no-csr > $out/$tag.json 2> $out/$tag.err || exit $?
  python - $out/$tag.json "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[2]:12s} {d['value']:9.2f} it/s | {d['config']['parallelism']} | {ks}", flush=True)
PY
}
BARGS="--steps 8 --warmup 2 --local-shards 8" run ls8 KR_NONE=1
BARGS="--nz 64 --steps 40 --warmup 4" run slab_duals KR_BOX=0
BARGS="--nz 64 --steps 40 --warmup 4" run slab_box KR_NONE=1
NCCL_DEBUG=ERROR timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
    --master-addr=127.0.0.1 --master-port=29651 tests/bench_rank_wrapper.py --gpus 4 --steps 3 \
    --warmup 1 --no-csr > $out/rehearse_n4.log 2>&1 || { tail -30 $out/rehearse_n4.log; exit 1; }
grep "^{" $out/rehearse_n4.log | tail -1 > $out/rehearse_bench_n4.json
python3 -c "
import json; d=json.load(open('$out/rehearse_bench_n4.json')); print('n4', d['value'], d['config']['parallelism'])"
