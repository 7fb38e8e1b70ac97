#!/bin/bash
# Round 6 (GPU box): C4 A/B of the box-walk knobs at the step pair + head
# build, the driver's N = 2 launch rehearsed at full size (two ranks on the one
# GPU, RCCL over loopback sockets), then graph_min pattern 7 (last).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06h
mkdir -p $out
for rep in 1 2; do
  for env in "KR_NONE=1" "KR_ST2B_Z=2" "KR_ST2B_XS=1" "KR_STEP2_Z=2" "KR_STEP2_Z=8"; do
    env $env timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-csr \
        --profile-every 1 > $out/c4_${env}_$rep.json 2> $out/c4_${env}_$rep.err || exit $?
    python - $out/c4_${env}_$rep.json "$env" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items() if k.startswith("spmv"))
print(f"{sys.argv[2]:13s} {d['value']:8.2f} it/s | {ks}", flush=True)
PY
  done
done
NCCL_DEBUG=ERROR timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
    --master-addr=127.0.0.1 --master-port=29641 tests/bench_rank_wrapper.py --gpus 2 --steps 4 \
    --warmup 1 > $out/rehearse_n2.log 2>&1 || { tail -30 $out/rehearse_n2.log; exit 1; }
grep "^{" $out/rehearse_n2.log | tail -1 > $out/rehearse_bench_n2.json
python3 -c "
import json; d=json.load(open('$out/rehearse_bench_n2.json')); print('n2', d['value'], d['config']['parallelism'], (d.get('csr') or {}).get('value'))"
timeout -k 10 60 ./tools/micro/graph_min 7 > $out/graph_min7.txt 2>&1
echo "exit $?" >> $out/graph_min7.txt
tail -3 $out/graph_min7.txt
