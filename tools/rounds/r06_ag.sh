#!/bin/bash
# Round 6 (GPU box): the driver's N = 2 launch rehearsed on the final tree (two
# ranks sharing the one GPU over RCCL, tests/bench_rank_wrapper.py as in r06h).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06ag
mkdir -p $out
NCCL_DEBUG=ERROR timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
    --master-addr=127.0.0.1 --master-port=29641 tests/bench_rank_wrapper.py --gpus 2 --steps 4 \
    --warmup 1 > $out/rehearse_n2.log 2>&1 || { tail -30 $out/rehearse_n2.log; exit 1; }
grep "^{" $out/rehearse_n2.log | tail -1 > $out/rehearse_bench_n2.json
python3 -c "
import json; d=json.load(open('$out/rehearse_bench_n2.json')); print('n2', d['value'], d['config']['parallelism'], (d.get('parity') or {}).get('ok'), (d.get('csr') or {}).get('value'))"
