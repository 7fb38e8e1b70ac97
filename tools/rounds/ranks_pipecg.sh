#!/bin/bash
# One GPU-box session: bench.py under torch.distributed.run with 4 and 8 ranks
# sharing the GPU (NCCL_HOSTID per rank: socket transport; a functional check
# of the N-rank path, not a scaling measurement), the RCCL solver worker at 4
# ranks, and C2-size bench lines of the pipelined CG family.
mkdir -p gpurun_out/ranks
export TMPDIR=/tmp NCCL_DEBUG=ERROR
for n in 4 8; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29700 + n)) tests/bench_rank_wrapper.py --gpus $n \
    --n-side 64 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ranks/bench_$n.log 2>&1 || exit $?
  grep "^{" gpurun_out/ranks/bench_$n.log | tail -1 | cut -c1-300
done
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29720 tests/rccl_2rank_worker.py > gpurun_out/ranks/worker_4.log 2>&1 || exit $?
grep -c -- "-> ok" gpurun_out/ranks/worker_4.log
for m in pcg chronopoulos_gear gropp pipeline; do
  timeout -k 10 300 python bench.py --config C2 --method $m --steps 200 --warmup 20 --no-cpu-baseline \
    --no-csr > gpurun_out/ranks/C2_$m.log 2>&1 || exit $?
  grep "^{" gpurun_out/ranks/C2_$m.log | tail -1 > gpurun_out/ranks/bench_C2_$m.json
  python -c "
import json; d=json.load(open('gpurun_out/ranks/bench_C2_$m.json'))
print('$m', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
done
