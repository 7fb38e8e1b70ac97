#!/bin/bash
# Diagnosis of the 8-rank shared-GPU collapse: bench.py with
# 8 ranks on ONE GPU (NCCL_HOSTID per rank) under the default HIP hardware
# queues per process (4) and under GPU_MAX_HW_QUEUES=2 / 1, and 4 ranks as the
# control. 8 processes x 4 queues oversubscribe the hardware queue slots;
# the scheduler then time-slices them.
mkdir -p gpurun_out/ranksq
export TMPDIR=/tmp NCCL_DEBUG=ERROR
run() {  # ranks, queues (default = unset), tag
  local n=$1 q=$2 tag=$3
  if [ -n "$q" ]; then export GPU_MAX_HW_QUEUES=$q; else unset GPU_MAX_HW_QUEUES; fi
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29700 + n + ${q:-0})) tests/bench_rank_wrapper.py \
    --gpus $n --n-side 64 --steps 4 --warmup 1 --no-cpu-baseline --no-csr > gpurun_out/ranksq/$tag.log 2>&1 || return $?
  grep "^{" gpurun_out/ranksq/$tag.log | tail -1 > gpurun_out/ranksq/$tag.json
  python -c "
import json; d=json.load(open('gpurun_out/ranksq/$tag.json'))
print('$tag', d['value'], 'it/s', d['ms_per_step'], 'ms/step', {k: v['avg_ms'] for k, v in d['kernels'].items()})"
}
# the driver's scheduling parameters (read-only module parameters)
for f in hws_max_conc_proc sched_policy mes cwsr_enable no_system_mem_limit; do
  echo "amdgpu.$f=$(cat /sys/module/amdgpu/parameters/$f 2>/dev/null || echo n/a)"
done > gpurun_out/ranksq/amdgpu_params.txt
cat gpurun_out/ranksq/amdgpu_params.txt
run 4 "" r4_default && run 8 2 r8_q2 && run 8 1 r8_q1 && run 8 "" r8_default
