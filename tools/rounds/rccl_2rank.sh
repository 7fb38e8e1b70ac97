#!/bin/bash
# Two ranks over RCCL on whatever GPUs the box has (modulo mapping), small
# system, short limit: exercises the RCCL halo + Gram all-gather path.
mkdir -p gpurun_out
export TMPDIR=/tmp NCCL_DEBUG=WARN
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --n-side 64 --steps 5 \
  --warmup 1 --no-cpu-baseline > gpurun_out/rccl2.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/rccl2.log | tail -25
exit $rc
