# diagnostics of the several-shards-per-rank worker: one torchrun per case list
mkdir -p gpurun_out/hy
i=0
for cases in "$@"; do
  i=$((i+1))
  KR_WORKER_CASES=$cases NCCL_DEBUG=ERROR timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=$((29670+i)) tests/rccl_2rank_worker.py --shards ${SHARDS:-2,1} > gpurun_out/hy/x$i.log 2>&1
  rc=$?
  echo "[$cases] rc=$rc"
  grep -h "nosl\|Error" gpurun_out/hy/x$i.log | grep -v "^\[rank.\]:  " | head -5
  if [ $rc -ne 0 ]; then exit $rc; fi
done
