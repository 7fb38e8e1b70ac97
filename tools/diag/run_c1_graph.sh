mkdir -p gpurun_out/hy gpurun_out/c1
KR_WORKER_INPROC=0 NCCL_DEBUG=ERROR timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29661 tests/rccl_2rank_worker.py --shards 2,1 > gpurun_out/hy/w21c.log 2>&1
echo "worker rc=$?"
for g in 0 1; do
  KR_GRAPH=$g timeout -k 10 120 python bench.py --config C1 --steps 2000 --warmup 200 --no-cpu-baseline > gpurun_out/c1/g$g.log 2>&1 || exit $?
done
