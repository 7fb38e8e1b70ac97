"""Runs bench.py as one rank of a multi-rank job on a one-GPU box
(tests/test_gpu_rccl.py): a distinct NCCL_HOSTID per rank lets RCCL run
ranks that share the GPU (socket transport on loopback). Test infrastructure
only: the driver runs bench.py itself, one rank per GPU."""
import os
import runpy
import sys

os.environ["NCCL_HOSTID"] = f"kr-test-rank-{os.environ['RANK']}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_IB_DISABLE", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.argv = [os.path.join(REPO, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
