"""The one-process-per-GPU family over a real RCCL communicator with several
ranks, on a one-GPU box: tests/rccl_2rank_worker.py gives every rank its own
NCCL_HOSTID, so RCCL runs the ranks as separate hosts (socket transport on
loopback) on the shared GPU instead of refusing a duplicate device. Covers
the RCCL halo exchange (split interior/boundary SpMV), the Gram all-gather
and the device-resident CG/MrR scalars across ranks, against the oracle."""
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ranks", [2, 3, 4])
def test_mpi_family_over_rccl(ranks):
    env = dict(os.environ, NCCL_DEBUG="ERROR")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ranks}", "--master-addr=127.0.0.1",
           f"--master-port={29620 + ranks}", os.path.join(REPO, "tests", "rccl_2rank_worker.py")]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=110)
    out = "\n".join(l for l in (p.stdout + p.stderr).splitlines() if "WARN" not in l)
    assert p.returncode == 0, out[-3000:]
    assert out.count("-> ok") == 7, out[-3000:]


@pytest.mark.parametrize("shards,stage", [("2,2", "0"), ("2,1", "0"), ("1,3", "0"), ("2,2", "1")])
def test_mpi_family_several_shards_per_rank(shards, stage):
    """Several GPUs per rank (GPU_IDS range, v3/gpu/mpi/common.py:100-118):
    one RCCL rank per process, its shards exchanging halos by device copies
    and with the other rank over RCCL; equal to the same partition run in
    one process bit for bit, and to the oracle. stage=1 routes every RCCL
    piece through the communicator-device staging buffers (the path of
    shards on other GPUs than the communicator's)."""
    env = dict(os.environ, NCCL_DEBUG="ERROR", KR_HYBRID_STAGE=stage)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=2", "--master-addr=127.0.0.1",
           f"--master-port={29640 + int(shards.replace(',', '')) % 97 + 50 * int(stage)}",
           os.path.join(REPO, "tests", "rccl_2rank_worker.py"), "--shards", shards]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=110)
    out = "\n".join(l for l in (p.stdout + p.stderr).splitlines() if "WARN" not in l)
    # the solver lines and every rank's error, not torchrun's own traceback
    brief = "\n".join(l for l in out.splitlines()
                      if "nosl" in l or "Error" in l or l.startswith("[rank"))
    assert p.returncode == 0, brief[-4000:]
    assert out.count("-> ok") == 9, brief[-4000:]


def test_bench_two_ranks_json_line():
    """bench.py --gpus 2 under torch.distributed.run (the driver's N>1 launch):
    rank 0 prints one JSON line for the whole job."""
    import json
    env = dict(os.environ, NCCL_DEBUG="ERROR")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29631",
           os.path.join(REPO, "tests", "bench_rank_wrapper.py"), "--gpus", "2", "--n-side", "48",
           "--steps", "4", "--warmup", "1", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 4 and rec["value"] > 0
    assert rec["scaling"] == "strong" and rec["cpu_baseline"] is None
    assert rec["roofline"]["bound"] == "hbm"
