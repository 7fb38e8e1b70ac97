"""Worker of tests/test_gpu_rccl.py (started by torch.distributed.run, 2-4
ranks): the v3/gpu/mpi solvers over a real RCCL communicator against the
oracle. Both ranks may share one GPU: each rank gets its own NCCL_HOSTID so
RCCL treats them as two hosts (socket transport over loopback) instead of
refusing a duplicate GPU -- test infrastructure only, the product path is
unchanged.

``--shards 2,1`` gives rank r that many local shards on the GPU
(KRYLOV_AMD_RANK_SHARDS: several GPUs per rank, one RCCL rank per process).
Then rank 0 also runs the same global partition in-process (one process, all
shards) first: the RCCL run must equal it bit for bit (shard sums in global
shard order on both paths)."""
import contextlib
import io
import os
import sys

RANK = int(os.environ["RANK"])
os.environ["NCCL_HOSTID"] = f"kr-test-rank-{RANK}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_IB_DISABLE", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402


CASES = [("poisson", "cg", 0), ("poisson", "mrr", 0), ("poisson", "kskipcg", 3),
         ("poisson", "kskipmrr", 4), ("poisson", "adaptivekskipmrr", 4),
         ("banded", "mrr", 0), ("banded", "kskipmrr", 3)]
# several shards per rank: + the stencil kernel (32^3 Poisson, 8192-row shards)
CASES_LOCAL = CASES + [("p3d32", "cg", 0), ("p3d32", "adaptivekskipmrr", 6)]


def matrix(name):
    from oracle import matrices
    # 12^3 Poisson (short rows, row walk) / banded 27 nnz per row (DIA kernel)
    if name == "poisson":
        return matrices.poisson(12, 3)
    if name == "p3d32":
        return matrices.poisson(32, 3)
    return matrices.banded(3000, 13, 64, 0)


def in_process(A, b, part, method, kw):
    """The same global partition, every shard in this process (GPU 0)."""
    from parallel_krylov_amd.system import KrylovSystem
    import torch
    P = len(part) - 1
    sysm = KrylovSystem(A.shape[0], part, [0] * P)
    try:
        for s in range(P):
            sysm.adopt_csr(s, A[part[s]:part[s + 1]])
        sysm.finalize()
        bp = [torch.from_numpy(np.ascontiguousarray(b[part[s]:part[s + 1]])).to("cuda:0")
              for s in range(P)]
        out = sysm.solve(method, bp, None, tol=kw["tol"], maxiter=kw["maxiter"],
                         k=kw.get("k", 0))
        return torch.cat(out.x).cpu().numpy(), out.info
    finally:
        sysm.close()


def main():
    import importlib
    from oracle import gpu_order, v3cpu
    from parallel_krylov_amd.system import balanced_partition
    counts = None
    if "--shards" in sys.argv:
        counts = [int(t) for t in sys.argv[sys.argv.index("--shards") + 1].split(",")]
        os.environ["KRYLOV_AMD_RANK_SHARDS"] = ",".join(["0"] * counts[RANK])
    dist.init_process_group("gloo")
    world = dist.get_world_size()
    failures = []
    only = os.environ.get("KR_WORKER_CASES")  # diagnostics: e.g. "poisson:kskipcg"
    for mat, method, k in (CASES_LOCAL if counts else CASES):
        if only and f"{mat}:{method}" not in only.split(","):
            continue
        A = matrix(mat)
        n = A.shape[0]
        b = np.random.default_rng(5).standard_normal(n)
        rows = [n * r // world for r in range(world + 1)]
        local = A[rows[RANK]:rows[RANK + 1]]
        fn = getattr(importlib.import_module(f"parallel_krylov_amd.v3.gpu.mpi.{method}"), method)
        kw = dict(tol=1e-10, maxiter=400)
        if k:
            kw["k"] = k
        same = None
        part = [0]
        for r in range(world):
            part += [rows[r] + t for t in balanced_partition(rows[r + 1] - rows[r],
                                                             counts[r] if counts else 1)[1:]]
        if counts and RANK == 0 and os.environ.get("KR_WORKER_INPROC", "1") != "0":
            same = in_process(A, b, part, method, kw)
        runs = []
        for dev_scalars in (("1", "0") if method in ("cg", "mrr") else ("1",)):
            os.environ["KR_DEVICE_SCALARS"] = dev_scalars
            with contextlib.redirect_stdout(io.StringIO()):
                x, info = fn(None, local, b, **kw)
            runs.append((x, info))
        if RANK != 0:
            continue
        x, info = runs[0]
        exact = counts is not None and method in gpu_order.SPMV_ONLY_METHODS
        with contextlib.redirect_stdout(io.StringIO()):
            if exact:  # the oracle in the engine's summation order: bit for bit
                x_ref, info_ref = gpu_order.run(method, A, b, gpu_order.shard_scheds(A, part),
                                                **kw)
            else:
                x_ref, info_ref = getattr(v3cpu, method)(A, b, **kw)
        r, rr = info["residual"], info_ref["residual"]
        big = rr > 1e-6
        rel = float(np.max(np.abs(r[big] - rr[big]) / rr[big]))
        xr = float(np.linalg.norm(x.cpu().numpy() - x_ref) / np.linalg.norm(x_ref))
        ok = np.array_equal(info["nosl"], info_ref["nosl"]) and rel < 1e-8 and xr < 1e-7
        if exact:
            ok = ok and np.array_equal(r, rr) and np.array_equal(x.cpu().numpy(), x_ref)
        if len(runs) == 2:  # device-resident scalars == host scalars, bit for bit
            x2, info2 = runs[1]
            ok = ok and np.array_equal(info2["residual"], info["residual"]) and \
                np.array_equal(x2.cpu().numpy(), x.cpu().numpy())
        if same is not None:  # RCCL ranks x local shards == one process, bit for bit
            ok = ok and np.array_equal(same[1]["residual"], info["residual"]) and \
                np.array_equal(same[0], x.cpu().numpy())
        print(f"{mat} {method}: nosl {int(info['nosl'][-1])} vs {int(info_ref['nosl'][-1])}, "
              f"residual rel {rel:.1e}, x rel {xr:.1e} -> {'ok' if ok else 'FAIL'}", flush=True)
        if not ok:
            failures.append((mat, method))
    dist.barrier()
    dist.destroy_process_group()
    if failures:
        sys.exit(1)


if __name__ == "__main__":
    main()
