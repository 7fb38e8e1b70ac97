"""Worker of tests/test_gpu_rccl.py (started by torch.distributed.run, 2-4
ranks): the v3/gpu/mpi solvers over a real RCCL communicator against the
oracle. Both ranks may share one GPU: each rank gets its own NCCL_HOSTID so
RCCL treats them as two hosts (socket transport over loopback) instead of
refusing a duplicate GPU -- test infrastructure only, the product path is
unchanged."""
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


def main():
    import importlib
    from oracle import matrices, v3cpu
    dist.init_process_group("gloo")
    world = dist.get_world_size()
    failures = []
    cases = [("poisson", "cg", 0), ("poisson", "mrr", 0), ("poisson", "kskipcg", 3),
             ("poisson", "kskipmrr", 4), ("poisson", "adaptivekskipmrr", 4),
             ("banded", "mrr", 0), ("banded", "kskipmrr", 3)]
    for mat, method, k in cases:
        # 12^3 Poisson (short rows, row walk) / banded 27 nnz per row (DIA kernel)
        A = matrices.poisson(12, 3) if mat == "poisson" else matrices.banded(3000, 13, 64, 0)
        n = A.shape[0]
        b = np.random.default_rng(5).standard_normal(n)
        rows = [n * r // world for r in range(world + 1)]
        local = A[rows[RANK]:rows[RANK + 1]]
        fn = getattr(importlib.import_module(f"parallel_krylov_amd.v3.gpu.mpi.{method}"), method)
        kw = dict(tol=1e-10, maxiter=400)
        if k:
            kw["k"] = k
        runs = []
        for dev_scalars in (("1", "0") if method in ("cg", "mrr") else ("1",)):
            os.environ["KR_DEVICE_SCALARS"] = dev_scalars
            with contextlib.redirect_stdout(io.StringIO()):
                x, info = fn(None, local, b, **kw)
            runs.append((x, info))
        if RANK != 0:
            continue
        x, info = runs[0]
        with contextlib.redirect_stdout(io.StringIO()):
            x_ref, info_ref = getattr(v3cpu, method)(A, b, **kw)
        r, rr = info["residual"], info_ref["residual"]
        big = rr > 1e-6
        rel = float(np.max(np.abs(r[big] - rr[big]) / rr[big]))
        xr = float(np.linalg.norm(x.cpu().numpy() - x_ref) / np.linalg.norm(x_ref))
        ok = np.array_equal(info["nosl"], info_ref["nosl"]) and rel < 1e-8 and xr < 1e-7
        if len(runs) == 2:  # device-resident scalars == host scalars, bit for bit
            x2, info2 = runs[1]
            ok = ok and np.array_equal(info2["residual"], info["residual"]) and \
                np.array_equal(x2.cpu().numpy(), x.cpu().numpy())
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
