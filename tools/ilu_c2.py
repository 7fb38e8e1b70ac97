"""PCG at C2's size with the ILU preconditioner next to Jacobi (review item 8).

The system is C2's: the 3-D 7-point Poisson matrix, n = 256 (N = 16.7M),
generated on the device. A SuperLU spilu at that size is out of reach on the
host, so the factors are ILU(0) (L unit lower, U upper, A's pattern, natural
order, no pivoting) computed here level by level: row i's pivot is
d_i = 6 - sum over its lower neighbours k of 1 / d_k, and the rows of one
level (x + y + z = s) depend only on level s - 1. They go through
kr_solve_set_precond_ilu like any (L, U, perm_r, perm_c) factors; their level
schedule is the hyperplanes, 766 levels of up to ~49,000 rows.

Runs (pcg, v1/threads/pipeline/pcg.py's algorithm):
  jacobi     d = diag(A) = 6, to relative residual 1e-8
  ilu        ILU(0) with wide levels over the grid (default KR_ILU_WIDE), to 1e-8
  ilu_wide0  ILU(0) with every level in one workgroup (KR_ILU_WIDE=0), 3 iterations
Prints one JSON line: iterations, seconds, ms per iteration and the sweeps'
ms per application (profile events).
  python tools/ilu_c2.py [n]
"""
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_krylov_amd.system import KrylovSystem  # noqa: E402


def ilu0_poisson3d(n):
    N = n ** 3
    i = np.arange(N, dtype=np.int64)
    x, y, z = i % n, (i // n) % n, i // (n * n)
    nbrs = [(z > 0, n * n), (y > 0, n), (x > 0, 1)]  # ascending column order
    s = x + y + z
    order = np.argsort(s, kind="stable")
    ends = np.cumsum(np.bincount(s))
    d = np.zeros(N)
    start = 0
    for e in ends:
        rows = order[start:e]
        acc = np.full(rows.size, 6.0)
        for m, off in nbrs:
            r = rows[m[rows]]
            acc[m[rows]] -= 1.0 / d[r - off]
        d[rows] = acc
        start = e
    del order, s

    def rows_of(entries):
        """CSR from per-row entry lists [(mask, column offset, values)], in
        ascending column order per row."""
        cnt = sum(m.astype(np.int64) for m, _, _ in entries)
        ptr = np.zeros(N + 1, np.int64)
        np.cumsum(cnt, out=ptr[1:])
        pos = ptr[:-1].copy()
        col = np.empty(ptr[-1], np.int32)
        val = np.empty(ptr[-1])
        for m, off, v in entries:
            r = np.nonzero(m)[0]
            col[pos[r]] = r + off
            val[pos[r]] = v[r] if isinstance(v, np.ndarray) else v
            pos[r] += 1
        return sp.csr_matrix((val, col, ptr), shape=(N, N))

    one = np.ones(N, bool)
    # L: -1 / d_k at the lower neighbours k (ascending), 1 on the diagonal
    lower = []
    for m, off in nbrs:
        v = np.zeros(N)
        v[m] = -1.0 / d[np.nonzero(m)[0] - off]
        lower.append((m, -off, v))
    L = rows_of(lower + [(one, 0, 1.0)])
    # U: d on the diagonal, -1 at the upper neighbours
    U = rows_of([(one, 0, d), (x < n - 1, 1, -1.0), (y < n - 1, n, -1.0),
                 (z < n - 1, n * n, -1.0)])
    return L, U, np.arange(N), np.arange(N)


def run(sysm, b, tol, maxiter, precond):
    kind, obj = precond
    if kind == "ilu":
        sysm.set_precond_ilu(obj)
    else:
        sysm.set_precond_ilu(None)
        sysm.set_precond(obj)
    sysm.solve("pcg", b, tol=tol, maxiter=2)  # warm-up (kernel loads, ILU upload)
    t0 = time.time()
    out = sysm.solve("pcg", b, tol=tol, maxiter=maxiter, profile=True)
    wall = time.time() - t0
    its = int(out.info["nosl"][-1])
    st = {k["name"]: k for k in out.kernel_stats}
    sw = st.get("ilu_sweeps")
    return dict(iterations=its, seconds=round(out.info["time"], 4), wall_s=round(wall, 3),
                ms_per_iteration=round(1e3 * out.info["time"] / max(its, 1), 4),
                final_residual=float(out.info["residual"][-1]), converged=out.converged,
                sweeps_ms_per_apply=round(sw["total_ms"] / sw["launches"], 4) if sw else None)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    N = n ** 3
    t0 = time.time()
    L, U, pr, pc = ilu0_poisson3d(n)
    t_fact = time.time() - t0
    sysm = KrylovSystem(N, [0, N], [0])
    sysm.gen_poisson(n, 3)
    sysm.finalize()
    b = sysm.rhs(1)
    rec = dict(system=f"3-D 7-point Poisson {n}^3 (N={N})", ilu="ILU(0), natural order",
               factor_host_s=round(t_fact, 1), l_nnz=int(L.nnz), u_nnz=int(U.nnz), levels=3 * n - 2)
    d6 = sysm.split(np.full(N, 6.0))
    rec["jacobi"] = run(sysm, b, 1e-8, 4000, ("diag", d6))
    rec["ilu"] = run(sysm, b, 1e-8, 4000, ("ilu", (L, U, pr, pc)))
    os.environ["KR_ILU_WIDE"] = "0"
    rec["ilu_wide0"] = run(sysm, b, 0.0, 3, ("ilu", (L, U, pr, pc)))
    os.environ.pop("KR_ILU_WIDE")
    sysm.close()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
