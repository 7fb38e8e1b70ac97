"""Diagnostic (GPU box): where does the 3-shard mixed stencil / row-walk SpMV differ from scipy?"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import test_gpu_stencil as t  # noqa: E402
from parallel_krylov_amd.system import KrylovSystem, balanced_partition  # noqa: E402

for name in ("box32x32x7", "p3d64"):
    A = t.MATRICES[name]()
    n = A.shape[0]
    x = np.random.default_rng(5).standard_normal(n)
    ref = A @ x
    for env in ({}, {"KR_OVERLAP": "0"}, {"KR_STENCIL": "0"}):
        for k in ("KR_OVERLAP", "KR_STENCIL"):
            os.environ.pop(k, None)
        os.environ.update(env)
        part = balanced_partition(n, 3)
        sysm = KrylovSystem(n, part, [0, 0, 0])
        sysm.set_matrix(A)
        sysm.finalize()
        sc = [sysm.shard_sched(s) for s in range(3)]
        y = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
        bad = np.nonzero(y != ref)[0]
        print(name, env, "part", part, "sched", [(s["int_lo"], s["int_hi"], s["stencil_walk"], s["spmv_grid"]) for s in sc],
              "bad", bad[:10].tolist(), [(float(y[i]), float(ref[i])) for i in bad[:3]], flush=True)
        sysm.close()
