"""Repeatability of one multi-shard solve: runs the same k-skip solve R times
per setting in one process and prints the history length and a hash of x, so a
run-to-run difference (an ordering bug) shows as differing lines.
Usage: python tools/race_probe.py R SETTING ...   (SETTING: KR_X=1,KR_Y=0 or base)"""
import contextlib
import hashlib
import io
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main(R, *settings, method="kskipcg", n_side=64, k=3, shards="0,0,0"):
    import importlib
    import numpy as np
    from conftest import golden_matrix  # noqa: E402
    A = golden_matrix(["poisson", n_side, 3])
    b = np.random.default_rng(3).standard_normal(A.shape[0])
    solver = getattr(importlib.import_module(f"parallel_krylov_amd.v3.gpu.{method}"), method)
    os.environ["KRYLOV_AMD_SHARDS"] = shards
    for setting in settings or ("base",):
        env = {} if setting == "base" else dict(kv.split("=") for kv in setting.split(","))
        saved = {key: os.environ.get(key) for key in env}
        os.environ.update(env)
        try:
            for r in range(R):
                with contextlib.redirect_stdout(io.StringIO()):
                    x, info = solver(A, b, tol=1e-10, maxiter=300, k=k)
                h = hashlib.sha1(x.cpu().numpy().tobytes()).hexdigest()[:12]
                res = np.asarray(info["residual"])
                print(f"{setting} run {r}: nosl {len(info['nosl'])} last {res[-1]:.6e} x {h}",
                      flush=True)
        finally:
            for key, v in saved.items():
                if v is None:
                    os.environ.pop(key, None)
                else:
                    os.environ[key] = v


if __name__ == "__main__":
    main(int(sys.argv[1]), *sys.argv[2:])
