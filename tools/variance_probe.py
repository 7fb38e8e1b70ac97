"""Run-to-run variance of the C4 kernels: is it per process (where the
vectors landed in HBM) or per moment? Builds the 512^3 k-skip MrR system T
times per setting in one process (fresh allocations each time, settings
interleaved) and times B batches of S outer iterations on each, printing the
per-kernel averages (HIP events, every step sampled) and the wall rate.
Usage: python tools/variance_probe.py T B S [SETTING ...]
  SETTING = comma-separated KR_* assignments read at begin(), e.g.
  KR_VEC_POOL=1,KR_VEC_PAD=4096 ("base" = none)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(sysm, setting, t, B, S, k):
    import torch
    env = {} if setting == "base" else dict(kv.split("=") for kv in setting.split(","))
    saved = {key: os.environ.get(key) for key in env}
    os.environ.update(env)
    try:
        b = sysm.rhs(1 + t)
        sysm.begin("kskipmrr", b, None, tol=0.0, maxiter=(2 + B * S + 4) * (k + 1) + 2, k=k,
                   profile=1)
    finally:
        for key, v in saved.items():
            if v is None:
                os.environ.pop(key, None)
            else:
                os.environ[key] = v
    sysm.step(2)
    rates = []
    for bi in range(B):
        sysm.reset_kernel_stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sysm.step(S)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        rates.append(S * (k + 1) / el)
        ks = {r["name"]: r["total_ms"] / r["launches"] for r in sysm.kernel_stats()
              if r["launches"] and not r["name"].startswith("host_")}
        row = " ".join(f"{name.replace('spmv_step_mrr_', '').replace('spmv2_gram_mrr', 'dual')}"
                       f"={v:.3f}" for name, v in sorted(ks.items()) if v > 0.1)
        print(f"{setting} #{t} batch {bi}: {rates[-1]:7.1f} it/s (events on) | {row}", flush=True)
    sysm.finish("kskipmrr")
    del b
    return sum(rates) / len(rates)


def main(T=3, B=3, S=6, *settings, n_side=512, k=4):
    import torch
    from parallel_krylov_amd.system import KrylovSystem
    settings = settings or ("base",)
    n = n_side ** 3
    sysm = KrylovSystem(n, [0, n], [0], None)
    sysm.gen_poisson(n_side, 3)
    sysm.finalize()
    res = {s: [] for s in settings}
    for t in range(T):
        for s in settings:  # begin() reallocates the vectors
            res[s].append(run(sysm, s, t, B, S, k))
            torch.cuda.empty_cache()
    sysm.close()
    for s, r in res.items():
        print(f"SUMMARY {s}: mean {sum(r) / len(r):.1f} min {min(r):.1f} max {max(r):.1f} it/s",
              flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(*[int(v) for v in a[:3]], *a[3:])
