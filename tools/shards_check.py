"""Full-size check of the partitioned path on one GPU: the headline system
(512^3 Poisson, k-skip MrR k=4) as 1 shard and as P in-process shards on the
same device (halo copies of one 512^2 plane per neighbour, shard partials
summed in shard order -- the layout of a P-GPU run). Prints the residual
histories' largest relative difference (dot-product order only) and the
outer-iteration time of each; exits non-zero if they disagree beyond 1e-10.
Usage: python tools/shards_check.py [side] [P] [outer]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(side, parts, outer, k=4):
    import torch
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition
    n = side ** 3
    sysm = KrylovSystem(n, balanced_partition(n, parts), [0] * parts)
    sysm.gen_poisson(side, 3)
    sysm.finalize()
    b = sysm.rhs(1)
    sysm.begin("kskipmrr", b, None, tol=0.0, maxiter=(outer + 2) * (k + 1) + 2, k=k)
    sysm.step(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sysm.step(outer)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / outer
    out = sysm.finish("kskipmrr")
    sysm.close()
    return out.info["residual"], dt


def main():
    import numpy as np
    side = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    parts = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    outer = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    r1, t1 = run(side, 1, outer)
    rp, tp = run(side, parts, outer)
    m = min(len(r1), len(rp))
    print("1 shard :", " ".join(f"{v:.15e}" for v in r1), flush=True)
    print(f"{parts} shards:", " ".join(f"{v:.15e}" for v in rp), flush=True)
    nz = np.abs(r1[:m]) > 0
    rel = float(np.max(np.abs(r1[:m] - rp[:m])[nz] / np.abs(r1[:m])[nz]))
    print(f"{side}^3 k-skip MrR k=4: 1 shard {t1 * 1e3:.2f} ms/outer, {parts} shards on one "
          f"GPU {tp * 1e3:.2f} ms/outer, histories {len(r1)}/{len(rp)} entries, "
          f"max rel diff {rel:.2e}", flush=True)
    sys.exit(0 if len(r1) == len(rp) and rel < 1e-10 else 1)


if __name__ == "__main__":
    main()
