"""Dense-A GEMV microbenchmark (GPU box only): y = A x for a dense n x n
float64 block through the system path (gemv_kernel), HIP-event timed, in
algorithmic GB/s (8 n^2 + 16 n bytes).  python tools/dense_micro.py --n 20000"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[4096, 20000, 40000])
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from parallel_krylov_amd.system import KrylovSystem
    dev = torch.device("cuda", 0)
    for n in args.n:
        A = torch.rand((n, n), dtype=torch.float64, device=dev)
        sysm = KrylovSystem(n, [0, n], [0])
        sysm.adopt_dense(0, A)
        sysm.finalize()
        x = [torch.rand(n, dtype=torch.float64, device=dev)]
        y = sysm.spmv(x)
        torch.cuda.synchronize()
        err = (y[0] - A @ x[0]).abs().max().item() / (A @ x[0]).abs().max().item()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.reps):
            sysm.spmv(x)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / args.reps
        gb = (8.0 * n * n + 16.0 * n) / 1e9
        print(f"n={n}: {ms:.3f} ms/gemv (incl. spmv() call overhead) {gb / ms * 1e3:.0f} GB/s "
              f"rel err vs torch {err:.1e}", flush=True)
        sysm.close()
        del A


if __name__ == "__main__":
    main()
