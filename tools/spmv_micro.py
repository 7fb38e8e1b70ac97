"""SpMV microbenchmark on the device-generated Poisson matrix (GPU box only).

Times the single- and two-vector SpMV primitives under each kernel variant
(KR_SPMV_VARIANT) with HIP events, plus streaming references (dot = pure
read, torch copy = read+write), and prints algorithmic GB/s.

  python tools/spmv_micro.py --n-side 512 --variants 0 1 2 11 12 13
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-side", type=int, default=512)
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--banded", type=int, nargs=3, metavar=("N", "H", "W"), default=None,
                    help="use the banded generator instead of Poisson")
    args = ap.parse_args()
    import torch
    from parallel_krylov_amd._lib import library
    from parallel_krylov_amd.system import KrylovSystem

    lib = library()
    if args.banded:
        n = args.banded[0]
        sysm = KrylovSystem(n, [0, n], [0])
        sysm.gen_banded(args.banded[1], args.banded[2], 0)
    else:
        n = args.n_side ** 3
        sysm = KrylovSystem(n, [0, n], [0])
        sysm.gen_poisson(args.n_side, 3)
    sysm.finalize()
    nnz = sysm.shard_info(0)["nnz"]
    c = sysm.csr_pointers(0)
    dev = torch.device("cuda", 0)
    x = sysm.rhs(1)[0]
    x2 = sysm.rhs(2)[0]
    y = torch.empty_like(x)
    y2 = torch.empty_like(x)
    rp_b = 8 if c["rowptr64"] else 4
    b1 = 12.0 * nnz + rp_b * (n + 1) + 16.0 * n
    b2 = 12.0 * nnz + rp_b * (n + 1) + 32.0 * n

    def timeit(fn, reps):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps

    single = lambda: lib.kr_spmv_csr_f64(c["rowptr"], c["rowptr64"], c["col"], c["val"], n,
                                         x.data_ptr(), y.data_ptr(), None)
    dual = lambda: lib.kr_spmv2_csr_f64(c["rowptr"], c["rowptr64"], c["col"], c["val"], n,
                                        x.data_ptr(), x2.data_ptr(), y.data_ptr(),
                                        y2.data_ptr(), None)
    dual_alias = lambda: lib.kr_spmv2_csr_f64(c["rowptr"], c["rowptr64"], c["col"], c["val"],
                                              n, x.data_ptr(), x.data_ptr(), y.data_ptr(),
                                              y2.data_ptr(), None)
    print(f"N={n} nnz={nnz} single={b1/1e9:.2f} GB dual={b2/1e9:.2f} GB per launch")
    for v in args.variants:
        os.environ["KR_SPMV_VARIANT"] = str(v)
        t1 = timeit(single, args.reps)
        t2 = timeit(dual, args.reps)
        t3 = timeit(dual_alias, args.reps)
        print(f"variant {v:3d}: single {t1:7.3f} ms {b1/t1/1e6:7.1f} GB/s | "
              f"dual {t2:7.3f} ms {b2/t2/1e6:7.1f} GB/s | dual x2=x1 {t3:7.3f} ms", flush=True)
    os.environ["KR_SPMV_VARIANT"] = "0"
    out = torch.empty(1, dtype=torch.float64, device=dev)
    big = torch.empty(12 * nnz // 8, dtype=torch.float64, device=dev).fill_(1.0)
    td = timeit(lambda: lib.kr_dot_f64(big.data_ptr(), big.data_ptr(), big.numel(),
                                       out.data_ptr(), None), args.reps)
    print(f"dot read {big.numel()*8/1e9:.2f} GB: {td:.3f} ms {big.numel()*8/td/1e6:.1f} GB/s")
    dst = torch.empty_like(big)
    tc = timeit(lambda: dst.copy_(big), args.reps)
    print(f"torch copy {big.numel()*8/1e9:.2f} GB: {tc:.3f} ms "
          f"{2*big.numel()*8/tc/1e6:.1f} GB/s (read+write)")
    sysm.close()


if __name__ == "__main__":
    main()
