"""Infinity-Cache (MALL) reuse probe for the SpMV (GPU box only).

Runs the single SpMV over a contiguous row segment of the 512^3 Poisson matrix
back to back; if the segment's matrix bytes stay resident in the 256 MiB MALL
between launches, repeated launches run faster than a full-matrix sweep.
Prints algorithmic GB/s per segment size.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from parallel_krylov_amd._lib import library
    from parallel_krylov_amd.system import KrylovSystem

    lib = library()
    side = 512
    n = side ** 3
    sysm = KrylovSystem(n, [0, n], [0])
    sysm.gen_poisson(side, 3)
    sysm.finalize()
    c = sysm.csr_pointers(0)
    x = sysm.rhs(1)[0]
    y = torch.empty_like(x)
    rp = torch.empty(0)  # noqa: F841

    def run(r0, rows):
        lib.kr_spmv_csr_f64(c["rowptr"] + 4 * r0, 0, c["col"], c["val"], rows, x.data_ptr(),
                            y.data_ptr() + 8 * r0, None)

    for rows in [1 << 18, 1 << 19, 1 << 20, 1 << 21, 1 << 22, 1 << 23, 1 << 24, n]:
        r0 = (n - rows) // 2
        run(r0, rows)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = max(3, min(200, (1 << 26) // rows))
        s.record()
        for _ in range(reps):
            run(r0, rows)
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / reps
        byt = rows * (12 * 7 + 4 + 16)
        print(f"rows {rows:10d} matrix {rows*88/2**20:8.1f} MiB  {t*1e3:9.1f} us  "
              f"{byt/t/1e6:8.1f} GB/s (algorithmic)", flush=True)
    sysm.close()


if __name__ == "__main__":
    main()
