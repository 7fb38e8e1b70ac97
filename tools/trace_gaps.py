"""Timeline view of a rocprofv3 kernel trace (tools/profile.sh <tag>): for the
last `--window` kernels of the run, the GPU busy fraction, the idle gaps
between consecutive kernels and the largest ones with their neighbours.
Shows how much of a bench step is kernel time and how much is host/launch
idle (e.g. the once-per-outer-iteration Gram sync)."""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--window", type=int, default=150)
    p.add_argument("--top", type=int, default=12)
    a = p.parse_args()
    rows = list(csv.DictReader(open(os.path.join(a.dir, "trace", "run_kernel_trace.csv"))))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                 for r in rows), key=lambda t: t[0])
    ks = ks[-a.window:]
    span = ks[-1][1] - ks[0][0]
    busy = sum(e - s for s, e, _ in ks)
    gaps = [(ks[i + 1][0] - ks[i][1], ks[i][2], ks[i + 1][2]) for i in range(len(ks) - 1)]
    print(f"{len(ks)} kernels, span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms "
          f"({busy / span:.1%}), idle {(span - busy) / 1e6:.3f} ms")
    pos = sorted(g for g in gaps if g[0] > 0)
    if pos:
        print(f"gaps > 0: {len(pos)}, median {pos[len(pos) // 2][0] / 1e3:.1f} us")
    for g, before, after in sorted(gaps, reverse=True)[:a.top]:
        print(f"  {g / 1e3:9.1f} us  {before} -> {after}")


if __name__ == "__main__":
    main()
