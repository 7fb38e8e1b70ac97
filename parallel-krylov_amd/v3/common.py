"""Console report of a solve, byte-for-byte the reference's (v3/common.py:2-23).

The INFO block is part of the drop-in behaviour: scripts that scrape
``Iteration:`` / ``Final_Residual:`` keep working.
"""
from __future__ import annotations

_RULE = "=" * 16


def _start(method_name: str = "", k: int = None) -> None:
    lines = [f"# {_RULE} INFO {_RULE} #", f"Method:\t\t{method_name}"]
    if k is not None:
        lines.append(f"Initial_k:\t{k}")
    print("\n".join(lines))


def _finish(elapsed_time: float, isConverged: bool, num_of_iter: int,
            final_residual: float, final_k: int = None) -> None:
    lines = [
        f"Time:\t\t{elapsed_time} s",
        "Status:\t\t" + ("converged" if isConverged else "diverged"),
        f"Iteration:\t{num_of_iter} times",
        f"Final_Residual:\t{final_residual}",
    ]
    if final_k:
        lines.append(f"Final_k:\t{final_k}")
    lines.append("# " + "=" * 38 + " #")
    print("\n".join(lines))
