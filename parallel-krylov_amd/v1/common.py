"""Console report of the v1 generation, byte-for-byte the reference's
(v1/common.py:18-54: green rules, lower-case keys, ``initial_k`` always
printed)."""
from __future__ import annotations

_GREEN, _END = "\033[32m", "\033[0m"


def _start(method_name: str = "", k: int = None) -> None:
    print("\n".join([f"{_GREEN}# {'=' * 16} INFO {'=' * 16} #{_END}",
                     f"Method:\t\t{method_name}", f"initial_k:\t{k}"]))


def _end(elapsed_time: float, isConverged: bool, num_of_iter: int, final_residual: float,
         final_k: int = None) -> None:
    lines = [f"time:\t\t{elapsed_time} s",
             "status:\t\t" + ("converged" if isConverged else "diverged"),
             f"iteration:\t{num_of_iter} times",
             f"final residual:\t{final_residual}"]
    if final_k:
        lines.append(f"final k:\t{final_k}")
    lines.append(f"{_GREEN}# {'=' * 38} #{_END}")
    print("\n".join(lines))
