"""CPU restatement of the reference's preconditioned / pipelined CG variants
(TEST INFRASTRUCTURE ONLY: tests/ may import it; the product path never does).

Reference: 5enxia/parallel-krylov ``v1/threads/pipeline/{pcg,chronopoulos_gear,
gropp,pipeline}.py`` -- ``method(A, b, ilu, epsilon, T=np.float64, pt='cpu')``
returning ``(elapsed_time, num_of_solution_updates, residual)``, with
``ilu.solve(v)`` applying the preconditioner M^-1 and the loop bookkeeping of
``v1/threads/common.py:41-52`` (max_iter = 2N, ``for i in range(1, max_iter)``,
``residual[i]`` after the i-th update).

PARITY UNPINNED against those files: they cannot run (``from .common import``
names a module absent from ``v1/threads/pipeline/``; a stand-in would be a
rebuilt reference) and, read as written, each misstates the algorithm it is
named after (a numpy run of their statements on 16^2 Poisson
stagnates or stops early). This module states the textbook algorithms the files
name, in the files' statement order wherever that order is right:

* pcg: ``beta = (r_new, u_new) / (r_old, u_old)``; the file divides by
  ``dot(old_r, old_u)`` with ``old_r`` copied AFTER r was updated
  (pcg.py:39-42), i.e. by (r_new, u_old).
* chronopoulos_gear: ``old_gamma`` is advanced every iteration; the file sets
  it once before the loop (chronopoulos_gear.py:32,50).
* gropp: ``beta = gamma_new / gamma_old``; the file assigns ``old_gamma =
  gamma`` right after computing gamma (gropp.py:42-43,45), so beta == 1.
* pipeline (Ghysels-Vanroose): ``m = M^-1 w`` (the file preconditions r,
  pipeline.py:39) and ``gamma_old`` taken before gamma is recomputed (the file
  assigns it right after, pipeline.py:35-36).
* ``num_of_solution_updates[j] = j`` for every recorded entry (the files leave
  the converged entry, and gropp/pipeline every entry, at 0).

What pins it: with ``ilu=None`` (M = I) ``pcg`` is statement for statement
v3/cpu/cg.py (dot(p, s) == dot(s, p) elementwise; u = r), so it reproduces the
reference-generated CG fixtures bit for bit (tests/test_pipecg.py); the four
variants are the same Krylov iteration in exact arithmetic, so their
histories agree with each other and with scipy's CG to rounding.
"""
from __future__ import annotations

import time

import numpy as np

_dot = np.dot
_norm = np.linalg.norm


class Jacobi:
    """Diagonal preconditioner with the ``solve`` interface the reference's
    ``ilu`` argument has (scipy SuperLU): M^-1 v = v / d."""

    def __init__(self, A=None, d=None):
        self.d = np.asarray(A.diagonal() if d is None else d, dtype=np.float64)

    def solve(self, v):
        return v / self.d


class IluSweeps:
    """``solve`` of a scipy SuperLU (``spilu`` / ``splu``: A ~ Pr^T L U Pc^T,
    ilu.solve(v) = Pc U^-1 L^-1 Pr v) restated as the device's two
    level-scheduled triangular sweeps (kr_kernels.hip ilu_sweep_kernel): row i
    of a sweep is s = rhs; s = s - T[i][j] * x[j] over its strictly-triangular
    entries in ascending column order (each product rounded, then the
    difference); x[i] = s / T[i][i]. Level order does not change any row's
    arithmetic, so this restates the device bit for bit; SuperLU's own solve
    (supernodal, column-oriented) agrees to rounding
    (tests/test_pipecg.py::test_ilu_sweeps_match_superlu)."""

    def __init__(self, ilu):
        import scipy.sparse as sp
        self.L = sp.csr_matrix(ilu.L)
        self.U = sp.csr_matrix(ilu.U)
        for T in (self.L, self.U):
            T.sum_duplicates()
            T.sort_indices()
        self.pr = np.asarray(ilu.perm_r)
        self.pc = np.asarray(ilu.perm_c)
        self.n = self.L.shape[0]

    def _sweep(self, T, rhs, lower):
        n = self.n
        x = np.zeros(n)
        order = range(n) if lower else range(n - 1, -1, -1)
        ip, ix, dv = T.indptr, T.indices, T.data
        for i in order:
            s = rhs[i]
            d = None
            for jj in range(ip[i], ip[i + 1]):
                j = ix[jj]
                if j == i:
                    d = dv[jj]
                elif (j < i) == lower:
                    s = s - dv[jj] * x[j]
            x[i] = s / d
        return x

    def solve(self, v):
        w = np.empty(self.n)
        w[self.pr] = v                      # Pr v
        y = self._sweep(self.L, w, True)    # L^-1
        z = self._sweep(self.U, y, False)   # U^-1
        return z[self.pc]                   # Pc z


class _Identity:
    def solve(self, v):
        return v.copy()


def _init(A, b, maxiter, x0):
    """v1/threads/common.py:41-52 (max_iter = 2N)."""
    b = np.asarray(b, dtype=np.float64)
    N = b.size
    x = np.zeros(N, np.float64) if x0 is None else np.array(x0, dtype=np.float64)
    max_iter = 2 * N if maxiter is None else int(maxiter)
    residual = np.zeros(max(max_iter, 1) + 1, np.float64)
    nosl = np.zeros(max(max_iter, 1) + 1, np.int64)
    return x, _norm(b), N, max_iter, residual, nosl


def _out(t0, nosl, residual, i, x, converged, return_x):
    elapsed = time.perf_counter() - t0
    out = (elapsed, nosl[:i + 1], residual[:i + 1])
    return out + (x, converged) if return_x else out


def pcg(A, b, ilu, epsilon, T=np.float64, pt="cpu", maxiter=None, x0=None, return_x=False):
    """Preconditioned CG, v1/threads/pipeline/pcg.py:4-48 (beta fixed)."""
    ilu = _Identity() if ilu is None else ilu
    x, b_norm, N, max_iter, residual, nosl = _init(A, b, maxiter, x0)
    t0 = time.perf_counter()
    r = b - A.dot(x)                      # :21
    residual[0] = _norm(r) / b_norm       # :22
    u = ilu.solve(r)                      # :26
    p = u.copy()                          # :27
    gamma = _dot(r, u)
    i, conv = 0, False
    for i in range(1, max_iter):          # :29
        s = A.dot(p)                      # :30
        alpha = gamma / _dot(p, s)        # :32
        x += alpha * p                    # :33
        r -= alpha * s                    # :34
        residual[i] = _norm(r) / b_norm   # :35
        nosl[i] = i
        if residual[i] < epsilon:         # :36
            conv = True
            break
        u = ilu.solve(r)                  # :41
        gnew = _dot(r, u)
        beta = gnew / gamma               # :42 (fixed: (r_new,u_new)/(r_old,u_old))
        gamma = gnew
        p = u + beta * p                  # :43
    return _out(t0, nosl, residual, i, x, conv, return_x)


def chronopoulos_gear(A, b, ilu, epsilon, T=np.float64, pt="cpu", maxiter=None, x0=None,
                      return_x=False):
    """Chronopoulos-Gear CG (one reduction point per iteration),
    v1/threads/pipeline/chronopoulos_gear.py:7-56 (old_gamma advanced)."""
    ilu = _Identity() if ilu is None else ilu
    x, b_norm, N, max_iter, residual, nosl = _init(A, b, maxiter, x0)
    t0 = time.perf_counter()
    r = b - A.dot(x)                      # :23
    residual[0] = _norm(r) / b_norm       # :24
    u = ilu.solve(r)                      # :26
    w = A.dot(u)                          # :27
    alpha = _dot(r, u) / _dot(w, u)       # :29
    beta = 0.0                            # :30
    gamma = _dot(r, u)                    # :31
    p = np.zeros(N, np.float64)           # :34
    s = np.zeros(N, np.float64)           # :35
    i, conv = 0, False
    for i in range(1, max_iter):          # :37
        p = u + beta * p                  # :38
        s = w + beta * s                  # :39
        x += alpha * p                    # :40
        r -= alpha * s                    # :41
        residual[i] = _norm(r) / b_norm   # :42
        nosl[i] = i
        if residual[i] < epsilon:
            conv = True
            break
        u = ilu.solve(r)                  # :46
        w = A.dot(u)                      # :47
        gnew = _dot(r, u)                 # :48
        delta = _dot(w, u)                # :49
        beta = gnew / gamma               # :50 (fixed: gamma of the previous iteration)
        alpha = gnew / (delta - beta * gnew / alpha)  # :51
        gamma = gnew
    return _out(t0, nosl, residual, i, x, conv, return_x)


def gropp(A, b, ilu, epsilon, T=np.float64, pt="cpu", maxiter=None, x0=None, return_x=False):
    """Gropp's asynchronous CG, v1/threads/pipeline/gropp.py:7-50 (beta fixed)."""
    ilu = _Identity() if ilu is None else ilu
    x, b_norm, N, max_iter, residual, nosl = _init(A, b, maxiter, x0)
    t0 = time.perf_counter()
    r = b - A.dot(x)                      # :23
    residual[0] = _norm(r) / b_norm       # :24
    u = ilu.solve(r)                      # :25
    p = u.copy()                          # :26
    s = A.dot(p)                          # :27
    gamma = _dot(r, u)                    # :28
    i, conv = 0, False
    for i in range(1, max_iter):          # :31
        delta = _dot(p, s)                # :32
        q = ilu.solve(s)                  # :33
        alpha = gamma / delta             # :34
        x += alpha * p                    # :35
        r -= alpha * s                    # :36
        residual[i] = _norm(r) / b_norm   # :37
        nosl[i] = i
        if residual[i] < epsilon:
            conv = True
            break
        u -= alpha * q                    # :41
        gnew = _dot(r, u)                 # :42
        w = A.dot(u)                      # :44
        beta = gnew / gamma               # :45 (fixed: gamma of the previous iteration)
        gamma = gnew
        p = u + beta * p                  # :46
        s = w + beta * s                  # :47
    return _out(t0, nosl, residual, i, x, conv, return_x)


def pipeline(A, b, ilu, epsilon, T=np.float64, pt="cpu", maxiter=None, x0=None,
             return_x=False):
    """Pipelined CG (Ghysels-Vanroose), v1/threads/pipeline/pipeline.py:7-62
    (m = M^-1 w, gamma_old taken before gamma is recomputed)."""
    ilu = _Identity() if ilu is None else ilu
    x, b_norm, N, max_iter, residual, nosl = _init(A, b, maxiter, x0)
    t0 = time.perf_counter()
    r = b - A.dot(x)                      # :23
    residual[0] = _norm(r) / b_norm       # :24
    u = ilu.solve(r)                      # :26
    w = A.dot(u)                          # :27
    z = np.zeros(N)                       # :29-32
    q = np.zeros(N)
    s = np.zeros(N)
    p = np.zeros(N)
    alpha = gamma_old = 0.0
    i, conv = 0, False
    for i in range(1, max_iter):          # :34
        gamma = _dot(r, u)                # :35
        delta = _dot(w, u)                # :37
        m = ilu.solve(w)                  # :39 (fixed: M^-1 w)
        n = A.dot(m)                      # :41
        if i > 1:                         # :42-47
            beta = gamma / gamma_old
            alpha = gamma / (delta - beta * gamma / alpha)
        else:
            beta = 0.0
            alpha = gamma / delta
        gamma_old = gamma                 # (fixed: before the next recomputation)
        z = n + beta * z                  # :48
        q = m + beta * q                  # :49
        s = w + beta * s                  # :50
        p = u + beta * p                  # :51
        x += alpha * p                    # :52
        r -= alpha * s                    # :53
        residual[i] = _norm(r) / b_norm   # :54
        nosl[i] = i
        if residual[i] < epsilon:
            conv = True
            break
        u -= alpha * q                    # :58
        w -= alpha * z                    # :59
    return _out(t0, nosl, residual, i, x, conv, return_x)


METHODS = {"pcg": pcg, "chronopoulos_gear": chronopoulos_gear, "gropp": gropp,
           "pipeline": pipeline}
