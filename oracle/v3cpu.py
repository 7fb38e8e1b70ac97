"""CPU restatement of the reference's v3/cpu solvers (TEST INFRASTRUCTURE ONLY).

This is the parity oracle. Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it; the product path
(``parallel-krylov_amd``) never does, and fails loudly when its HIP library is
missing instead of falling back to anything here.

It restates, statement for statement and with the same numpy/scipy calls, the
algorithms of 5enxia/parallel-krylov ``v3/cpu`` (cited per function). On the
same machine it is bitwise identical to the reference: tests/test_oracle.py
checks it against golden vectors produced by running the reference itself
(tests/golden/make_golden.py). The v3/gpu family is line-for-line the same
algorithm with cupy in place of numpy, so this is also the
oracle of the GPU path.

Differences from the reference that do not change any computed value:
* no banner printing (pass ``verbose=True`` to get the v3/common.py banner);
* the caller's ``x`` is copied, not mutated in place (v3/cpu mutates it);
* ``numpy.int`` (removed in numpy >= 1.24) is spelled ``numpy.int64``;
* sparse ``A`` is multiplied with ``A.dot`` everywhere (v3/cpu/kskipcg.py and
  adaptivekskipmrr.py call ``numpy.dot(A, x)``, which raises on scipy sparse
  matrices; ``A @ x`` and ``A.dot(x)`` run the same csr_matvec);
* adaptive k-skip MrR starts with ``pre_x = x0`` so a residual increase at
  the first check does not raise NameError (v3/cpu/adaptivekskipmrr.py:47).
"""
from __future__ import annotations

import time

import numpy as np

_dot = np.dot
_norm = np.linalg.norm


def _matvec(A, v):
    return A.dot(v)


class _History:
    """residual / nosl / khistory bookkeeping of v3/cpu/common.py:22-36."""

    def __init__(self, b, x, maxiter, k=None):
        self.b_norm = _norm(b)
        self.N = b.size
        self.x = np.array(x, dtype=np.float64) if isinstance(x, np.ndarray) \
            else np.zeros(self.N, dtype=np.float64)
        self.maxiter = self.N if maxiter is None else maxiter
        self.residual = np.zeros(self.maxiter + 1, np.float64)
        self.nosl = np.zeros(self.maxiter + 1, np.int64)
        self.khistory = None if k is None else np.zeros(self.N + 1, np.int64)

    def info(self, elapsed, last, with_k=False):
        out = {'time': elapsed, 'nosl': self.nosl[:last + 1],
               'residual': self.residual[:last + 1]}
        if with_k:
            out['khistory'] = self.khistory[:last + 1]
        return out


def _banner(verbose, name, k=None):
    if verbose:
        print('# ', '=' * 16, ' INFO ', '=' * 16, ' #', sep='')
        print(f'Method:\t\t{name}')
        if k is not None:
            print(f'Initial_k:\t{k}')


def _banner_end(verbose, elapsed, converged, iters, final, final_k=None):
    if verbose:
        print(f'Time:\t\t{elapsed} s')
        print(f"Status:\t\t{'converged' if converged else 'diverged'}")
        print(f'Iteration:\t{iters} times')
        print(f'Final_Residual:\t{final}')
        if final_k:
            print(f'Final_k:\t{final_k}')
        print('# ', '=' * 38, ' #', sep='')


# ---------------------------------------------------------------------- CG
def cg(A, b, x=None, tol=1e-05, maxiter=None, M=None, callback=None, atol=None,
       verbose=False):
    """Conjugate gradient, v3/cpu/cg.py:7-48."""
    h = _History(b, x, maxiter)
    x = h.x
    r = b - _matvec(A, x)
    p = r.copy()
    gamma = _dot(r, r)
    i = 0
    _banner(verbose, 'CG')
    t0 = time.perf_counter()
    converged = False
    while i < h.maxiter:
        h.residual[i] = _norm(r) / h.b_norm
        if h.residual[i] < tol:
            converged = True
            break
        v = _matvec(A, p)
        sigma = _dot(p, v)
        alpha = gamma / sigma
        x += alpha * p
        r -= alpha * v
        previous = gamma.copy()
        gamma = _dot(r, r)
        beta = gamma / previous
        p = r + beta * p
        i += 1
        h.nosl[i] = i
    else:
        h.residual[i] = _norm(r) / h.b_norm
    elapsed = time.perf_counter() - t0
    _banner_end(verbose, elapsed, converged, i, h.residual[i])
    return x, h.info(elapsed, i)


# --------------------------------------------------------------------- MrR
def mrr(A, b, x=None, tol=1e-05, maxiter=None, M=None, callback=None, atol=None,
        verbose=False):
    """Minimal residual (MrR), v3/cpu/mrr.py:7-61."""
    h = _History(b, x, maxiter)
    x = h.x
    r = b - _matvec(A, x)
    h.residual[0] = _norm(r) / h.b_norm
    i = 0
    _banner(verbose, 'MrR')
    t0 = time.perf_counter()
    # first iteration: a plain minimal-residual step
    Ar = _matvec(A, r)
    zeta = _dot(r, Ar) / _dot(Ar, Ar)
    y = zeta * Ar
    z = -zeta * r
    r -= y
    x -= z
    h.nosl[1] = 1
    i += 1
    converged = False
    while i < h.maxiter:
        h.residual[i] = _norm(r) / h.b_norm
        if h.residual[i] < tol:
            converged = True
            break
        Ar = _matvec(A, r)
        mu = _dot(y, y)
        nu = _dot(y, Ar)
        gamma = nu / mu
        s = Ar - gamma * y
        rs = _dot(r, s)
        ss = _dot(s, s)
        zeta = rs / ss
        eta = -zeta * gamma
        y = eta * y + zeta * Ar
        z = eta * z - zeta * r
        r -= y
        x -= z
        i += 1
        h.nosl[i] = i
    else:
        h.residual[i] = _norm(r) / h.b_norm
    elapsed = time.perf_counter() - t0
    _banner_end(verbose, elapsed, converged, i, h.residual[i])
    return x, h.info(elapsed, i)


# ------------------------------------------------------ k-skip recurrences
def kskipmrr_coefficients(alpha, beta, delta):
    """(zeta, eta) of one MrR step from the Gram arrays, v3/cpu/kskipmrr.py:62-64."""
    d = alpha[2] * delta[0] - beta[1] ** 2
    zeta = alpha[1] * delta[0] / d
    eta = -alpha[1] * beta[1] / d
    return zeta, eta


def kskipmrr_advance(k, j, alpha, beta, delta, zeta, eta):
    """Gram update between inner steps j and j+1, v3/cpu/kskipmrr.py:73-84."""
    delta[0] = zeta ** 2 * alpha[2] + eta * zeta * beta[1]
    alpha[0] -= zeta * alpha[1]
    delta[1] = eta ** 2 * delta[1] + 2 * eta * zeta * beta[2] + zeta ** 2 * alpha[3]
    beta[1] = eta * beta[1] + zeta * alpha[2] - delta[1]
    alpha[1] = -beta[1]
    for l in range(2, 2 * (k - j) + 1):
        delta[l] = eta ** 2 * delta[l] + 2 * eta * zeta * beta[l + 1] + zeta ** 2 * alpha[l + 2]
        tau = eta * beta[l] + zeta * alpha[l + 1]
        beta[l] = tau - delta[l]
        alpha[l] -= tau + beta[l]


def kskipmrr_scalars(k, alpha, beta, delta):
    """All k+1 (zeta, eta) pairs of one outer iteration (arrays are consumed)."""
    out = [kskipmrr_coefficients(alpha, beta, delta)]
    for j in range(k):
        kskipmrr_advance(k, j, alpha, beta, delta, *out[-1])
        out.append(kskipmrr_coefficients(alpha, beta, delta))
    return out


def kskipcg_coefficients(a, f):
    """(alpha, beta) of one CG step from the Gram arrays, v3/cpu/kskipcg.py:51-52."""
    alpha = a[0] / f[1]
    beta = alpha ** 2 * f[2] / a[0] - 1
    return alpha, beta


def kskipcg_advance(k, j, a, f, c, alpha, beta):
    """Gram update between inner steps, v3/cpu/kskipcg.py:60-64."""
    for l in range(0, 2 * (k - j) + 1):
        a[l] += alpha * (alpha * f[l + 2] - 2 * c[l + 1])
        d = c[l] - alpha * f[l + 1]
        c[l] = a[l] + d * beta
        f[l] = c[l] + beta * (d + beta * f[l])


def kskipcg_scalars(k, a, f, c):
    out = [kskipcg_coefficients(a, f)]
    for j in range(k):
        kskipcg_advance(k, j, a, f, c, *out[-1])
        out.append(kskipcg_coefficients(a, f))
    return out


def _gram_pairs(basis_u, basis_v, count, start=0):
    """g[j] = <U[j//2], V[j//2 + j%2]> for j in [start, count)."""
    g = {}
    for j in range(start, count):
        jj = j // 2
        g[j] = _dot(basis_u[jj], basis_v[jj + j % 2])
    return g


# -------------------------------------------------------------- k-skip CG
def kskipcg(A, b, x=None, tol=1e-05, maxiter=None, k=0, M=None, callback=None,
            atol=None, verbose=False):
    """k-skip CG, v3/cpu/kskipcg.py:8-87."""
    h = _History(b, x, maxiter)
    x = h.x
    N = h.N
    Ar = np.zeros((k + 2, N), np.float64)
    Ap = np.zeros((k + 3, N), np.float64)
    a = np.zeros(2 * k + 2, np.float64)
    f = np.zeros(2 * k + 4, np.float64)
    c = np.zeros(2 * k + 2, np.float64)
    Ar[0] = b - _matvec(A, x)
    Ap[0] = Ar[0]
    i = 0
    index = 0
    _banner(verbose, 'k-skip CG', k)
    t0 = time.perf_counter()
    converged = False
    while i < h.maxiter:
        h.residual[index] = _norm(Ar[0]) / h.b_norm
        if h.residual[index] < tol:
            converged = True
            break
        for j in range(1, k + 1):
            Ar[j] = _matvec(A, Ar[j - 1])
        for j in range(1, k + 2):
            Ap[j] = _matvec(A, Ap[j - 1])
        for j, v in _gram_pairs(Ar, Ar, 2 * k + 1).items():
            a[j] = v
        for j, v in _gram_pairs(Ap, Ap, 2 * k + 4).items():
            f[j] = v
        for j, v in _gram_pairs(Ar, Ap, 2 * k + 2).items():
            c[j] = v
        alpha, beta = kskipcg_coefficients(a, f)
        for j in range(k + 1):
            if j > 0:
                kskipcg_advance(k, j - 1, a, f, c, alpha, beta)
                alpha, beta = kskipcg_coefficients(a, f)
            x += alpha * Ap[0]
            Ar[0] -= alpha * Ap[1]
            Ap[0] = Ar[0] + beta * Ap[0]
            Ap[1] = _matvec(A, Ap[0])
        i += (k + 1)
        index += 1
        h.nosl[index] = i
    else:
        h.residual[index] = _norm(Ar[0]) / h.b_norm
    elapsed = time.perf_counter() - t0
    _banner_end(verbose, elapsed, converged, i, h.residual[index])
    return x, h.info(elapsed, index)


# ------------------------------------------------------------- k-skip MrR
def _kskipmrr_gram(k, Ar, Ay, alpha, beta, delta):
    """Gram coefficients, v3/cpu/kskipmrr.py:50-59."""
    for j, v in _gram_pairs(Ar, Ar, 2 * k + 3).items():
        alpha[j] = v
    for j, v in _gram_pairs(Ay, Ar, 2 * k + 2, start=1).items():
        beta[j] = v
    for j, v in _gram_pairs(Ay, Ay, 2 * k + 1).items():
        delta[j] = v


def _kskipmrr_inner(A, k, Ar, Ay, alpha, beta, delta, z, x):
    """The k+1 vector steps of one outer iteration, v3/cpu/kskipmrr.py:61-93."""
    zeta, eta = kskipmrr_coefficients(alpha, beta, delta)
    for j in range(k + 1):
        if j > 0:
            kskipmrr_advance(k, j - 1, alpha, beta, delta, zeta, eta)
            zeta, eta = kskipmrr_coefficients(alpha, beta, delta)
        Ay[0] = eta * Ay[0] + zeta * Ar[1]
        z = eta * z - zeta * Ar[0]
        Ar[0] -= Ay[0]
        Ar[1] = _matvec(A, Ar[0])
        x -= z
    return z


def _mrr_start(A, Ar, Ay, x):
    """Plain MrR first step, v3/cpu/kskipmrr.py:26-31."""
    Ar[1] = _matvec(A, Ar[0])
    zeta = _dot(Ar[0], Ar[1]) / _dot(Ar[1], Ar[1])
    Ay[0] = zeta * Ar[1]
    z = -zeta * Ar[0]
    Ar[0] -= Ay[0]
    x -= z
    return z


def kskipmrr(A, b, x=None, tol=1e-05, maxiter=None, k=0, M=None, callback=None,
             atol=None, verbose=False):
    """k-skip MrR, v3/cpu/kskipmrr.py:8-108."""
    h = _History(b, x, maxiter)
    x = h.x
    N = h.N
    Ar = np.zeros((k + 2, N), np.float64)
    Ay = np.zeros((k + 1, N), np.float64)
    alpha = np.zeros(2 * k + 3, np.float64)
    beta = np.zeros(2 * k + 2, np.float64)
    delta = np.zeros(2 * k + 1, np.float64)
    Ar[0] = b - _matvec(A, x)
    h.residual[0] = _norm(Ar[0]) / h.b_norm
    _banner(verbose, 'k-skip MrR', k)
    t0 = time.perf_counter()
    z = _mrr_start(A, Ar, Ay, x)
    h.nosl[1] = 1
    i = 1
    index = 1
    converged = False
    while i < h.maxiter:
        h.residual[index] = _norm(Ar[0]) / h.b_norm
        if h.residual[index] < tol:
            converged = True
            break
        for j in range(1, k + 2):
            Ar[j] = _matvec(A, Ar[j - 1])
        for j in range(1, k + 1):
            Ay[j] = _matvec(A, Ay[j - 1])
        _kskipmrr_gram(k, Ar, Ay, alpha, beta, delta)
        z = _kskipmrr_inner(A, k, Ar, Ay, alpha, beta, delta, z, x)
        i += (k + 1)
        index += 1
        h.nosl[index] = i
    else:
        h.residual[index] = _norm(Ar[0]) / h.b_norm
    elapsed = time.perf_counter() - t0
    _banner_end(verbose, elapsed, converged, i, h.residual[index])
    return x, h.info(elapsed, index)


def adaptivekskipmrr(A, b, x=None, tol=1e-05, maxiter=None, k=0, M=None, callback=None,
                     atol=None, verbose=False):
    """Adaptive k-skip MrR, v3/cpu/adaptivekskipmrr.py:8-141."""
    h = _History(b, x, maxiter, k=k)
    x = h.x
    N = h.N
    Ar = np.zeros((k + 3, N), np.float64)
    Ay = np.zeros((k + 2, N), np.float64)
    alpha = np.zeros(2 * k + 3, np.float64)
    beta = np.zeros(2 * k + 2, np.float64)
    delta = np.zeros(2 * k + 1, np.float64)
    h.khistory[0] = k
    Ar[0] = b - _matvec(A, x)
    h.residual[0] = _norm(Ar[0]) / h.b_norm
    pre_residual = h.residual[0]
    pre_x = x.copy()
    _banner(verbose, 'Adaptive k-skip MrR', k)
    t0 = time.perf_counter()
    z = _mrr_start(A, Ar, Ay, x)
    h.nosl[1] = 1
    h.khistory[1] = k
    i = 1
    index = 1
    converged = False
    while i < h.maxiter:
        h.residual[index] = _norm(Ar[0]) / h.b_norm
        if h.residual[index] > pre_residual:
            # residual went up: restart from the snapshot with k - 1
            x = pre_x.copy()
            Ar[0] = b - _matvec(A, x)
            z = _mrr_start(A, Ar, Ay, x)
            i += 1
            index += 1
            h.residual[index] = _norm(Ar[0]) / h.b_norm
            h.nosl[index] = i
            if k > 1:
                k -= 1
            h.khistory[index] = k
        else:
            pre_residual = h.residual[index]
            pre_x = x.copy()
        if h.residual[index] < tol:
            converged = True
            break
        for j in range(1, k + 2):
            Ar[j] = _matvec(A, Ar[j - 1])
        for j in range(1, k + 1):
            Ay[j] = _matvec(A, Ay[j - 1])
        _kskipmrr_gram(k, Ar, Ay, alpha, beta, delta)
        z = _kskipmrr_inner(A, k, Ar, Ay, alpha, beta, delta, z, x)
        i += (k + 1)
        index += 1
        h.nosl[index] = i
        h.khistory[index] = k
    else:
        h.residual[index] = _norm(Ar[0]) / h.b_norm
    elapsed = time.perf_counter() - t0
    _banner_end(verbose, elapsed, converged, i, h.residual[index], k)
    return x, h.info(elapsed, index, with_k=True)


METHODS = {
    'cg': cg,
    'mrr': mrr,
    'kskipcg': kskipcg,
    'kskipmrr': kskipmrr,
    'adaptivekskipmrr': adaptivekskipmrr,
}
