"""Headline benchmark: k-skip MrR (k = 4) on the 512^3 7-point Poisson CSR system.

BASELINE.json metric: "solver iterations/sec + achieved HBM GB/s, k-skip MrR
k=4 on 512^3 Poisson CSR" (configs[3]; it fits one MI355X: ~27 GB).

One "step" = one outer k-skip iteration = k+1 solver iterations over the
whole system (3k+1 SpMVs incl. k two-vector ones, the Gram reduction, k+1
fused vector updates). The matrix and b are generated on the device before the
timed region. N GPUs (torchrun, one rank per GPU) solve the SAME global system
row-partitioned (strong scaling); the halo exchange and the Gram all-gather go
over RCCL.

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for the roofline
accounting).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# the guide's measured float4 copy (MI355X_MICROARCH.md: 6.29 TB/s, 79 % of
# spec): reported beside frac as what a streaming kernel can reach in practice
HBM_COPY_GBS = 6290.0

# BASELINE.json configs. C4 is the headline (metric) and the default; the others
# are available as --config for parity/perf runs.
# BASELINE.json's metric (the headline, C4); the HBM GB/s half of it is the
# "roofline" object of the same line.
HEADLINE_METRIC = "solver iterations/sec + achieved HBM GB/s, k-skip MrR k=4 on 512\u00b3 Poisson CSR"

CONFIGS = {
    "C1": dict(method="cg", matrix=("poisson", 256, 2), k=0,
               label="CG on 2D 5-point Poisson 256^2"),
    "C2": dict(method="cg", matrix=("poisson", 256, 3), k=0,
               label="CG on 3D 7-point Poisson 256^3"),
    "C3": dict(method="mrr", matrix=("banded", 10_000_000, 13, 64, 0), k=0,
               label="MrR on random banded CSR N=10M, 27 nnz/row"),
    "C4": dict(method="kskipmrr", matrix=("poisson", 512, 3), k=4,
               label="k-skip MrR k=4 on 3D 7-point Poisson 512^3"),
    "C5": dict(method="adaptivekskipmrr", matrix=("banded", 50_000_000, 31, 256, 0), k=4,
               label="Adaptive k-skip MrR on banded CSR N=50M, 63 nnz/row"),
}


# Per-kernel event sampling per config (bench --profile-every default).
PROFILE_EVERY = {"C1": 64, "C2": 8, "C3": 8}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="C4", choices=sorted(CONFIGS))
    p.add_argument("--n-side", type=int, default=None, help="override the Poisson grid side")
    p.add_argument("--nz", type=int, default=None,
                   help="Poisson planes (a side^2 x nz box, e.g. --nz 64: one rank's slab of "
                        "512^3 at 8 GPUs, for per-rank studies on one GPU)")
    p.add_argument("--local-shards", type=int, default=1,
                   help="split this rank's rows into S in-process shards on its one GPU "
                        "(the single-process multi-GPU layout, for host-enqueue studies; "
                        "halos are device copies)")
    p.add_argument("--k", type=int, default=None)
    p.add_argument("--method", default=None)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--rhs", default="normal", choices=["normal", "hash"],
                   help="b = default_rng(1).standard_normal(N) on the host (SURVEY.md 8(d), "
                        "default) or the device counter hash 2u-1")
    p.add_argument("--no-csr", action="store_true",
                   help="skip the plain-CSR sub-record (KR_MASK=0 KR_VDICT=0 run)")
    p.add_argument("--cpu-n-side", type=int, default=512,
                   help="grid side of the CPU-baseline sample (512 = the benchmark system)")
    p.add_argument("--no-profile", action="store_true",
                   help="skip the per-kernel HIP-event timing")
    p.add_argument("--profile-every", type=int, default=None,
                   help="per-kernel HIP events on every N-th step (1 = all); default 4, "
                        "64 for C1 and 8 for C2/C3, whose steps are 16-600 us long and "
                        "would pay the ~10 us per event pair too often")
    return p.parse_args()


def cpu_model():
    """Host CPU model name (/proc/cpuinfo), or the platform string."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


# CPU-baseline sample per config (C1 runs to convergence,
# C2-C5 are capped; C5 at a stated reduced N of the same banded family, its
# rate scaled by the row ratio since SpMV and dots are linear in N).
CPU_SAMPLE = {
    "C1": dict(tol=1e-10),                 # the config itself: v3/cpu CG to 1e-10
    "C2": dict(maxiter=16),                # 16 CG iterations of 256^3
    "C3": dict(maxiter=12),                # 12 MrR iterations of N = 10M
    "C4": dict(outer=2),                   # initial step + 2 outer iterations of 512^3
    "C5": dict(outer=1, n=5_000_000),      # initial step + 1 outer iteration at N = 5M
}


def rhs_host(n: int):
    """b = default_rng(1).standard_normal(N), on the host."""
    import numpy as np
    return np.random.default_rng(1).standard_normal(n)


def cpu_baseline(config: str, mat, k: int, method: str, n_side=None, return_info=False):
    """The oracle (numpy/scipy restatement of v3/cpu, bitwise the reference) on
    the host cores, on the bounded sample CPU_SAMPLE[config] of the config's
    system (same generator, same b = default_rng(1).standard_normal(N), x0 = 0).
    Timed region = the reference's info['time']; it/s of a reduced sample
    (--cpu-n-side for Poisson, CPU_SAMPLE's n for C5) is scaled to the
    config's N by the row ratio. With return_info, also the oracle's (x-free)
    info dict: when the sample is the config's own system, its residual history
    is the full-size parity check of the GPU run (bench `parity`).

    Threads: scipy's csr_matvec is single-threaded; numpy's dots run on
    OpenBLAS with its default pool, which follows OPENBLAS_NUM_THREADS /
    OMP_NUM_THREADS (the GPU box sets 16: the CPU share of one GPU of the
    node, although the process may be scheduled on more affinity cores)."""
    from oracle import matrices, v3cpu
    try:
        from threadpoolctl import threadpool_info
        blas_threads = max([i.get("num_threads", 1) for i in threadpool_info()
                            if i.get("user_api") == "blas"] or [1])
    except Exception:  # pragma: no cover
        blas_threads = None
    samp = CPU_SAMPLE[config]
    if mat[0] == "poisson":
        side = n_side or mat[1]
        dims = mat[2]
        A = matrices.poisson(side, dims) if len(mat) == 3 else None
        if A is None:  # --nz boxes: no CPU sample
            return (None, None) if return_info else None
        n_full = mat[1] ** dims
        desc = f"{side}^{dims} Poisson"
    else:
        n_s = samp.get("n", mat[1])
        A = matrices.banded(n_s, mat[2], mat[3], mat[4])
        n_full = mat[1]
        desc = f"banded N={n_s}, {2 * mat[2] + 1} nnz/row, band {mat[3]}"
    n = A.shape[0]
    b = rhs_host(n)
    fn = v3cpu.METHODS[method]
    if "tol" in samp:
        kw = dict(tol=samp["tol"])
        what = f"to tol {samp['tol']:g}"
    elif "kskip" in method:
        kw = dict(tol=0.0, maxiter=samp["outer"] * (k + 1) + 1)
        what = f"initial step + {samp['outer']} outer"
    else:
        kw = dict(tol=0.0, maxiter=samp["maxiter"])
        what = f"{samp['maxiter']} iterations"
    if "kskip" in method:
        kw["k"] = k
    t0 = time.perf_counter()
    _, info = fn(A, b, **kw)
    wall = time.perf_counter() - t0
    del A, b
    its = int(info["nosl"][-1])
    rate = its / info["time"]
    cores = len(os.sched_getaffinity(0))
    scale = n / n_full
    scaled = "" if n == n_full else f", scaled x{scale:.4f} to N={n_full}"
    env_threads = {v: os.environ[v] for v in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS")
                   if v in os.environ}
    rec = dict(value=rate * scale, unit="iterations/s",
               cores=blas_threads if blas_threads else cores,
               kind="port",
               cpu_model=cpu_model(), affinity_cores=cores, blas_threads=blas_threads,
               thread_env=env_threads, sample_n=n, full_n=n_full,
               sample=(f"oracle.v3cpu.{method} (numpy/scipy restatement of v3/cpu, bitwise "
                       f"the reference) on {desc}, {its} iterations ({what}) in "
                       f"{info['time']:.2f} s ({rate:.3f} it/s){scaled}; "
                       f"b = default_rng(1).standard_normal(N); "
                       f"scipy SpMV 1 thread, OpenBLAS dot {blas_threads} threads "
                       f"({', '.join(f'{k_}={v}' for k_, v in env_threads.items()) or 'no thread env'}), "
                       f"{cores} affinity cores, {cpu_model()}; wall {wall:.1f} s; "
                       f"cores = the BLAS threads (the SpMV, most of the time, uses one); "
                       f"the BLAS runs on the thread count the environment sets -- the GPU "
                       f"box's CPU share is 16 cores of the node and its harness fixes "
                       f"OMP/OpenBLAS at 16, so the other affinity cores belong to other "
                       f"jobs; scipy's csr_matvec is single-threaded whatever the count"))
    full = n == n_full
    return (rec, info if full else None) if return_info else rec


# SURVEY.md 8(c) contract for CG, MrR and k-skip MrR (k <= 4): nosl
# identical, residual entries >= 1e-8 within 1e-12 relative.
PARITY_RTOL = 1e-12


def history_parity(gpu_info, ref_info, rtol=PARITY_RTOL, overlap=False):
    """Full-size parity: the GPU run's first history entries against the
    oracle's run of the SAME system (same b, x0 = 0) in the cpu_baseline leg.
    The oracle stops at maxiter (its last entry is the exit branch's
    recomputed norm of the same r), so entries are compared by index. A GPU
    history shorter than the oracle's is a parity failure (ok false, both
    lengths recorded), never an exception -- unless `overlap` (C1: the oracle
    runs to convergence, the timed GPU run a fixed count), where the common
    prefix is compared."""
    import numpy as np
    g_all = np.asarray(gpu_info["residual"], dtype=np.float64)
    r_all = np.asarray(ref_info["residual"], dtype=np.float64)
    m = min(len(r_all), len(g_all)) if overlap else len(r_all)
    r_res = r_all[:m]
    ref_info = dict(ref_info, nosl=np.asarray(ref_info["nosl"])[:m])
    c = min(m, len(g_all))
    g_res = g_all[:c]
    nosl_eq = bool(len(gpu_info["nosl"]) >= m and
                   np.array_equal(np.asarray(gpu_info["nosl"][:m]), ref_info["nosl"]))
    big = r_res[:c] >= 1e-8
    rel = np.abs(g_res - r_res[:c]) / np.abs(r_res[:c])
    max_rel = float(rel[big].max()) if big.any() else 0.0
    ok = nosl_eq and c == m and max_rel <= rtol
    return dict(ok=bool(ok), entries=int(c), oracle_entries=int(len(r_all)), nosl_equal=nosl_eq,
                max_rel=max_rel, rtol=rtol,
                reference="oracle.v3cpu (bitwise the reference's v3/cpu), same b, x0 = 0",
                shown=min(c, 12), gpu=[float(v) for v in g_res[:12]],
                oracle=[float(v) for v in r_res[:12]])


def stored_format_delta(nnz, n, lay, long_row=12.0):
    """CSR algorithmic bytes (12 nnz + rowptr + vectors) minus
    the bytes the shard's stored format streams for the same SpMV: offset
    masks replace the 4-byte columns by mw/8 bytes per row, a value
    dictionary the 8-byte values by 1-byte codes; long masked rows use the
    diagonal-offset values (8 bytes per offset and row, no rowptr); the
    stencil SpMV streams code_bits bytes of codes per row (8 slots of
    code_bits bits) and nothing else of A -- or, with code patterns, one
    4-byte pattern id per 512-row block plus the pattern table once. The DIA
    walk loads no masks over its run of full blocks (dia_full_blocks)."""
    if lay.get("stencil_walk"):
        if lay.get("code_patterns"):
            cb = float(lay.get("code_bits") or 8)
            a_bytes = 4.0 * -(-n // 512) + lay["code_patterns"] * 512 * cb
            return 12.0 * nnz + 4.0 * (n + 1) - a_bytes
        return 12.0 * nnz + 4.0 * (n + 1) - float(lay.get("code_bits") or 8) * n
    mw = lay["mask_bits"]
    if mw and lay["dict_values"] == 0 and nnz >= long_row * n:  # DIA (KR_DIA=1)
        n_pad = -(-n // 256) * 256
        # symmetric values: the lower entries are read as the mirrored upper
        # ones (L2 hits), so only the upper half + diagonal must stream
        slots = (lay["n_offsets"] + 1) // 2 if lay.get("dia_sym") else lay["n_offsets"]
        mask_rows = max(n - 256 * int(lay.get("dia_full_blocks") or 0), 0)
        return 12.0 * nnz + 4.0 * (n + 1) - (8.0 * slots * n_pad + mw / 8 * mask_rows)
    d = 0.0
    if mw:
        d += 4.0 * nnz - mw / 8 * n
    if lay["dict_values"]:
        d += 7.0 * nnz
    return d


def format_name(lay):
    if lay.get("stencil_walk"):
        cb = lay.get("code_bits") or 8
        codes = (f"{lay['code_patterns']} distinct 512-row code blocks, a 4-byte pattern id per "
                 f"block" if lay.get("code_patterns") else "per row")
        return (f"stencil codes (8 x {cb}-bit dictionary codes per row, {codes}; "
                f"{lay['dict_values']}-entry table; walk {lay['stencil_walk']} blocks)")
    if lay.get("dia_sym"):
        return (f"diagonal-offset values, {lay['n_offsets']} offsets, symmetric (upper half + "
                f"diagonal streamed, lower entries read as the mirrored upper ones)")
    parts = [f"offset masks ({lay['mask_bits']}-bit)" if lay["mask_bits"] else "CSR columns"]
    parts.append(f"{lay['dict_values']}-entry value dictionary (1-byte codes)"
                 if lay["dict_values"] else "8-byte values")
    return ", ".join(parts)


def pmc_traffic(config, kernel):
    """Beyond-L2 bytes per launch of `kernel` in config `config` (e.g. "C4",
    "C4_csr") from the committed rocprofv3 PMC summary profiles/pmc/<config>.json
    (tools/profile.sh + tools/pmc_summary.py on that config's bench command:
    TCC_EA0_RDREQ_{32B,64B,128B} / WRREQ request sizes). None when no profile
    of this (config, kernel) pair exists: a kernel of another config or
    another format never lends its bytes."""
    path = os.path.join(REPO, "profiles", "pmc", f"{config}.json")
    try:
        with open(path) as f:
            prof = json.load(f)
    except (OSError, ValueError):
        return None
    if prof.get("_meta", {}).get("config") != config:
        return None
    rec = prof.get("kernels", {}).get(kernel)
    return None if rec is None else rec.get("traffic_bytes")


def run_system(args, cfg, mat, n, world, rank, local, comm, method, k, env=None):
    """Build the system (optionally under KR_* format overrides, read at
    finalize), run warmup + the timed steps, and return the measurements.
    Timed region: barrier + device sync on both sides, max over ranks."""
    import torch
    import torch.distributed as dist
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition
    saved = {key: os.environ.get(key) for key in (env or {})}
    os.environ.update(env or {})
    try:
        part = balanced_partition(n, world)
        S = max(1, args.local_shards)
        lo, hi = part[rank], part[rank + 1]
        rows = [lo + (hi - lo) * j // S for j in range(S + 1)]
        sysm = KrylovSystem(n, rows, [local] * S, comm)
        if mat[0] == "poisson":
            sysm.gen_poisson(mat[1], mat[2])
        else:
            sysm.gen_banded(mat[2], mat[3], mat[4])
        sysm.finalize()
    finally:
        for key, v in saved.items():
            if v is None:
                os.environ.pop(key, None)
            else:
                os.environ[key] = v
    info = sysm.shard_info(0)
    shards = []  # (info, layout) per local shard: the stored-format bytes per shard
    for j in range(S):
        l_ = sysm.shard_layout(j)
        l_["stencil_walk"] = sysm.shard_sched(j)["stencil_walk"]
        shards.append((sysm.shard_info(j), l_))
    lay = shards[0][1]
    # b = default_rng(1).standard_normal(N), the global
    # vector's own rows per shard; --rhs hash: the device counter hash (2u-1)
    b = sysm.split(rhs_host(n)) if args.rhs == "normal" else sysm.rhs(1)
    per_step = (k + 1) if "kskip" in method else 1
    maxiter = (args.warmup + args.steps + 4) * per_step + 2
    # per-kernel HIP events on every 4th step (each event pair costs ~10 us of
    # launch gap; sampled, the timing costs <1 % at the 8-GPU shard size)
    sysm.begin(method, b, None, tol=0.0, maxiter=maxiter, k=k,
               profile=0 if args.no_profile else (args.profile_every or PROFILE_EVERY.get(
                   args.config, 4)))
    sysm.step(args.warmup)
    sysm.reset_kernel_stats()

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sysm.step(args.steps)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    stats = sysm.kernel_stats()
    out = sysm.finish(method)
    sysm.close()
    del b
    torch.cuda.empty_cache()
    return dict(info=info, lay=lay, shards=shards, per_step=per_step, elapsed=elapsed,
                stats=stats, history=out.info)


def parallelism(world: int, local_shards: int) -> str:
    """What the run actually exchanges: one shard on one GPU moves nothing."""
    if world == 1 and local_shards <= 1:
        return "1 GPU, one shard (no halo exchange, no collective)"
    if world == 1:
        return (f"1 GPU, {local_shards} in-process shards (halo device copies, shard "
                f"partials summed in shard order)")
    return (f"row-partitioned x{world} ranks (one GPU each), RCCL halo send/recv + Gram "
            f"all-gather" + (f"; {local_shards} in-process shards per rank"
                             if local_shards > 1 else ""))


METHOD_NAMES = {"cg": "CG", "mrr": "MrR", "kskipcg": "k-skip CG", "kskipmrr": "k-skip MrR",
                "adaptivekskipmrr": "Adaptive k-skip MrR"}


def workload_label(config, method, k, mat, n):
    """The workload actually run (method, k, matrix, N), not the config's
    default label: --n-side / --nz / --method / --k change it."""
    m = METHOD_NAMES.get(method, method) + (f" k={k}" if "kskip" in method else "")
    if mat[0] == "poisson":
        side, dim = mat[1], mat[2]
        pts = 5 if dim == 2 else 7
        grid = f"{side}^{dim}" if len(mat) == 3 else f"{side}^{dim - 1} x {mat[3]} planes"
        a = f"{dim}D {pts}-point Poisson {grid}"
    else:
        a = f"random banded CSR N={mat[1]}, {2 * mat[2] + 1} nnz/row (band {mat[3]})"
    return f"{config}: {m} on {a} (N={n})"


def kernel_table(stats, deltas):
    """Per kernel: launches, average ms and GB/s on the stored format's bytes
    and on SURVEY.md 8(d)'s CSR bytes. A launch is one call of the op on the
    first shard's device (kr_solve_kernel_stats): its time is the device
    window of the `shards` shards it covers there, its CSR bytes theirs
    summed, so the stored-format bytes subtract those shards' own deltas
    (`deltas`: stored_format_delta per shard, in shard order; a float is one
    shard's). The same figures whether the shards share a stream or not."""
    if not isinstance(deltas, (list, tuple)):
        deltas = [float(deltas)]
    kernels, stored = {}, {}
    for s_ in stats:
        if s_["name"].startswith("host_"):  # host-side timing (host_table)
            continue
        if s_["launches"]:
            avg = s_["total_ms"] / s_["launches"]
            nsh = max(1, int(s_.get("shards", 1)))
            csr = s_["bytes_per_launch"]
            # the launch covers the first nsh shards of this process, each of
            # which has its delta: more shards than deltas is a bookkeeping
            # error of the caller, never padded over
            if nsh > len(deltas):
                raise ValueError(f"{s_['name']}: a launch covers {nsh} shards but only "
                                 f"{len(deltas)} stored-format deltas were given")
            d = sum(deltas[:nsh])
            st = csr - (d if s_["name"].startswith("spmv") else 0.0)
            stored[s_["name"]] = (st, csr)
            kernels[s_["name"]] = dict(launches=s_["launches"], avg_ms=round(avg, 5),
                                       gbs=round(st / avg / 1e6, 1),
                                       csr_gbs=round(csr / avg / 1e6, 1),
                                       total_ms=round(s_["total_ms"], 3))
            if nsh > 1:
                kernels[s_["name"]]["shards"] = nsh
    return kernels, stored


def checked_frac(achieved_gbs, peak=None):
    """achieved / peak, or None when that exceeds 1: a fraction above the HBM
    peak is a bookkeeping error (bytes and time of different shard sets),
    never a measurement, so it is not printed as one."""
    peak = HBM_PEAK_GBS if peak is None else peak
    f = achieved_gbs / peak
    return round(f, 4) if f <= 1.0 else None


def frac_fields(achieved_gbs, peak=None):
    """{"frac": ...}, plus "frac_error" saying why when checked_frac refuses
    the value (above the peak): the record shows the mismatch instead of a
    silent null."""
    peak = HBM_PEAK_GBS if peak is None else peak
    f = checked_frac(achieved_gbs, peak)
    out = dict(frac=f)
    if f is None:
        out["frac_error"] = (f"achieved {achieved_gbs} GB/s exceeds the {peak} GB/s peak: "
                             f"bytes and time of different shard sets")
    return out


def host_table(stats):
    """Host time per outer iteration (every iteration, not sampled): enqueue =
    the launch / copy / event calls the host thread issues, wait = blocked in
    the sync point's device-to-host read (kr_solve_step, System::reduce)."""
    out = {}
    for s_ in stats:
        if s_["name"].startswith("host_") and s_["launches"]:
            out[s_["name"][5:] + "_ms_per_step"] = round(s_["total_ms"] / s_["launches"], 4)
    return out or None


def kernel_sampling(kernels, run, args):
    """How the per-kernel table was measured, and its overhead: HIP events
    around every kernel of every N-th outer iteration only; the event pairs
    delay the launches they bracket, so the sampled steps run slower than the
    unsampled ones (sum of per-kernel averages per step vs ms_per_step)."""
    if not kernels:
        return None
    every = args.profile_every or PROFILE_EVERY.get(args.config, 4)
    # kr_solve_kernel_stats_reset restarts the sampling at the first timed
    # step: steps 0, N, 2N, ... of the window are the sampled ones
    sampled_steps = max(1, -(-args.steps // every))
    per_step = sum(v["total_ms"] for v in kernels.values()) / sampled_steps
    step_ms = run["elapsed"] / args.steps * 1e3
    return dict(every=every, sampled_steps=sampled_steps,
                kernel_sum_ms_per_step=round(per_step, 4),
                over_ms_per_step=round(per_step / step_ms - 1.0, 4),
                note="kernel times are HIP events on the solver stream around every kernel of "
                     "every N-th step; the sum per sampled step exceeds ms_per_step by the "
                     "event pairs' launch gaps (not counted in value)")


def step_roofline(kernels, stored, run, args, per_step, n, nnz_total, method, k):
    """The whole outer iteration against HBM (report the
    whole-iteration fraction beside the SpMV kernel's): the stored-format
    bytes of every kernel of a sampled step, divided by ms_per_step, and
    SURVEY 8(d)'s fused-minimal CSR bytes per solver iteration with the
    it/s they would allow at the 8 TB/s peak (k-skip MrR: (3k+1) B_spmv +
    (2k+3) 8N + 9(k+1) 8N per outer iteration; one-GPU runs). Per GPU."""
    if not kernels:
        return None
    every = args.profile_every or PROFILE_EVERY.get(args.config, 4)
    sampled = max(1, -(-args.steps // every))
    byts = sum(stored[n_][0] * v["launches"] for n_, v in kernels.items()) / sampled
    step_s = run["elapsed"] / args.steps
    out = dict(stored_bytes_per_step=round(byts), achieved=round(byts / step_s / 1e9, 1),
               peak=HBM_PEAK_GBS, unit="GB/s", **frac_fields(round(byts / step_s / 1e9, 1)))
    if method in ("kskipmrr", "adaptivekskipmrr") and k > 0 and nnz_total > 0:
        b_spmv = 12.0 * nnz_total + 4.0 * (n + 1) + 16.0 * n
        per_iter = ((3 * k + 1) * b_spmv + (2 * k + 3) * 8.0 * n + 9 * (k + 1) * 8.0 * n) / (k + 1)
        out.update(survey_csr_bytes_per_iteration=round(per_iter),
                   survey_csr_ideal_its=round(HBM_PEAK_GBS * 1e9 / per_iter, 1))
    return out


def dominant(kernels):
    spmv = {n_: v for n_, v in kernels.items() if n_.startswith("spmv")}
    return max(spmv or kernels, key=lambda n_: kernels[n_]["total_ms"])


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    from parallel_krylov_amd.system import Communicator

    cfg = dict(CONFIGS[args.config])
    method = args.method or cfg["method"]
    mat = list(cfg["matrix"])
    if args.n_side is not None and mat[0] == "poisson":
        mat[1] = args.n_side
    comm = None
    if world > 1:
        dist.init_process_group("gloo")
        comm = Communicator.from_torch(None, local)
    if args.nz is not None and mat[0] == "poisson":
        n = mat[1] ** (mat[2] - 1) * args.nz
        mat.append(args.nz)
    else:
        n = mat[1] ** mat[2] if mat[0] == "poisson" else mat[1]
    k = (args.k if args.k is not None else cfg["k"]) if "kskip" in method else 0

    run = run_system(args, cfg, mat, n, world, rank, local, comm, method, k)
    info, lay, per_step = run["info"], run["lay"], run["per_step"]
    deltas = [stored_format_delta(i_["nnz"], i_["n_local"], l_) for i_, l_ in run["shards"]]
    iterations = args.steps * per_step
    value = iterations / run["elapsed"]
    kernels, stored = kernel_table(run["stats"], deltas)
    roofline = None
    if kernels:
        dom = dominant(kernels)
        d = kernels[dom]
        ach = d["gbs"]
        # achieved = the minimum bytes of the format the kernel streams (offset
        # masks instead of columns, 1-byte dictionary codes instead of values:
        # DESIGN.md 9); the CSR figure of SURVEY.md 8(d) is csr_equiv_gbs
        roofline = dict(bound="hbm", kernel=dom, achieved=ach, peak=HBM_PEAK_GBS, unit="GB/s",
                        **frac_fields(ach),
                        copy_peak=HBM_COPY_GBS, frac_of_copy=round(ach / HBM_COPY_GBS, 4),
                        traffic=pmc_traffic(args.config, dom),
                        traffic_source=f"profiles/pmc/{args.config}.json",
                        bytes_per_launch=stored[dom][0], csr_bytes_per_launch=stored[dom][1],
                        csr_equiv_gbs=d["csr_gbs"], format=format_name(lay),
                        avg_ms=d["avg_ms"])

    # The same workload on plain CSR (no offset masks, no value dictionary:
    # 4-byte columns and 8-byte values streamed), timed in the same run: the
    # north star's "CSR SpMV" roofline on SURVEY.md 8(d)'s bytes.
    csr_rec = None
    if not args.no_csr and (lay["mask_bits"] or lay["dict_values"]):
        rc = run_system(args, cfg, mat, n, world, rank, local, comm, method, k,
                        env={"KR_MASK": "0", "KR_VDICT": "0", "KR_STENCIL": "0"})
        kc, _ = kernel_table(rc["stats"], [0.0])
        csr_rec = dict(value=round(iterations / rc["elapsed"], 3), unit="iterations/s",
                       ms_per_step=round(rc["elapsed"] / args.steps * 1e3, 4),
                       format=format_name(rc["lay"]), env="KR_MASK=0 KR_VDICT=0 KR_STENCIL=0")
        if kc:
            dc = dominant(kc)
            csr_rec.update(kernel=dc, avg_ms=kc[dc]["avg_ms"], achieved=kc[dc]["gbs"],
                           **frac_fields(kc[dc]["gbs"]),
                           traffic=pmc_traffic(args.config + "_csr", dc),
                           traffic_source=f"profiles/pmc/{args.config}_csr.json",
                           kernels=kc)

    base = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.local_shards == 1:
        n_side = args.cpu_n_side if args.config == "C4" else None
        base, ref_info = cpu_baseline(args.config, mat, k, method, n_side=n_side,
                                      return_info=True)
        if ref_info is not None and args.rhs == "normal":
            parity = history_parity(run["history"], ref_info, overlap=args.config == "C1")
    if rank == 0:
        rec = {
            "metric": (HEADLINE_METRIC if args.config == "C4" and method == cfg["method"]
                       else f"solver iterations/sec, {cfg['label']}"
                       + ("" if method == cfg["method"] else f" ({method})")),
            "value": round(value, 3),
            "unit": "iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(run["elapsed"] / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic: CSR matrix generated on device; b = "
                     + ("default_rng(1).standard_normal(N) (host, SURVEY.md 8(d))"
                        if args.rhs == "normal" else "2u-1 counter hash (device)")),
            "config": {"workload": workload_label(args.config, method, k, mat, n)
                                   + f", nnz/shard={info['nnz']}, tol=0 fixed iterations",
                       "method": method, "k": k, "matrix": mat,
                       "step": f"one outer iteration = {per_step} solver iterations",
                       "parallelism": parallelism(world, args.local_shards)},
            "roofline": roofline,
            "cpu_baseline": base,
            "parity": parity,
            "csr": csr_rec,
            "kernels": kernels,
            "kernel_sampling": kernel_sampling(kernels, run, args),
            "step_roofline": step_roofline(kernels, stored, run, args, run["per_step"], n,
                                           run["info"].get("nnz", 0) if world == 1 else 0,
                                           method, k),
            "host": host_table(run["stats"]),
            "residual_tail": [float(v) for v in run["history"]["residual"][-3:-1]],
        }
        print(json.dumps(rec))
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
