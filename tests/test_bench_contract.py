"""bench.py pieces that run without a GPU: the headline metric string is
BASELINE.json's, the configs match BASELINE.json's list, the CPU-baseline leg
(the oracle, bitwise the reference's v3/cpu) produces the cpu_baseline object,
the PMC traffic lookup reads profiles/pmc/<config>.json keyed by (config,
kernel), and the full-size parity check compares history entries."""
import json
import os

import pytest

from conftest import REPO


def test_headline_metric_is_baselines():
    import bench
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        base = json.load(f)
    assert bench.HEADLINE_METRIC == base["metric"]
    # the bench's default config is the headline one (512^3 7-point, k=4)
    c4 = bench.CONFIGS["C4"]
    assert c4["method"] == "kskipmrr" and c4["k"] == 4 and c4["matrix"] == ("poisson", 512, 3)


def test_cpu_baseline_object_small_sample():
    import bench
    rec = bench.cpu_baseline("C4", ["poisson", 512, 3], 4, "kskipmrr", n_side=12)
    assert set(rec) >= {"value", "unit", "cores", "kind", "sample", "cpu_model",
                        "affinity_cores", "blas_threads"}
    assert rec["kind"] == "port" and rec["unit"] == "iterations/s"
    assert rec["cpu_model"] and rec["affinity_cores"] >= 1
    assert "2 outer" in rec["sample"]  # initial step + 2 outer iterations
    assert rec["value"] > 0 and rec["cores"] >= 1
    assert "scaled" in rec["sample"]  # a 12^3 sample is scaled to 512^3 by rows
    assert "standard_normal" in rec["sample"]


def test_cpu_baseline_every_config(monkeypatch):
    """Every config line carries a cpu_baseline: C1 is the v3/cpu CG run to
    1e-10 on its own system (the config BASELINE.json defines as v3/cpu) and
    returns the oracle history for the bench's parity field; banded configs
    sample the same generator at a stated N, scaled by the row ratio."""
    import numpy as np
    import bench
    from oracle import matrices, v3cpu
    rec, info = bench.cpu_baseline("C1", ["poisson", 256, 2], 0, "cg", return_info=True)
    assert rec["sample_n"] == rec["full_n"] == 65536 and "to tol 1e-10" in rec["sample"]
    assert info["residual"][-1] < 1e-10 and rec["value"] > 0
    A = matrices.poisson(256, 2)
    _, ref = v3cpu.cg(A, np.random.default_rng(1).standard_normal(A.shape[0]), tol=1e-10)
    np.testing.assert_array_equal(info["residual"], ref["residual"])
    monkeypatch.setitem(bench.CPU_SAMPLE, "C5", dict(outer=1, n=3000))
    rec, info = bench.cpu_baseline("C5", ["banded", 50_000_000, 31, 256, 0], 4,
                                   "adaptivekskipmrr", return_info=True)
    assert info is None  # a reduced sample is no parity reference
    assert rec["sample_n"] == 3000 and "scaled" in rec["sample"] and "1 outer" in rec["sample"]


def test_parallelism_is_truthful():
    import bench
    assert "no halo exchange" in bench.parallelism(1, 1)
    assert "in-process" in bench.parallelism(1, 8) and "RCCL" not in bench.parallelism(1, 8)
    assert "RCCL" in bench.parallelism(8, 1)


def test_pmc_traffic_from_committed_profile():
    import bench
    with open(os.path.join(REPO, "profiles", "pmc", "C4.json")) as f:
        prof = json.load(f)
    assert prof["_meta"]["config"] == "C4"
    # the headline's box walks (the step triple is C4's roofline kernel)
    kern = "spmv_step3_mrr_stencil"
    t = bench.pmc_traffic("C4", kern)
    assert t == prof["kernels"][kern]["traffic_bytes"] and t > 1e9
    assert bench.pmc_traffic("C4", "no_such_kernel") is None
    # another config never borrows C4's bytes
    assert bench.pmc_traffic("C1", kern) is None
    assert bench.pmc_traffic("C5", kern) is None or bench.pmc_traffic("C5", kern) != t


def test_history_parity_contract():
    """bench `parity`: nosl equal and entries >= 1e-8 within 1e-12 relative."""
    import numpy as np
    import bench
    ref = {"nosl": np.array([0, 1, 6]), "residual": np.array([1.0, 0.5, 0.25])}
    gpu = {"nosl": np.array([0, 1, 6, 11]), "residual": np.array([1.0, 0.5 * (1 + 1e-13), 0.25, 0.1])}
    p = bench.history_parity(gpu, ref)
    assert p["ok"] and p["entries"] == 3 and p["max_rel"] < 1e-12
    gpu["residual"][2] = 0.25 * (1 + 1e-10)
    assert not bench.history_parity(gpu, ref)["ok"]
    gpu["residual"][2] = 0.25
    gpu["nosl"][2] = 5
    assert not bench.history_parity(gpu, ref)["ok"]
    # a GPU history shorter than the oracle's: ok false with both lengths, no raise
    short = {"nosl": np.array([0, 1]), "residual": np.array([1.0, 0.5])}
    p = bench.history_parity(short, ref)
    assert not p["ok"] and p["entries"] == 2 and p["oracle_entries"] == 3
    # C1: the oracle ran to convergence, the timed GPU run a fixed count --
    # the common prefix is the comparison
    p = bench.history_parity(short, ref, overlap=True)
    assert p["ok"] and p["entries"] == 2 and p["oracle_entries"] == 3


def test_stored_format_bytes():
    """The roofline's bytes are the stored format's: masks replace the 4-byte
    columns, a value dictionary the 8-byte values; long masked rows are DIA."""
    import bench
    n, nnz = 1000, 7000
    csr = dict(mask_bits=0, n_offsets=0, dict_values=0)
    assert bench.stored_format_delta(nnz, n, csr) == 0.0
    masked = dict(mask_bits=8, n_offsets=7, dict_values=0)
    assert bench.stored_format_delta(nnz, n, masked) == 4.0 * nnz - 1.0 * n
    both = dict(mask_bits=8, n_offsets=7, dict_values=2)
    assert bench.stored_format_delta(nnz, n, both) == 11.0 * nnz - 1.0 * n
    dia = dict(mask_bits=32, n_offsets=27, dict_values=0)
    nnz_long = 27 * n
    assert bench.stored_format_delta(nnz_long, n, dia) == (
        12.0 * nnz_long + 4.0 * (n + 1) - (8.0 * 27 * 1024 + 4.0 * n))
    # the DIA walk's full-block run: no mask bytes for its rows
    dia_run = dict(dia, dia_sym=1, dia_full_blocks=2)
    assert bench.stored_format_delta(nnz_long, n, dia_run) == (
        12.0 * nnz_long + 4.0 * (n + 1) - (8.0 * 14 * 1024 + 4.0 * (n - 512)))
    assert "dictionary" in bench.format_name(both) and "masks" in bench.format_name(both)
    st = dict(mask_bits=8, n_offsets=7, dict_values=2, stencil_walk=512)
    assert bench.stored_format_delta(nnz, n, st) == 12.0 * nnz + 4.0 * (n + 1) - 8.0 * n
    assert "stencil" in bench.format_name(st)
    # narrow codes: 2 bits per slot (<= 3 dictionary values) stream 2 B per row
    st2 = dict(st, code_bits=2)
    assert bench.stored_format_delta(nnz, n, st2) == 12.0 * nnz + 4.0 * (n + 1) - 2.0 * n
    assert "2-bit" in bench.format_name(st2)
    # code patterns: a 4-byte pattern id per 512-row block + the table once
    stp = dict(st2, code_patterns=9)
    assert bench.stored_format_delta(nnz, n, stp) == (
        12.0 * nnz + 4.0 * (n + 1) - (4.0 * 2 + 9 * 512 * 2.0))
    assert "9 distinct 512-row code blocks" in bench.format_name(stp)


def test_step_roofline_survey_figures():
    """bench.step_roofline: the whole outer iteration's stored bytes per
    ms_per_step, and SURVEY.md 8(d)'s fused-minimal CSR bytes of k-skip MrR
    (C4: 48.27 GB per solver iteration, ideal 166 it/s at 8 TB/s)."""
    import argparse
    import bench
    n = 512 ** 3
    nnz = 937951232
    kernels = {"spmv2_gram_mrr": {"launches": 6}, "spmv_step_mrr_nox": {"launches": 4}}
    stored = {"spmv2_gram_mrr": (4.56e9, 16.09e9), "spmv_step_mrr_nox": (6.7e9, 18e9)}
    args = argparse.Namespace(profile_every=4, config="C4", steps=8)
    run = {"elapsed": 8 * 9.5e-3}
    out = bench.step_roofline(kernels, stored, run, args, 5, n, nnz, "kskipmrr", 4)
    assert out["stored_bytes_per_step"] == round((6 * 4.56e9 + 4 * 6.7e9) / 2)
    assert abs(out["survey_csr_bytes_per_iteration"] / 1e9 - 48.27) < 0.01
    assert abs(out["survey_csr_ideal_its"] - 165.7) < 0.2
    assert 0 < out["frac"] == round(out["achieved"] / 8000.0, 4) or abs(
        out["frac"] - out["achieved"] / 8000.0) < 1e-3


def test_multi_shard_kernel_table_is_per_device():
    """Review item (round 4): with several in-process shards the stats record
    one device window per call covering `shards` shards, with their CSR bytes
    summed (kr_solve_kernel_stats, ABI 204): the stored-format bytes must
    subtract every covered shard's delta, not shard 0's alone, and a frac
    above 1 is never printed (bench.checked_frac). The same stats read the
    same whether the shards shared a stream (one group window) or ran on a
    stream each (overlapping windows, merged by the engine)."""
    import bench
    n, nnz = 512 ** 3 // 8, 937951232 // 8  # one 64-plane shard of C4
    lay = dict(mask_bits=8, n_offsets=7, dict_values=2, stencil_walk=512, code_bits=2,
               code_patterns=9)
    d = bench.stored_format_delta(nnz, n, lay)
    csr = 12.0 * nnz + 4.0 * (n + 1) + 32.0 * n  # one shard's dual, CSR bytes
    stored1 = csr - d
    # 1 shard: 0.11 ms per dual; 8 shards on one device: 8 x 0.11 ms window
    one = [dict(name="spmv2_gram_mrr", launches=10, total_ms=10 * 0.11, bytes_per_launch=csr,
                shards=1)]
    eight = [dict(name="spmv2_gram_mrr", launches=10, total_ms=10 * 0.88,
                  bytes_per_launch=8 * csr, shards=8)]
    k1, s1 = bench.kernel_table(one, [d])
    k8, s8 = bench.kernel_table(eight, [d] * 8)
    assert s1["spmv2_gram_mrr"][0] == stored1
    assert s8["spmv2_gram_mrr"][0] == 8 * stored1
    assert k8["spmv2_gram_mrr"]["shards"] == 8
    f1 = bench.checked_frac(k1["spmv2_gram_mrr"]["gbs"])
    f8 = bench.checked_frac(k8["spmv2_gram_mrr"]["gbs"])
    assert f1 is not None and f8 is not None and f8 <= 1.0
    assert abs(f8 - f1) / f1 < 0.01
    # the round-4 bookkeeping (8 shards' bytes less ONE shard's delta) would
    # have claimed more than the HBM peak: refused
    bogus = (8 * csr - d) / (0.88 * 1e6)
    assert bench.checked_frac(bogus) is None
    rec = bench.frac_fields(bogus)
    assert rec["frac"] is None and "exceeds" in rec["frac_error"]  # said, not a silent null
    assert "frac_error" not in bench.frac_fields(k1["spmv2_gram_mrr"]["gbs"])
    # a shard count past the listed deltas is a bookkeeping error: refused
    with pytest.raises(ValueError):
        bench.kernel_table([dict(eight[0], shards=2)], [d])
    # non-SpMV kernels keep their bytes
    kv, sv = bench.kernel_table([dict(name="update_mrr", launches=2, total_ms=1.0,
                                      bytes_per_launch=1e9, shards=8)], [d] * 8)
    assert sv["update_mrr"][0] == 1e9
