"""bench.py pieces that run without a GPU: the headline metric string is
BASELINE.json's, the configs match BASELINE.json's list, the CPU-baseline leg
(the oracle, bitwise the reference's v3/cpu) produces the cpu_baseline object,
and the PMC traffic lookup reads profiles/latest.json."""
import json
import os

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
    rec = bench.cpu_baseline(12, 4, "kskipmrr")
    assert set(rec) == {"value", "unit", "cores", "kind", "sample"}
    assert rec["kind"] == "port" and rec["unit"] == "iterations/s"
    assert rec["value"] > 0 and rec["cores"] >= 1
    assert "scaled" in rec["sample"]  # a 12^3 sample is scaled to 512^3 by rows


def test_pmc_traffic_from_committed_profile():
    import bench
    with open(os.path.join(REPO, "profiles", "latest.json")) as f:
        prof = json.load(f)
    t = bench.pmc_traffic("spmv2_gram_mrr")
    assert t == prof["spmv2_gram_mrr"]["traffic_bytes"] and t > 1e9
    assert bench.pmc_traffic("no_such_kernel") is None


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
    assert "dictionary" in bench.format_name(both) and "masks" in bench.format_name(both)
