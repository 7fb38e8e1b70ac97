"""Publish one config's PMC summary for bench.py's roofline `traffic`.

    python tools/pmc_publish.py <profile dir> <config> [source tag]

<profile dir> is a tools/profile.sh output (summary.json by
tools/pmc_summary.py) of ONE config's bench command; <config> names it as
bench.py does ("C4", "C4_csr" for the KR_MASK=0 KR_VDICT=0 run, "C5", ...).
Writes profiles/pmc/<config>.json:

    {"_meta": {"config": ..., "source": ..., "counters": ...},
     "kernels": {<engine kernel name>: {"traffic_bytes", "read_bytes",
                                        "write_bytes", "avg_ms", ...}}}

Kernel names are the engine's (kr_engine.cpp epi_name / ew_name), the names
bench.py's per-kernel table uses: pmc_summary's "_dia" / "_dense" / "_stencil" / "_rp64"
variant suffixes are folded (one config runs one variant of a kernel).
bench.pmc_traffic(config, kernel) returns null for any other pair.
"""
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def engine_name(name):
    if name.startswith(("spmv_step2_mrr_stencil", "spmv_step3_mrr_stencil", "spmv_step2h_mrr_stencil")):
        return name  # the box step walks: the engine books them under these names
    return re.sub(r"(_rp64)?(_dia|_dense|_stencil)?$", "", name)


def main(d, config, source=None):
    with open(os.path.join(d, "summary.json")) as f:
        summ = json.load(f)
    kernels = {}
    for name, rec in summ.items():
        if "traffic_bytes" not in rec:
            continue
        en = engine_name(name)
        if en in kernels:
            raise SystemExit(f"{config}: two variants of {en} in one profile ({name})")
        kernels[en] = {k: rec[k] for k in ("traffic_bytes", "read_bytes", "write_bytes",
                                          "avg_ms", "launches", "l2_hit", "dram_read_share",
                                          "fetch_size_kb", "write_size_kb") if k in rec}
        kernels[en]["profiled_as"] = name
    meta = {"config": config, "source": source or os.path.relpath(d, REPO),
            "counters": "TCC_EA0_RDREQ_{128B,64B,32B} x {128,64,32} B + TCC_EA0_WRREQ(_64B) "
                        "x {64,32} B per launch (beyond-L2 requests; FETCH_SIZE/WRITE_SIZE "
                        "recorded beside them, FETCH_SIZE = RDREQ x 64 B on gfx950)"}
    out_dir = os.path.join(REPO, "profiles", "pmc")
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, f"{config}.json"), "w") as f:
        json.dump({"_meta": meta, "kernels": kernels}, f, indent=1, sort_keys=True)
    print(f"profiles/pmc/{config}.json: {len(kernels)} kernels")


if __name__ == "__main__":
    main(*sys.argv[1:])
