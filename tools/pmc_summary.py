"""Summarise a tools/profile.sh directory: per kernel, average duration
(rocprofv3 kernel trace) and per-launch HBM-side traffic from the TCC EA
request counters. Writes <dir>/summary.json and prints a table.

Read bytes = 128*RDREQ_128B + 64*RDREQ_64B + 32*RDREQ_32B, write bytes =
64*WRREQ_64B + 32*(WRREQ - WRREQ_64B) (request-size counters, so no width
calibration is needed; FETCH_SIZE is kept for reference: on gfx950 it counts
128-B requests as 64 B). The sizes are checked against the elementwise kernels
whose byte counts are exact (see 'calibration')."""
import collections
import csv
import glob
import json
import os
import re
import sys

# Names follow kr_internal.h's SpmvEpi / EwOp enums (and kr_engine's epi_name/ew_name).
EPI = ["spmv", "spmv_bminus", "spmv_xy", "spmv_head_mrr", "spmv_head_kcg", "spmv_mrr_loop",
       "spmv2", "spmv2_gram_mrr", "spmv2_gram_kcg", "spmv_step_mrr_nox", "spmv_step_mrr_x2",
       "spmv_step_mrr_x", "spmv_step_kcg", "spmv_step_mrr_first2", "spmv_xy_vp", "spmv_mrr_v"]
EW = ["dot", "update_mrr_first", "update_mrr", "update_cg", "update_cg_p", "update_kcg",
      "mrr_s", "copy", "update_mrr_nox", "update_mrr_x2", "fill_one", "precond", "update_pcg",
      "update_cg_gear", "update_gropp_xru", "update_gropp_ps", "precond_div", "update_cg_nox",
      "update_cg_x2", "update_x", "update_pipecg"]


def short(name):
    # the box fused walks (kr_pair.hip), named as System::spmv_pair / spmv_step2 book them
    m = re.search(r"spmv_stencil2b_kernel<(\d+), (\w+), \d+>", name)
    if m:
        base = "spmv2x2_gram_" + ("kcg" if int(m.group(1)) == 8 else "mrr")
        return base + ("_last" if m.group(2) == "true" else "")
    m = re.search(r"spmv_step2b_kernel<(\w+), \d+>", name)
    if m:
        return "spmv_step3_mrr_stencil" if m.group(1) == "true" else "spmv_step2_mrr_stencil"
    if re.search(r"spmv_step2h_kernel<\d+>", name):
        return "spmv_step2h_mrr_stencil"
    m = re.search(r"spmv_kernel2_po<(\w+), (\d+), (\w+)", name)
    if m:  # the plain-CSR row walk's products-only dual (engine name ..._last)
        return EPI[int(m.group(2))] + "_last" + ("" if m.group(1) == "int" else "_rp64")
    m = re.search(r"spmv_kernel\w*<(\w+), (\d+), (\w+)", name)
    if m:
        return EPI[int(m.group(2))] + ("" if m.group(1) == "int" else "_rp64")
    m = re.search(r"spmv_stencil_kernel(?:_w4|_po)?<(\d+), \d+, \w+, \w+, (\d+)(?:, \d+)?>", name)
    if m:  # NTM bit 2: the products-only dual (engine name ..._last)
        return EPI[int(m.group(1))] + ("_last" if int(m.group(2)) & 4 else "") + "_stencil"
    m = re.search(r"spmv_stencil_kernel(?:_w4|_po)?<(\d+)\b", name)
    if m:
        return EPI[int(m.group(1))] + "_stencil"
    m = re.search(r"spmv_diawalk_kernel<(\d+), \d+(?:, (\w+))?>", name)
    if m:  # the symmetric DIA walk (PO = true: the products-only dual, ..._last)
        return EPI[int(m.group(1))] + ("_last" if m.group(2) == "true" else "") + "_dia"
    m = re.search(r"(spmv_dia|gemv)_kernel<(\d+)\b", name)
    if m:
        return EPI[int(m.group(2))] + ("_dia" if m.group(1) == "spmv_dia" else "_dense")
    m = re.search(r"ew_kernel<(\d+), (\w+)", name)
    if m:
        i = int(m.group(1))
        return (EW[i] if i < len(EW) else f"ew{i}") + ("" if m.group(2) == "true" else "_scalar")
    m = re.search(r"(\w+_kernel)\b", name)
    if m and name.startswith(("kr::", "void kr::")):
        return m.group(1)
    return re.sub(r"\(.*", "", name.replace("void ", ""))[:48]


def main(d):
    durs = collections.defaultdict(list)
    for row in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv"))):
        durs[short(row["Kernel_Name"])].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    cnt = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv")):
        for row in csv.DictReader(open(path)):
            cnt[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for k in sorted(set(durs) | set(cnt)):
        c = {n: sum(v) / len(v) for n, v in cnt[k].items()}
        rec = {"launches": len(durs.get(k, [])),
               "avg_ms": (sum(durs[k]) / len(durs[k]) / 1e6) if durs.get(k) else None}
        if "TCC_EA0_RDREQ_128B_sum" in c and "TCC_EA0_RDREQ_64B_sum" in c:
            rd = 128 * c["TCC_EA0_RDREQ_128B_sum"] + 64 * c["TCC_EA0_RDREQ_64B_sum"] + \
                32 * c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
            rec["read_bytes"] = rd
        if "TCC_EA0_WRREQ_sum" in c:
            w64 = c.get("TCC_EA0_WRREQ_64B_sum", 0.0)
            rec["write_bytes"] = 64 * w64 + 32 * (c["TCC_EA0_WRREQ_sum"] - w64)
        if "read_bytes" in rec and "write_bytes" in rec:
            rec["traffic_bytes"] = rec["read_bytes"] + rec["write_bytes"]
        if "FETCH_SIZE" in c:
            rec["fetch_size_kb"] = c["FETCH_SIZE"]
        if "WRITE_SIZE" in c:
            rec["write_size_kb"] = c["WRITE_SIZE"]
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            rec["l2_hit"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        if "TCC_EA0_RDREQ_DRAM_sum" in c and "TCC_EA0_RDREQ_sum" in c:
            # share of the beyond-L2 read requests that go to DRAM (the rest
            # are served by the fabric / Infinity Cache side)
            rec["dram_read_share"] = c["TCC_EA0_RDREQ_DRAM_sum"] / max(1.0, c["TCC_EA0_RDREQ_sum"])
        rec["counters"] = c
        out[k] = rec
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
    print(f"{'kernel':28s} {'n':>4s} {'avg_ms':>8s} {'read GB':>8s} {'write GB':>8s} {'GB/s':>8s} "
          f"{'L2hit':>6s} {'DRAMrd':>6s}")
    for k, r in out.items():
        if r["avg_ms"] is None:
            continue
        rd = r.get("read_bytes", float("nan")) / 1e9
        wr = r.get("write_bytes", float("nan")) / 1e9
        bw = (r.get("traffic_bytes", float("nan")) / (r["avg_ms"] * 1e6))
        print(f"{k:28s} {r['launches']:4d} {r['avg_ms']:8.3f} {rd:8.3f} {wr:8.3f} {bw:8.1f} "
              f"{r.get('l2_hit', float('nan')):6.3f} {r.get('dram_read_share', float('nan')):6.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
