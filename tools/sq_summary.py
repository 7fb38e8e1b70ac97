"""Per-kernel SQ/TA issue figures from a tools/sq_profile.sh directory (mean
per launch). SQ cycle counters are quad-cycles summed over waves; ratios are
shares of SQ_WAVE_CYCLES; instruction counts are per wave."""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main(d):
    cnt = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv")):
        for row in csv.DictReader(open(path)):
            cnt[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k in sorted(cnt):
        c = {n: sum(v) / len(v) for n, v in cnt[k].items()}
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        waves = max(1.0, c.get("SQ_WAVES", 1.0))
        parts = []
        for n in ("WAIT_ANY", "WAIT_INST_ANY", "ACTIVE_INST_ANY", "ACTIVE_INST_VALU",
                  "ACTIVE_INST_LDS", "ACTIVE_INST_VMEM", "WAIT_INST_LDS"):
            if wc and "SQ_" + n in c:
                parts.append(f"{n.lower()} {100 * c['SQ_' + n] / wc:.0f}%")
        for n in ("VALU", "LDS", "VMEM_RD", "VMEM_WR", "SALU", "SMEM"):
            if "SQ_INSTS_" + n in c:
                parts.append(f"{n.lower()}/wave {c['SQ_INSTS_' + n] / waves:.0f}")
        if "SQ_LDS_BANK_CONFLICT" in c:
            parts.append(f"lds_conf {c['SQ_LDS_BANK_CONFLICT']:.3g}")
        if "TA_TA_BUSY_sum" in c and "GRBM_GUI_ACTIVE" in c:
            parts.append(f"ta_busy/CU {c['TA_TA_BUSY_sum'] / 256:.3g} gui {c['GRBM_GUI_ACTIVE']:.3g}")
        print(f"{k:34s} waves {waves:.0f} wave_cyc {wc:.3g} " + " ".join(parts))


if __name__ == "__main__":
    main(sys.argv[1])
