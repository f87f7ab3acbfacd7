"""Summarise tools/ab_pmc.sh output: per variant, the icp_kernel counters."""
import csv
import glob
import os
import sys

root = sys.argv[1]
for v in sys.argv[2:]:
    files = glob.glob(os.path.join(root, v, "**", "*counter_collection.csv"), recursive=True)
    tot = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if "icp_kernel" not in row["Kernel_Name"]:
                continue
            tot[row["Counter_Name"]] = tot.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    wc = tot.get("SQ_WAVE_CYCLES", 1.0)
    line = " ".join(f"{k}={tot[k]:.4g}" for k in sorted(tot))
    frac = " ".join(f"{k[3:]}/WC={tot[k] / wc:.3f}" for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                             "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SALU") if k in tot)
    print(v, line)
    print(v, frac)
