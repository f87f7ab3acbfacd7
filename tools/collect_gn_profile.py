"""Copy a GN kernel-trace pass (tools/run_gpu_gnprof.sh: tools/prof_gn.py under
rocprofv3 --kernel-trace --stats) into profiles/ and tie it to the GN kernel
sources it measured: profiles/<tag>_gn_kernel_stats.csv plus
profiles/<tag>_gn_profile.json (source hash, commit, per-iteration device time
by kernel from the dispatch trace).

    python tools/collect_gn_profile.py r05
"""
import csv
import hashlib
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GN_SOURCES = ["icp-slam-with-loop-closure_amd/csrc/gn_kernels.hip", "icp-slam-with-loop-closure_amd/csrc/gn_bcr.hip",
              "icp-slam-with-loop-closure_amd/csrc/gn_bcr_gj.hip", "icp-slam-with-loop-closure_amd/csrc/gn_bcr.hpp",
              "icp-slam-with-loop-closure_amd/csrc/common.hpp"]


def gn_source_sha():
    h = hashlib.sha256()
    for p in GN_SOURCES:
        with open(os.path.join(REPO, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def main(tag):
    src = os.path.join(REPO, "gpurun_out", f"gnprof_{tag}")
    dst = os.path.join(REPO, "profiles")
    shutil.copy(os.path.join(src, "gn_kernel_stats.csv"), os.path.join(dst, f"{tag}_gn_kernel_stats.csv"))
    rows = sorted(csv.DictReader(open(os.path.join(src, "gn_kernel_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
    # iterations: each starts with gn_linearize_kernel; per kernel name the mean
    # device time per iteration and the iteration's first-start to last-end span
    its, cur = [], None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0]
        if "gn_linearize_kernel" in name:
            cur = {"kernels": {}, "t0": int(r["Start_Timestamp"]), "t1": 0}
            its.append(cur)
        if cur is None or "gn_" not in name and "bcrgj" not in name:
            continue
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        k = cur["kernels"].setdefault(name, [0, 0])
        k[0] += 1
        k[1] += d
        cur["t1"] = max(cur["t1"], int(r["End_Timestamp"]))
    n = len(its)
    per = {}
    for it in its:
        for name, (c, ns) in it["kernels"].items():
            p = per.setdefault(name, [0, 0])
            p[0] += c
            p[1] += ns
    out = {"tag": tag, "gn_source_sha256": gn_source_sha(), "gn_sources": GN_SOURCES,
           "workload": "tools/prof_gn.py: C4 (5,000 nodes / 20,000 edges) GN iterations, eager launches under "
                       "rocprofv3 --kernel-trace --stats",
           "iterations_traced": n,
           "per_iteration_us_by_kernel": {k: {"launches": round(c / max(n, 1), 2), "device_us": round(ns / max(n, 1) / 1e3, 2)}
                                          for k, (c, ns) in sorted(per.items(), key=lambda kv: -kv[1][1])},
           "per_iteration_span_us_mean_eager_incl_host_gaps": round(sum(it["t1"] - it["t0"] for it in its) / max(n, 1) / 1e3, 2)}
    try:
        out["commit"] = subprocess.run(["git", "-C", REPO, "rev-parse", "--short", "HEAD"], capture_output=True,
                                       text=True, check=True).stdout.strip()
    except Exception:
        out["commit"] = None
    json.dump(out, open(os.path.join(dst, f"{tag}_gn_profile.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r05")
