#!/usr/bin/env python3
"""Condense a scripts/profile.sh output directory into profiles/<tag>_rocprof.md and .json:
per-kernel average duration (kernel-trace stats) and per-dispatch PMC averages, plus the
corrected beyond-L2 byte count per launch of the dominant kernel."""
import csv
import json
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = name.replace("ofx::plan::", "").replace("ofx::", "")
    return name.split("(")[0]


def main(src, tag, dst="profiles", alg_bytes=None):
    stats = []
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        stats.append({"kernel": short(r["Name"]), "full_name": r["Name"], "calls": int(r["Calls"]),
                      "avg_us": float(r["AverageNs"]) / 1e3, "min_us": float(r["MinNs"]) / 1e3,
                      "max_us": float(r["MaxNs"]) / 1e3, "pct": float(r["Percentage"])})
    pmc = defaultdict(lambda: defaultdict(list))
    for sub in sorted(os.listdir(src)):
        f = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    pmc_avg = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in pmc.items()}
    main_s = max(stats, key=lambda s: s["pct"])
    main_k = main_s["kernel"]
    # a launch of more than 2^32 threads goes out in pieces (papers-scale: 3 dispatches of
    # spmm_main per op call); the planner runs once per call, so pieces = main / plan dispatches,
    # and per-launch figures are the per-dispatch averages times that
    plan_calls = [s["calls"] for s in stats if s["kernel"].startswith("spmm_plan_kernel")]
    pieces = 1
    if plan_calls and plan_calls[0] and main_s["calls"] % plan_calls[0] == 0:
        pieces = main_s["calls"] // plan_calls[0]
    c = {n: v * pieces for n, v in pmc_avg.get(main_k, {}).items()}
    traffic = {}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        # gfx950: FETCH_SIZE tallies 128-B requests of wide streaming reads at 64 B (x2 correction,
        # MI355X_MICROARCH.md §HBM); WRITE_SIZE is exact for 16-B-per-lane stores.
        traffic["fetch_size_bytes_raw"] = c["FETCH_SIZE"] * 1024
        traffic["write_size_bytes"] = c["WRITE_SIZE"] * 1024
        traffic["read_bytes_corrected_x2"] = 2 * c["FETCH_SIZE"] * 1024
    if "TCC_EA0_RDREQ_128B" in c:
        rd = 128 * c["TCC_EA0_RDREQ_128B"] + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0) + 32 * c.get("TCC_EA0_RDREQ_32B_sum", 0)
        traffic["read_bytes_by_request_size"] = rd
    if traffic:
        rd = traffic.get("read_bytes_by_request_size", traffic.get("read_bytes_corrected_x2"))
        traffic["beyond_l2_bytes_per_launch"] = rd + traffic.get("write_size_bytes", 0)
    if alg_bytes:
        # the gather model's bytes per launch against the measured beyond-L2 bytes,
        # and the dominant kernel's rate / fraction of the 8 TB/s HBM spec at its average duration
        avg_us = main_s["avg_us"] * pieces
        traffic["algorithmic_bytes_per_launch"] = float(alg_bytes)
        if "beyond_l2_bytes_per_launch" in traffic:
            traffic["beyond_l2_over_algorithmic"] = traffic["beyond_l2_bytes_per_launch"] / float(alg_bytes)
        traffic["dominant_kernel_avg_us"] = avg_us  # per launch (all its dispatches)
        traffic["achieved_gbs_gather_model"] = float(alg_bytes) / (avg_us * 1e-6) / 1e9
        traffic["frac_of_8tbs"] = traffic["achieved_gbs_gather_model"] / 8000.0
    traffic["dispatches_per_launch"] = pieces
    out = {"tag": tag, "dominant_kernel": main_k, "kernels": stats, "pmc_avg_per_dispatch": pmc_avg,
           "traffic": traffic}
    os.makedirs(dst, exist_ok=True)
    json.dump(out, open(os.path.join(dst, f"{tag}_rocprof.json"), "w"), indent=1)
    with open(os.path.join(dst, f"{tag}_rocprof.md"), "w") as f:
        f.write(f"# rocprofv3 summary — {tag}\n\nSource: `scripts/profile.sh` raw CSVs ({src}).\n\n")
        f.write("| kernel | calls | avg us | min us | max us | % |\n|---|---|---|---|---|---|\n")
        for s in stats:
            f.write(f"| {s['kernel']} | {s['calls']} | {s['avg_us']:.1f} | {s['min_us']:.1f} | {s['max_us']:.1f} | {s['pct']:.2f} |\n")
        f.write("\n## PMC (average per dispatch)\n\n")
        for k, d in pmc_avg.items():
            f.write(f"- **{k}**: " + ", ".join(f"{n}={v:.4g}" for n, v in sorted(d.items())) + "\n")
        f.write("\n## Traffic of the dominant kernel per launch\n\n")
        for n, v in traffic.items():
            if n.endswith("bytes") or n.endswith("per_launch"):
                f.write(f"- {n}: {v:.4g} bytes ({v / 1e9:.3f} GB)\n")
            else:
                f.write(f"- {n}: {v:.4g}\n")
    print(json.dumps(traffic))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], alg_bytes=float(sys.argv[3]) if len(sys.argv) > 3 else None)
