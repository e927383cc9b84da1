"""Summarize a tools/profile.sh run (gpurun_out/prof_TAG) into profiles/.

Writes
  profiles/<TAG>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<TAG>_summary.json       bench line + per-launch kernel time + PMC traffic
  profiles/pmc_search.json          (with --current) the figure bench.py reports as
                                    roofline.traffic for the same trees/sims

HBM bytes per k_search launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of wide reads, so it
is doubled (MI355X_MICROARCH.md "HBM"); WRITE_SIZE is exact for 16-B stores.
"""
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def read_counter(path, name, kernel="k_search"):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if KNAME[kernel].search(row["Kernel_Name"]) and row["Counter_Name"] == name:
                vals.append((int(row.get("Dispatch_Id", len(vals))), float(row["Counter_Value"])))
    return [v for _, v in sorted(vals)]   # dispatch order: the timed launches are the last


KNAME = {"k_search": re.compile(r"\bk_search<"), "k_im_search": re.compile(r"\bk_im_search<")}


def timed_launches(path, kernel):
    """Durations (ns) of the kernel's dispatches in dispatch order, from a
    rocprofv3 --kernel-trace CSV (empty if the file is absent)."""
    if not os.path.exists(path):
        return []
    rows = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if KNAME[kernel].search(row["Kernel_Name"]):
                rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    rows.sort()
    return [e - s for s, e in rows]


def bench_line(log):
    with open(log) as f:
        for line in f:
            if line.startswith("{"):
                return json.loads(line)
    return None


def main():
    tag = sys.argv[1]
    current = "--current" in sys.argv
    kernel = "k_search"
    pmc_out = "pmc_search.json"
    if "--intmcp" in sys.argv:
        kernel, pmc_out = "k_im_search", "pmc_intmcp.json"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(out, f"{tag}_kernel_stats.csv"))
    stats = {}
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            if KNAME[kernel].search(row["Name"]):
                stats = {"name": row["Name"], "calls": int(row["Calls"]),
                         "avg_ms_all_calls": float(row["AverageNs"]) / 1e6,
                         "min_ms": float(row["MinNs"]) / 1e6, "max_ms": float(row["MaxNs"]) / 1e6}
    fetch = read_counter(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE",
                         kernel)
    write = read_counter(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE",
                         kernel)
    # the timed launches are the last `steps` ones (before them: the warmup and,
    # for I-NTMCP, the arena-calibration probe's small launches)
    b = bench_line(os.path.join(src, "bench_trace.log"))
    k = max(1, int(b.get("steps", 1)))
    # avg_ms: the TIMED launches only (the last `steps` dispatches of the kernel in
    # the kernel trace), not the warmup or an arena-calibration probe's launches
    durs = timed_launches(os.path.join(src, "trace", "run_kernel_trace.csv"), kernel)
    if len(durs) >= k:
        stats["avg_ms"] = sum(durs[-k:]) / k / 1e6
        stats["timed_launches"] = k
        stats["timed_ms"] = [d / 1e6 for d in durs[-k:]]
    else:   # no kernel trace kept (profiles before round 4): the all-calls average
        stats["avg_ms"] = stats["avg_ms_all_calls"]
        stats["timed_launches"] = None
    f_avg = sum(fetch[-k:]) / len(fetch[-k:])
    w_avg = sum(write[-k:]) / len(write[-k:])
    hbm = (2 * f_avg + w_avg) * 1024
    cfg = b["config"]
    summary = {
        "tag": tag, "bench": b, kernel: stats,
        "pmc": {"FETCH_SIZE_KiB_per_launch": f_avg, "WRITE_SIZE_KiB_per_launch": w_avg,
                "hbm_bytes_per_launch": hbm,
                "hbm_GBps": hbm / (stats["avg_ms"] * 1e-3) / 1e9,
                "alg_bytes_per_launch": b["roofline"]["alg_bytes_per_launch"]},
        "bench_kernel_ms_vs_rocprof_avg_ms": [b["roofline"]["kernel_ms"], stats["avg_ms"]],
    }
    with open(os.path.join(out, f"{tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    if current:
        with open(os.path.join(out, pmc_out), "w") as f:
            trees = cfg.get("trees_per_gpu", cfg.get("pairs"))
            sims = cfg.get("sims_per_tree", cfg.get("sims_per_level"))
            json.dump({"tag": tag, "trees": trees, "sims": sims,
                       "env": b["metric"].split(" on ")[1].split(" ")[0],
                       "hbm_bytes_per_launch": hbm,
                       # bench.py reports this traffic only for the same library
                       "lib_sha16": cfg.get("lib_sha16"),
                       "source": f"profiles/{tag}_summary.json"}, f, indent=1)
    print(json.dumps(summary["pmc"], indent=1), stats)


if __name__ == "__main__":
    main()
