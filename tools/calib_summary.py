"""Counted bytes per access for each randrw kernel (tools/calib_fetch.sh)."""
import csv
import glob
import os
import sys

LANES, ITERS = 65536, 2000
d = sys.argv[1]
rows = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(d, c, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != c:
                continue
            key = (r["Kernel_Name"], int(r.get("Dispatch_Id", 0) or 0))
            rows.setdefault(key, {})[c] = float(r["Counter_Value"])
out = []
for (name, did), v in sorted(rows.items(), key=lambda x: x[0][1]):
    out.append((name, did, v.get("FETCH_SIZE"), v.get("WRITE_SIZE")))
# each run() launches a 50-iteration warm-up then the 2000-iteration launch;
# FETCH_SIZE / WRITE_SIZE are in KiB
for name, did, fe, wr in out:
    acc = LANES * ITERS
    f = "-" if fe is None else f"{fe * 1024 / acc:7.2f}"
    w = "-" if wr is None else f"{wr * 1024 / acc:7.2f}"
    print(f"{did:4d} {name[:60]:60s} FETCH B/access {f}  WRITE B/access {w}")
