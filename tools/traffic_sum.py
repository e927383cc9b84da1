"""HBM bytes per simulation of k_search from tools/traffic.sh output.
usage: python tools/traffic_sum.py gpurun_out/traffic_TAG SIMS_PER_LAUNCH"""
import csv, glob, os, sys

d, sims = sys.argv[1], float(sys.argv[2])
tot = {}
for name in ("FETCH_SIZE", "WRITE_SIZE"):
    v = []
    for f in glob.glob(os.path.join(d, name, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "k_search" in r["Kernel_Name"] and r["Counter_Name"] == name:
                v.append(float(r["Counter_Value"]))
    tot[name] = sum(v) / max(len(v), 1)   # per launch, KiB
hbm = (2 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024
print(f"per launch: fetch {2 * tot['FETCH_SIZE'] * 1024 / 1e9:.3f} GB  write "
      f"{tot['WRITE_SIZE'] * 1024 / 1e9:.3f} GB  -> {hbm / sims:.1f} B/sim")
