"""Per-simulation instruction mix of k_search (KERNEL=k_im_search: tools/pmc_im.sh) from tools/pmc.sh output.
usage: python tools/pmc_mix.py gpurun_out/pmc_TAG SIMS_TOTAL"""
import csv, glob, os, sys
from collections import defaultdict

d, sims = sys.argv[1], float(sys.argv[2])
tot = defaultdict(float)
for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if os.environ.get("KERNEL", "k_search") not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(tot):
    print(f"{k:24s} {tot[k]:16.4g}  per-sim {tot[k] / sims:10.2f}")
