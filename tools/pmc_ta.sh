#!/bin/bash
# Vector-memory pipeline counters (TA / TD / TCP) for a kernel of bench.py
# (GPU box, via gpurun).  usage: tools/pmc_ta.sh TAG KERNEL [bench args...]
TAG=$1; KERNEL=$2; shift 2
export TMPDIR=/tmp
OUT=gpurun_out/pmcta_$TAG
mkdir -p $OUT
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 bench.py --no-cpu-baseline $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed"; exit 1; }
}
ARGS="$@"
run t1 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT
run t2 TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum
run t3 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum
find $OUT -type f ! -name '*counter_collection.csv' ! -name '*.log' -delete
python3 - $OUT $KERNEL <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d, kern = sys.argv[1], sys.argv[2]
tot, n = defaultdict(float), defaultdict(int)
for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")) + glob.glob(os.path.join(d, "*", "*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:40s} {tot[k] / max(n[k], 1):16.5g} per launch ({n[k]} rows)")
PY
