#!/bin/bash
# SQ counter passes for k_im_search (run on the GPU box via gpurun).
# usage: tools/pmc_im.sh TAG [bench args...]
TAG=${1:-x}; shift || true
ARGS="$@"
export TMPDIR=/tmp
OUT=gpurun_out/pmcim_$TAG
mkdir -p $OUT
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 bench.py --planner intmcp --no-cpu-baseline $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed"; exit 1; }
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH
run p2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS
# keep only the counter summaries of the search kernel (gpurun merges <= 64 MiB back)
find $OUT -type f ! -name '*counter_collection.csv' ! -name '*.log' -delete
for f in $(find $OUT -name '*counter_collection.csv'); do
  python3 - "$f" <<'PY'
import csv, sys
p = sys.argv[1]
rows = [r for r in csv.DictReader(open(p)) if "k_im_search" in r.get("Kernel_Name", "")]
w = csv.DictWriter(open(p, "w"), fieldnames=list(rows[0].keys()) if rows else ["Kernel_Name"])
w.writeheader()
w.writerows(rows)
PY
done
du -sh $OUT
echo pmc-done
