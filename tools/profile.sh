#!/bin/bash
# Profile a bench command on the GPU box (run via gpurun).
#   kernel trace + stats, then separate PMC passes for HBM bytes.
# usage: tools/profile.sh TAG [bench args...]  -> gpurun_out/prof_TAG/
set -e
TAG=${1:-r1}
shift || true
# --no-sub: only the named configuration's launches (the default bench run appends
# secondary-configuration records whose kernels would mix into the trace)
ARGS="--no-sub $@"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --no-cpu-baseline $ARGS > $OUT/bench_fetch.log 2>&1
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --no-cpu-baseline $ARGS > $OUT/bench_write.log 2>&1
# keep only what tools/summarize_profile.py reads (the merge-back limit is 64 MiB)
du -ab $OUT | sort -n | tail -8
find $OUT -type f ! -name '*kernel_stats.csv' ! -name '*counter_collection.csv' ! -name '*kernel_trace.csv' ! -name '*.log' -delete
# the kernel trace is kept for the search kernels only: tools/summarize_profile.py
# averages the TIMED launches (the last `steps`), not a calibration probe's
for f in $(find $OUT -name '*kernel_trace.csv'); do
  python3 - "$f" <<'PY'
import csv, sys
p = sys.argv[1]
rows = [r for r in csv.DictReader(open(p)) if any(k in r.get("Kernel_Name", "")
        for k in ("k_search", "k_im_search", "k_update", "k_compact", "k_extract", "k_reroot"))]
if rows:
    w = csv.DictWriter(open(p, "w"), fieldnames=list(rows[0].keys()))
    w.writeheader()
    w.writerows(rows)
PY
done
for f in $(find $OUT -name '*counter_collection.csv'); do
  python3 - "$f" <<'PY'
import csv, sys
p = sys.argv[1]
rows = [r for r in csv.DictReader(open(p)) if "k_" in r.get("Kernel_Name", "")]
if rows:
    w = csv.DictWriter(open(p, "w"), fieldnames=list(rows[0].keys()))
    w.writeheader()
    w.writerows(rows)
PY
done
du -sh $OUT
echo profile-done
