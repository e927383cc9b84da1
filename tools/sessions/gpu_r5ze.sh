#!/bin/bash
# Round 5 closing library: per-kernel times of the update()-inclusive
# PursuitEvasion and Driving steps (rocprofv3 --kernel-trace --stats).
set -o pipefail
O=gpurun_out/r5ze; mkdir -p $O
export TMPDIR=/tmp
for e in PursuitEvasion-v1 Driving-v1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$e -o run -- python3 bench.py --env $e --trees 32768 --update-step --no-cpu-baseline --no-sub --steps 3 --warmup 1 > $O/bench_$e.log 2>&1 || { tail -20 $O/bench_$e.log; exit 1; }
  f=$(find $O/prof_$e -name "*kernel_stats.csv" | head -1); cp $f $O/${e}_kernel_stats.csv; cut -c1-150 $f | head -8
done
find $O -type f ! -name '*kernel_stats.csv' ! -name '*.log' -delete
echo done
