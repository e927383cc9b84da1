#!/bin/bash
# Round-4 profiles (via gpurun): headline k_search (trace + PMC), I-NTMCP (trace +
# PMC), and a kernel trace of the PursuitEvasion update()-inclusive step.
#   usage: tools/profile_r4.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=$1
bash tools/profile.sh ${T} --steps 3 --warmup 1 || exit 1
bash tools/profile.sh ${T}_intmcp --planner intmcp --steps 5 --warmup 1 || exit 1
O=gpurun_out/prof_${T}_pe; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --no-sub --steps 2 --warmup 1 --env PursuitEvasion-v1 --update-step --trees 32768 > $O/bench_trace.log 2>&1 || { tail -20 $O/bench_trace.log; exit 1; }
find $O -type f ! -name '*kernel_stats.csv' ! -name '*.log' -delete
echo all-done
