#!/bin/bash
# Round-6 closing run, part 2 (via gpurun): profiles of the final library -- the
# headline and I-NTMCP lines (kernel trace + separate FETCH_SIZE / WRITE_SIZE
# passes), the exact single tree's and the C3 update()-inclusive step's kernel
# traces (the re-root kernels' counters: tools/sessions/pmc_update.sh).   usage: tools/sessions/closing_r6b.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=$1
bash tools/profile.sh $T --steps 3 --warmup 1 || exit 1
bash tools/profile.sh ${T}_intmcp --planner intmcp --steps 5 --warmup 1 || exit 1
P=gpurun_out/prof_${T}_b1; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 bench.py --trees 1 --sims 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $P/b1_trace.log 2>&1 || exit 1
find $P -type f ! -name '*kernel_stats.csv' ! -name '*.log' -delete
P=gpurun_out/prof_${T}_c3; mkdir -p $P
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $P/c3_trace.log 2>&1 || exit 1
find $P -type f ! -name '*kernel_stats.csv' ! -name '*.log' -delete
echo closing-b-done
