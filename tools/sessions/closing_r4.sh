#!/bin/bash
# Round-4 closing run (via gpurun): the GPU suite, the driver's bench command
# (headline + sub records), and profiles of the headline and I-NTMCP lines
# (kernel trace + separate FETCH_SIZE / WRITE_SIZE passes) of the same library.
#   usage: tools/closing_r4.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=$1
bash tools/measure_r4.sh $T || exit 1
bash tools/profile.sh $T --steps 3 --warmup 1 || exit 1
bash tools/profile.sh ${T}_intmcp --planner intmcp --steps 5 --warmup 1 || exit 1
O=gpurun_out/prof_${T}_b1; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --trees 1 --sims 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/b1_trace.log 2>&1 || exit 1
find $O -type f ! -name '*kernel_stats.csv' ! -name '*.log' -delete
echo closing-done
