#!/bin/bash
# Round-3 final measurements (run via gpurun): tools/measure_r3.sh (GPU suite,
# headline bench + CPU baseline, config 3, exact single tree, headline profile),
# then the single-root sweep and a kernel trace of the exact single tree.
# usage: tools/measure_r3j.sh TAG
set -o pipefail
T=$1
bash tools/measure_r3.sh $T && \
bash tools/single_root.sh sr_$T && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}_b1/trace -o run -- \
  python3 bench.py --trees 1 --sims 65536 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sr_$T/b1_trace.log 2>&1 && \
find gpurun_out/prof_${T}_b1 -type f ! -name '*kernel_stats.csv' -delete
