#!/bin/bash
# Round-3 closing run (via gpurun): the GPU suite, the driver's own bench command,
# and a kernel trace of the exact single tree.  usage: tools/measure_r3k.sh TAG
set -o pipefail
T=$1
O=gpurun_out/m_$T
mkdir -p $O gpurun_out/prof_${T}_b1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 && \
tail -1 $O/gputest.log && \
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}_b1/trace -o run -- \
  python3 bench.py --trees 1 --sims 65536 --steps 3 --warmup 1 --no-cpu-baseline > $O/b1_trace.log 2>&1 && \
find gpurun_out/prof_${T}_b1 -type f ! -name '*kernel_stats.csv' -delete
