#!/bin/bash
# Round-3 measurements (run via gpurun): the GPU suite, the headline bench
# (with the CPU baseline), config 3, the exact single tree, then the rocprof
# profile of the headline (kernel trace + FETCH_SIZE / WRITE_SIZE passes).
# usage: tools/measure_r3.sh TAG      -> gpurun_out/m_TAG/, gpurun_out/prof_TAG/
set -o pipefail
T=$1
O=gpurun_out/m_$T
mkdir -p $O
B="timeout -k 10 400 python bench.py"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 && \
tail -1 $O/gputest.log && \
$B > $O/bench.log 2>&1 && \
$B --env PursuitEvasion-v1 --no-cpu-baseline > $O/bench_pe.log 2>&1 && \
$B --trees 1 --sims 65536 --steps 2 --no-cpu-baseline > $O/bench_b1.log 2>&1 && \
bash tools/profile.sh $T
