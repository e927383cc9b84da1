#!/bin/bash
# Round-5 closing run (via gpurun): the GPU suite, smoke, the driver's bench
# command (headline + sub records), and profiles of the headline and I-NTMCP
# lines (kernel trace + separate FETCH_SIZE / WRITE_SIZE passes) of the same
# library, plus the exact single tree's kernel trace.
#   usage: tools/closing_r5.sh TAG [skip-tests]
set -o pipefail
export TMPDIR=/tmp
T=$1
bash tools/measure_r4.sh $T $2 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/m_$T/smoke.log 2>&1 || { tail -20 gpurun_out/m_$T/smoke.log; exit 1; }
tail -1 gpurun_out/m_$T/smoke.log
bash tools/profile.sh $T --steps 3 --warmup 1 || exit 1
bash tools/profile.sh ${T}_intmcp --planner intmcp --steps 5 --warmup 1 || exit 1
O=gpurun_out/prof_${T}_b1; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --trees 1 --sims 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/b1_trace.log 2>&1 || exit 1
find $O -type f ! -name '*kernel_stats.csv' ! -name '*.log' -delete
echo closing-done
