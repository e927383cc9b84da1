#!/bin/bash
# Round 5: per-kernel times of the update()-inclusive PursuitEvasion step with
# the 16-wave log kernels (in-tree library).
set -o pipefail
O=gpurun_out/r5x; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o pe -- python3 bench.py --env PursuitEvasion-v1 --trees 32768 --update-step --no-cpu-baseline --no-sub --steps 3 --warmup 1 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cut -c1-150 $f | head -14
echo done
