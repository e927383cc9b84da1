#!/bin/bash
# Profile the default bench command on the GPU box (run via gpurun).
#   kernel trace + stats, then separate PMC passes for HBM bytes.
set -e
TAG=${1:-r1}
shift || true
ARGS="$@"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --no-cpu-baseline $ARGS > $OUT/bench_fetch.log 2>&1
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --no-cpu-baseline $ARGS > $OUT/bench_write.log 2>&1
echo profile-done
