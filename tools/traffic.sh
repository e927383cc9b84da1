#!/bin/bash
# HBM traffic of k_search for one bench configuration (run on the GPU box).
# usage: tools/traffic.sh TAG [bench args...]   -> gpurun_out/traffic_TAG/
TAG=${1:-x}; shift || true
export TMPDIR=/tmp
OUT=gpurun_out/traffic_$TAG
mkdir -p $OUT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o run -- python3 bench.py --no-cpu-baseline "$@" > $OUT/$C.log 2>&1 || { echo "pass $C failed"; exit 1; }
done
echo traffic-done
