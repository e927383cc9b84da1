#!/bin/bash
# Round-5 first GPU call: the GPU suite and the driver's bench line on the
# round-4 closing code (baseline for this round's A/Bs).
set -o pipefail
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests-failed; tail -30 $O/gpu_tests.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo bench-failed; tail -30 $O/bench.log; exit 1; }
tail -3 $O/gpu_tests.log
echo done
