#!/bin/bash
# Round 5: the GPU suite (new: launcher, exact-select fallback, PE deferred
# re-root, mode guard, step_statistics) and the bench line with the byte count
# of only the work k_search does.
set -o pipefail
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests-failed; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo bench-failed; tail -30 $O/bench.log; exit 1; }
echo done
