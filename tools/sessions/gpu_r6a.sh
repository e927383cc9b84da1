#!/bin/bash
# Round-6 first GPU call: the full-size re-root parity test (all search-kernel
# modes), the whole GPU suite on the two-ended belief region (ABI 7), the C3
# footprint probe and the C3 update()-inclusive step at 65,536 roots.
set -o pipefail
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k full_size_reroot --timeout 300 --timeout-method thread > $O/fullsize.log 2>&1 || { echo tests-failed; tail -40 $O/fullsize.log; exit 1; }
tail -14 $O/fullsize.log
timeout -k 10 300 python -u tools/c3_footprint.py > $O/footprint.log 2>&1 || { echo probe-failed; tail -30 $O/footprint.log; exit 1; }
cat $O/footprint.log
timeout -k 10 300 python -u bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/c3.log 2>&1 || { echo c3-failed; tail -30 $O/c3.log; exit 1; }
tail -c 1500 $O/c3.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo suite-failed; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
echo done
