#!/bin/bash
# Round 5: the step-limit cut-off parity test on every search kernel.
set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_intmcp.py -x -v -k "step_limit" --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo "FAILED"; grep -E "FAILED|Error|assert" $O/parity.log | head -20; tail -30 $O/parity.log; exit 1; }
grep -E "PASSED|passed" $O/parity.log | tail -9
echo done
