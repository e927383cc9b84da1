#!/bin/bash
# Round 5: I-NTMCP nesting level 3 on the GPU -- the whole I-NTMCP GPU file
# (nesting 0-3 goldens, batched pairs, wall clock), then smoke.
set -o pipefail
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_intmcp.py -x -v --timeout 300 --timeout-method thread > $O/intmcp.log 2>&1 || { echo "intmcp FAILED"; grep -E "FAILED|Error|assert" $O/intmcp.log | head -20; tail -30 $O/intmcp.log; exit 1; }
tail -2 $O/intmcp.log
echo done
