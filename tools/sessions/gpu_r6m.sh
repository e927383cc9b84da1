#!/bin/bash
# Round 6, call m: the compaction parity test in all three re-root scans, then
# the closing profiles of the final library (closing_r6b.sh).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6m; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "forced_small_arena" --timeout 300 --timeout-method thread > $O/scan_modes.log 2>&1 || { echo scan-modes-failed; tail -40 $O/scan_modes.log; exit 1; }
grep -E "PASSED|FAILED" $O/scan_modes.log
bash tools/sessions/closing_r6b.sh r6z || exit 1
