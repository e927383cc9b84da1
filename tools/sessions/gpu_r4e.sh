#!/bin/bash
# round-4 step e: I-NTMCP search policies on the GPU; where the PursuitEvasion
# update()-inclusive step spends its time (kernel trace of the update kernels)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_intmcp.py -k "sp_ or nesting0" -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pe -o run -- python3 bench.py --no-cpu-baseline --no-sub --steps 2 --warmup 1 --env PursuitEvasion-v1 --update-step --trees 16384 > $O/pe_bench.log 2>&1 || { tail -20 $O/pe_bench.log; exit 1; }
find $O/pe -type f ! -name '*kernel_stats.csv' -delete
f=$(find $O/pe -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} total {float(r["TotalDurationNs"])/1e6:9.1f} ms avg {float(r["AverageNs"])/1e6:8.2f} ms')
PY
