#!/bin/bash
# Round 5: kernel trace of the update()-inclusive PursuitEvasion step (which
# update kernels the 143 ms are).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5l; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --env PursuitEvasion-v1 --trees 32768 --update-step --no-cpu-baseline --no-sub --steps 3 --warmup 1 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
find $O -type f ! -name '*kernel_stats.csv' ! -name '*.log' -delete
f=$(find $O -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.1f} ms total  {int(r["Calls"]):5d} calls  {float(r["AverageNs"])/1e6:9.3f} ms avg  {r["Name"][:90]}')
PY
echo done
