#!/bin/bash
# Round 5: I-NTMCP -- the child's statistics heads and the other agent's next
# history view not loaded at the level where the descent stops (A/B vs the
# in-tree library), then the I-NTMCP GPU tests on the variant.
set -o pipefail
O=gpurun_out/r5i; mkdir -p $O
for v in cur imv imv2 cur imv imv2; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  echo "== $v" >> $O/ab.log
  POMCP_LIB_PATH=$lib timeout -k 10 300 python bench.py --planner intmcp --no-cpu-baseline --no-sub --steps 5 --warmup 1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
done
grep -E "^==|^\{" $O/ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.strip()
    else:
        d=json.loads(l); r=d['roofline']; print(n, round(d['value']/1e9,4), 'G', round(r['kernel_ms'],3), 'ms', round(r['frac'],4))"
POMCP_LIB_PATH=$PWD/variants/lib_imv2.so timeout -k 10 900 python -u -m pytest tests/test_gpu_intmcp.py -x -q --timeout 300 --timeout-method thread > $O/intmcp.log 2>&1 || { echo "intmcp FAILED"; grep -E "FAILED|Error|assert" $O/intmcp.log | head -20; tail -30 $O/intmcp.log; exit 1; }
echo "intmcp: $(tail -1 $O/intmcp.log)"
echo done
