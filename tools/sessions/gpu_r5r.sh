#!/bin/bash
# Round 5: the exact single tree -- the next level's LDS line read issued as
# soon as the child is known (lpf) vs the in-tree library; wave parity on lpf.
set -o pipefail
O=gpurun_out/r5r; mkdir -p $O
for v in cur lpf cur lpf cur lpf; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  echo "== $v" >> $O/ab.log
  POMCP_LIB_PATH=$lib timeout -k 10 300 python bench.py --trees 1 --sims 65536 --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
done
grep -E "^==|^\{" $O/ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.strip()
    else:
        d=json.loads(l); r=d['roofline']; print(n, round(d['value']/1e3,1), 'k sims/s', round(r['kernel_ms'],2), 'ms')"
POMCP_LIB_PATH=$PWD/variants/lib_lpf.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "wave" --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity FAILED"; grep -E "FAILED|Error|assert" $O/parity.log | head -20; tail -30 $O/parity.log; exit 1; }
echo "parity: $(tail -1 $O/parity.log)"
echo done
