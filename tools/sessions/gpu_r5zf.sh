#!/bin/bash
# Round 5: k_compact_log computes a node's visits address only for the thread
# that adds the pass's count (vo) vs the closing library (c); GPU parity of vo.
set -o pipefail
O=gpurun_out/r5zf; mkdir -p $O
run() {  # variant env
  echo "== $2 $1" >> $O/ab.log
  POMCP_LIB_PATH=$PWD/variants/lib_$1.so timeout -k 10 300 python bench.py --env $2 --trees 32768 --update-step --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
}
for v in c vo c vo; do run $v PursuitEvasion-v1 || exit 1; done
for v in c vo; do run $v Driving-v1 || exit 1; done
grep -E "^==|^\{" $O/ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.strip()
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,4), 'G', round(d['ms_per_step'],1), 'ms/step', 'update', round(d.get('update_ms', 0), 1), 'search', round(d['roofline']['kernel_ms'], 1))"
POMCP_LIB_PATH=$PWD/variants/lib_vo.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_potmmcp.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity FAILED"; grep -E "FAILED|Error|assert" $O/parity.log | head -20; tail -30 $O/parity.log; exit 1; }
echo "parity vo: $(tail -1 $O/parity.log)"
echo done
