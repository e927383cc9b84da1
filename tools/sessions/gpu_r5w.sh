#!/bin/bash
# Round 5: waves per workgroup of k_extract / k_compact_log (2 / 4 / 8 / 16;
# the same 4 records per thread per pass) on the update()-inclusive step.
set -o pipefail
O=gpurun_out/r5w; mkdir -p $O
run() {  # variant env
  lib=""; [ $1 != cur ] && lib=$PWD/variants/lib_$1.so
  echo "== $2 $1" >> $O/ab.log
  POMCP_LIB_PATH=$lib timeout -k 10 300 python bench.py --env $2 --trees 32768 --update-step --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
}
for v in cur lw8 lw16 lw2 cur lw8 lw16 lw2; do run $v PursuitEvasion-v1 || exit 1; done
for v in cur lw8 lw16 cur lw8 lw16; do run $v Driving-v1 || exit 1; done
grep -E "^==|^\{" $O/ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.strip()
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,4), 'G', round(d['ms_per_step'],1), 'ms/step', 'update', round(d.get('update_ms', 0), 1), 'search', round(d['roofline']['kernel_ms'], 1))"
for v in lw8 lw16; do
  POMCP_LIB_PATH=$PWD/variants/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "lane or batched or reroot" --timeout 300 --timeout-method thread > $O/parity_$v.log 2>&1 || { echo "parity $v FAILED"; grep -E "FAILED|Error|assert" $O/parity_$v.log | head -20; tail -30 $O/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $O/parity_$v.log)"
done
echo done
