#!/bin/bash
# Round 5: (1) I-NTMCP nesting 0-3 GPU file; (2) deferral parity with bulk
# materialisation of deferred children (k_compact_log queue); (3) A/B of the
# update()-inclusive PursuitEvasion / Driving step, deferred vs eager, old vs new.
set -o pipefail
O=gpurun_out/r5g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_intmcp.py -x -q --timeout 300 --timeout-method thread > $O/intmcp.log 2>&1 || { echo "intmcp FAILED"; grep -E "FAILED|Error|assert" $O/intmcp.log | head -20; tail -30 $O/intmcp.log; exit 1; }
echo "intmcp: $(tail -1 $O/intmcp.log)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity FAILED"; grep -E "FAILED|Error|assert" $O/parity.log | head -20; tail -30 $O/parity.log; exit 1; }
echo "parity: $(tail -1 $O/parity.log)"
for env in PursuitEvasion-v1 Driving-v1; do
  for v in base new; do
    for d in on off; do
      lib=""; [ $v = base ] && lib=$PWD/variants/lib_base.so
      echo "== $env $v defer=$d" >> $O/ab.log
      POMCP_LIB_PATH=$lib timeout -k 10 300 python bench.py --env $env --trees 32768 --update-step --defer $d --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
    done
  done
done
grep -E "^==|^\{" $O/ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.strip()
    else:
        d=json.loads(l); c=d['config']; print(n, round(d['value']/1e9,4), 'G', round(d['ms_per_step'],1), 'ms/step', 'update', round(d.get('update_ms', 0), 1), 'search', round(d['roofline']['kernel_ms'], 1))"
echo done
