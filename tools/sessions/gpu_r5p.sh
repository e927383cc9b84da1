#!/bin/bash
# Round 5: k_compact_log with its compaction-map lookups pipelined one pass
# ahead (records two passes ahead): A/B of the update()-inclusive step, then
# the parity tests that re-root (both deferral modes) on the variant.
set -o pipefail
O=gpurun_out/r5p; mkdir -p $O
for env in PursuitEvasion-v1 Driving-v1; do
  for vd in cur:on pipe:on cur:off pipe:off cur:on pipe:on; do
    v=${vd%%:*}; d=${vd#*:}
    lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
    echo "== $env $v defer=$d" >> $O/ab.log
    POMCP_LIB_PATH=$lib timeout -k 10 300 python bench.py --env $env --trees 32768 --update-step --defer $d --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
  done
done
grep -E "^==|^\{" $O/ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.strip()
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,4), 'G', round(d['ms_per_step'],1), 'ms/step', 'update', round(d.get('update_ms', 0), 1), 'search', round(d['roofline']['kernel_ms'], 1))"
POMCP_LIB_PATH=$PWD/variants/lib_pipe.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_root_parallel.py tests/test_gpu_potmmcp.py -x -q -k "lane or reroot or batched or defer or compact or overflow or mode or step_limit or episode or potmmcp" --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity FAILED"; grep -E "FAILED|Error|assert" $O/parity.log | head -20; tail -30 $O/parity.log; exit 1; }
echo "parity: $(tail -1 $O/parity.log)"
echo done
