#!/bin/bash
# Round 5: k_compact_log -- the deferred children's observation keys / flags
# computed at the flush (dense chunks) instead of during classification
# (A/B vs the in-tree library, update()-inclusive step, deferred), timing,
# deferral parity on the variant.
set -o pipefail
O=gpurun_out/r5k; mkdir -p $O
for env in PursuitEvasion-v1 Driving-v1; do
  for v in cur defk cur defk; do
    lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
    echo "== $env $v" >> $O/ab.log
    POMCP_LIB_PATH=$lib timeout -k 10 300 python bench.py --env $env --trees 32768 --update-step --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
  done
done
grep -E "^==|^\{" $O/ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.strip()
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,4), 'G', round(d['ms_per_step'],1), 'ms/step', 'update', round(d.get('update_ms', 0), 1), 'search', round(d['roofline']['kernel_ms'], 1))"
POMCP_LIB_PATH=$PWD/variants/lib_clogt2.so timeout -k 10 300 python tools/clog_timing.py --trees 32768 > $O/clogt_pe.txt 2>&1 || { tail -20 $O/clogt_pe.txt; exit 1; }
grep -v amdgpu.ids $O/clogt_pe.txt
POMCP_LIB_PATH=$PWD/variants/lib_defk.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "lane or reroot or batched or defer or compact or overflow or mode" --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity FAILED"; grep -E "FAILED|Error|assert" $O/parity.log | head -20; tail -30 $O/parity.log; exit 1; }
echo "parity: $(tail -1 $O/parity.log)"
echo done
