#!/bin/bash
# Round 5: root-belief extraction fused into k_compact_log (in-tree library)
# vs the separate k_extract scan (variants/lib_lw16.so = the previous library):
# GPU parity first, then the update()-inclusive steps.
set -o pipefail
O=gpurun_out/r5y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_potmmcp.py tests/test_gpu_mcts_policies.py tests/test_gpu_root_parallel.py tests/test_step_tree_invariant.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity FAILED"; grep -E "FAILED|Error|assert" $O/parity.log | head -20; tail -30 $O/parity.log; exit 1; }
echo "parity: $(tail -1 $O/parity.log)"
run() {  # variant env
  lib=""; [ $1 != cur ] && lib=$PWD/variants/lib_$1.so
  echo "== $2 $1" >> $O/ab.log
  POMCP_LIB_PATH=$lib timeout -k 10 300 python bench.py --env $2 --trees 32768 --update-step --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
}
for v in cur lw16 cur lw16; do run $v PursuitEvasion-v1 || exit 1; done
for v in cur lw16; do run $v Driving-v1 || exit 1; done
grep -E "^==|^\{" $O/ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.strip()
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,4), 'G', round(d['ms_per_step'],1), 'ms/step', 'update', round(d.get('update_ms', 0), 1), 'search', round(d['roofline']['kernel_ms'], 1))"
echo done
