#!/bin/bash
# round-4 step b: parity of the deferred-record k_search (lane kernel) and the
# new GPU tests (base planner with fixed-distribution policies, every batched
# I-NTMCP pair, the exact softmax path), A/B against the eager lookup, then the
# default bench with its sub-records
set -o pipefail
O=gpurun_out/r4b; mkdir -p $O
export POMCP_LIB_PATH=$PWD/variants/lib_cur.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "lane" -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_mcts_policies.py tests/test_gpu_intmcp.py -q --timeout 300 --timeout-method thread > $O/test2.log 2>&1 || { tail -40 $O/test2.log; exit 1; }
tail -2 $O/test2.log
for n in eager cur eager cur; do
  echo "== $n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/exp.log 2>&1 || exit 1
done
python3 - $O/exp.log <<'PY'
import json, sys
name = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        name = line.split()[1]
    elif line.startswith("{"):
        d = json.loads(line)
        print(f"{name:8s} {d['value']/1e9:6.3f} G sims/s  kernel {d['roofline']['kernel_ms']:8.1f} ms frac {d['roofline']['frac']:.4f} deferred/sim {d['config'].get('deferred_levels_per_sim')}")
PY
unset POMCP_LIB_PATH
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_sub.log 2>&1 || { tail -30 $O/bench_sub.log; exit 1; }
tail -c 3000 $O/bench_sub.log
