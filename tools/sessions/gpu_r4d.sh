#!/bin/bash
# round-4 step d: the fast UCB scores (k_search) and the workgroup-per-log
# update kernels (k_extract, k_compact_log): parity (lane kernel, root-parallel,
# the reciprocal error bound), A/B against the previous library, and the
# update()-inclusive PursuitEvasion step
set -o pipefail
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_intmcp.py tests/test_gpu_parity.py tests/test_gpu_potmmcp.py tests/test_gpu_mcts_policies.py -k "intmcp or lane or potmmcp or base_planner" -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
for n in exact upd exact upd; do
  echo "== $n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/exp.log 2>&1 || exit 1
done
for n in upd; do
  echo "== pe_$n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub --steps 2 --warmup 1 --env PursuitEvasion-v1 --update-step --trees 16384 >> $O/exp.log 2>&1 || exit 1
done
for n in exact upd exact upd; do
  echo "== im_$n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --planner intmcp --steps 3 --warmup 1 >> $O/exp.log 2>&1 || exit 1
done
python3 - $O/exp.log <<'PY'
import json, sys
name = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        name = line.split()[1]
    elif line.startswith("{"):
        d = json.loads(line)
        print(f"{name:8s} {d['value']/1e9:6.3f} G sims/s  kernel {d['roofline']['kernel_ms']:8.1f} ms frac {d['roofline']['frac']:.4f} update_ms {d.get('update_ms')}")
PY
