#!/bin/bash
# Round-6 closing run (via gpurun): the GPU suite, smoke, the driver's bench
# command (headline + sub records), profiles of the headline and I-NTMCP lines
# (kernel trace + separate FETCH_SIZE / WRITE_SIZE passes) of the same library,
# the exact single tree's kernel trace and the C3 update()-inclusive step's
# kernel trace (k_compact_log).   usage: tools/sessions/closing_r6.sh TAG [skip-tests]
set -o pipefail
export TMPDIR=/tmp
T=$1
O=gpurun_out/m_$T
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
  tail -1 $O/gputest.log
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || { tail -30 $O/bench_driver_cmd.log; exit 1; }
python3 - $O/bench_driver_cmd.log <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        r = d["roofline"]
        print(f"headline {d['value']/1e9:.3f} G sims/s  ms/step {d['ms_per_step']:.1f}  kernel {r['kernel_ms']:.1f} ms  frac {r['frac']:.4f} frac_hbm {r.get('frac_hbm')}")
        for s in d.get("sub", []):
            print("  sub", json.dumps(s)[:400])
PY
bash tools/profile.sh $T --steps 3 --warmup 1 || exit 1
bash tools/profile.sh ${T}_intmcp --planner intmcp --steps 5 --warmup 1 || exit 1
P=gpurun_out/prof_${T}_b1; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 bench.py --trees 1 --sims 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $P/b1_trace.log 2>&1 || exit 1
find $P -type f ! -name '*kernel_stats.csv' ! -name '*.log' -delete
P=gpurun_out/prof_${T}_c3; mkdir -p $P
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $P/c3_trace.log 2>&1 || exit 1
find $P -type f ! -name '*kernel_stats.csv' ! -name '*.log' -delete
echo closing-done
