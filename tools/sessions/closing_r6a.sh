#!/bin/bash
# Round-6 closing run, part 1 (via gpurun): the whole GPU suite, smoke, and the
# driver's bench command (headline + sub records) with the final library.
#   usage: tools/sessions/closing_r6a.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=$1
O=gpurun_out/m_$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
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
echo closing-a-done
