#!/bin/bash
# Round-6 closing run, part 3 (via gpurun): the driver's bench command with the
# final library, then the re-root kernels' counters (pmc_update.sh).
#   usage: tools/sessions/closing_r6c.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=$1
O=gpurun_out/m_$T
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || { tail -30 $O/bench_driver_cmd.log; exit 1; }
python3 - $O/bench_driver_cmd.log <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        r = d["roofline"]
        print(f"headline {d['value']/1e9:.3f} G sims/s  ms/step {d['ms_per_step']:.1f}  kernel {r['kernel_ms']:.1f} ms  frac {r['frac']:.4f} traffic {r['traffic']}")
        for s in d.get("sub", []):
            print("  sub", s["name"][:60], round(s["value"] / 1e9, 4), s.get("update_ms"), s.get("frac"), s.get("traffic"))
PY
bash tools/sessions/pmc_update.sh $T || exit 1
echo closing-c-done
