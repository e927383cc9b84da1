#!/bin/bash
# Round 5: the final library on the other BASELINE-named workloads (search only):
# PursuitEvasion-v1 (config 3), the deep configuration, POTMMCP.
set -o pipefail
O=gpurun_out/r5u; mkdir -p $O
timeout -k 10 400 python bench.py --env PursuitEvasion-v1 --no-sub --steps 5 --warmup 1 > $O/pe.log 2>&1 || { tail -20 $O/pe.log; exit 1; }
timeout -k 10 400 python bench.py --planner potmmcp --no-sub --no-cpu-baseline --steps 3 --warmup 1 > $O/potmmcp.log 2>&1 || { tail -20 $O/potmmcp.log; exit 1; }
for f in pe potmmcp; do
  python3 - $O/$f.log <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); r = d["roofline"]
        print(sys.argv[1].split("/")[-1], f"{d['value']/1e9:.3f} G sims/s", f"{d['ms_per_step']:.1f} ms/step", f"kernel {r['kernel_ms']:.1f} ms", f"frac {r['frac']:.4f}", "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
done
echo done
