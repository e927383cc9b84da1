#!/bin/bash
# I-NTMCP A/B: bench --planner intmcp per library (GPU box, via gpurun).
# usage: tools/ab_im.sh TAG lib1.so lib2.so ...   (default library: "default")
set -o pipefail
O=gpurun_out/abim_$1; shift
mkdir -p $O
for lib in "$@"; do
  if [ "$lib" = default ]; then unset POMCP_LIB_PATH; else export POMCP_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 240 python bench.py --planner intmcp --no-cpu-baseline --steps 3 --warmup 1 ${IM_ARGS} > $O/run.json 2>$O/run.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/run.json')); print('%-28s %6.3f G sims/s  kernel %7.2f ms  frac %.3f' % (sys.argv[1], d['value']/1e9, d['roofline']['kernel_ms'], d['roofline']['frac']))" "$lib" | tee -a $O/summary.txt
done
