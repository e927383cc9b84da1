# I-NTMCP layout variants: parity tests + bench per library (run via gpurun)
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
for lib in "$@"; do
  echo "== $lib" >> $O/exp.log
  POMCP_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_intmcp.py -m gpu -x -q --timeout 200 --timeout-method thread >> $O/exp.log 2>&1 || exit 1
  POMCP_LIB_PATH=$lib timeout -k 10 300 python bench.py --planner intmcp --no-cpu-baseline --steps 2 >> $O/exp.log 2>&1 || exit 1
done
