set -o pipefail
mkdir -p gpurun_out/st8
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_root_parallel.py -x -q --timeout 120 --timeout-method thread -k "wave or root" > gpurun_out/st8/parity.log 2>&1
echo rc=$?; tail -2 gpurun_out/st8/parity.log
for a in "1" "64" "256"; do
  timeout -k 10 200 python bench.py --trees $a --sims 65536 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/st8/b$a.log 2>&1 || exit 1
  echo b$a $(grep -h '^{' gpurun_out/st8/b$a.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), d['ms_per_step'])")
done
