set -o pipefail
mkdir -p gpurun_out/st6
for r in 1 2; do
timeout -k 10 120 python bench.py --trees 1 --sims 65536 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/st6/b1.log 2>&1 || exit 1
echo b1 $(grep -h '^{' gpurun_out/st6/b1.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), d['ms_per_step'])")
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "wave" > gpurun_out/st6/parity.log 2>&1
echo rc=$?
tail -2 gpurun_out/st6/parity.log
