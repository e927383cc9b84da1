set -o pipefail
mkdir -p gpurun_out/st1
timeout -k 10 120 python bench.py --trees 1 --sims 65536 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/st1/b1_spec.log 2>&1 && \
POMCP_STEP_TREE=0 timeout -k 10 120 python bench.py --trees 1 --sims 65536 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/st1/b1_plain.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k wave > gpurun_out/st1/parity.log 2>&1
echo rc=$?
tail -3 gpurun_out/st1/parity.log
grep -h '^{' gpurun_out/st1/b1_*.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['value'], d['ms_per_step'])"
