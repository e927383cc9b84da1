set -o pipefail
mkdir -p gpurun_out/st3
timeout -k 10 120 python bench.py --trees 1 --sims 65536 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/st3/b1.log 2>&1 && \
timeout -k 10 120 python bench.py --trees 1 --sims 65536 --steps 2 --warmup 1 --no-cpu-baseline --env PursuitEvasion-v1 > gpurun_out/st3/b1_pe.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "wave" > gpurun_out/st3/parity.log 2>&1 && \
timeout -k 10 300 python tools/phase_timing.py --kernel wave --trees 1 --sims 65536 > gpurun_out/st3/pt.log 2>&1
echo rc=$?
tail -2 gpurun_out/st3/parity.log
grep -h '^{' gpurun_out/st3/b1*.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['value'], d['ms_per_step'])"
tail -16 gpurun_out/st3/pt.log
