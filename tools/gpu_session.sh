set -o pipefail
mkdir -p gpurun_out/s3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/s3/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/s3/bench.log 2>&1 && \
timeout -k 10 200 python tools/phase_timing.py > gpurun_out/s3/phase.log 2>&1
echo done $?
