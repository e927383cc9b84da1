set -o pipefail
O=gpurun_out/s4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && \
bash tools/exp_variants.sh $O "65536 16384 variants/lib_s1_w1.so" "65536 16384 variants/lib_s0_w1.so" "65536 16384 variants/lib_s0_w2.so" "131072 8192 variants/lib_s0_w2.so" "131072 8192 variants/lib_s1_w1.so"
echo done $?
