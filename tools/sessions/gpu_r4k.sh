#!/bin/bash
# round-4 step k: parity of the deferred log record (k_search) and the deferred
# descent writes (k_im_search); the I-NTMCP backup queue variant (imq); A/Bs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/abh_r4k
POMCP_LIB_PATH=$PWD/variants/lib_imq.so timeout -k 10 600 python -u -m pytest tests/test_gpu_intmcp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/abh_r4k/imq_test.log 2>&1 || { tail -30 gpurun_out/abh_r4k/imq_test.log; exit 1; }
tail -1 gpurun_out/abh_r4k/imq_test.log
bash tools/ab_head.sh r4k "test_gpu_parity and lane or test_gpu_root_parallel or potmmcp or mcts_policies or test_gpu_intmcp" bq3 lq2 || exit 1
bash tools/ab_im2.sh r4k "" bq3 lq2 imq
