#!/bin/bash
# the lambda-free deferral of k_im_search's descent writes (variants/lib_pd.so):
# I-NTMCP GPU tests on it, then the I-NTMCP A/B against the shipped library
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/abi_pd
POMCP_LIB_PATH=$PWD/variants/lib_pd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_intmcp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/abi_pd/pd_test.log 2>&1 || { tail -30 gpurun_out/abi_pd/pd_test.log; exit 1; }
tail -1 gpurun_out/abi_pd/pd_test.log
bash tools/ab_im2.sh pd "" bq3 pd
