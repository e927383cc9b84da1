#!/bin/bash
# the register-trimmed backup queue (variants/lib_qt.so): lane parity on it,
# then the headline A/B against the shipped library
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/abh_qt
POMCP_LIB_PATH=$PWD/variants/lib_qt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_root_parallel.py -x -q -k "lane or root" --timeout 300 --timeout-method thread > gpurun_out/abh_qt/qt_test.log 2>&1 || { tail -30 gpurun_out/abh_qt/qt_test.log; exit 1; }
tail -1 gpurun_out/abh_qt/qt_test.log
bash tools/ab_head.sh qt "" bq3 qt
