#!/bin/bash
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
LSR_LIB=$B/var_s1024r23/liblsr.so timeout -k 10 600 python -u -m pytest tests/test_golden_fixtures.py tests/test_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ab3_tests.log 2>&1 || { echo "stg tests failed"; tail -30 gpurun_out/r03ab3_tests.log; exit 1; }
tail -1 gpurun_out/r03ab3_tests.log
bash tools/r03_ab.sh r03ab3 base=langsplatv2_amd/liblsr.so s512r34=$B/var_s512r34/liblsr.so s512r23=$B/var_s512r23/liblsr.so s1024r23=$B/var_s1024r23/liblsr.so s1024r17=$B/var_s1024r17/liblsr.so || exit 1
