#!/bin/bash
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
# parity of the staged-scatter variant first (binning lists vs the oracle, bit-exact), then timing
LSR_LIB=$B/var_stg/liblsr.so timeout -k 10 600 python -u -m pytest tests/test_golden_fixtures.py tests/test_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03aa_tests.log 2>&1 || { echo "stg tests failed"; tail -30 gpurun_out/r03aa_tests.log; exit 1; }
tail -2 gpurun_out/r03aa_tests.log
bash tools/r03_ab.sh r03aa3 base=langsplatv2_amd/liblsr.so stg=$B/var_stg/liblsr.so || exit 1
echo done
