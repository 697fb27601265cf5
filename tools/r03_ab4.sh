#!/bin/bash
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
LSR_LIB=$B/var_plds/liblsr.so timeout -k 10 600 python -u -m pytest tests/test_golden_fixtures.py tests/test_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ab4_tests.log 2>&1 || { echo "variant tests failed"; tail -30 gpurun_out/r03ab4_tests.log; exit 1; }
tail -1 gpurun_out/r03ab4_tests.log
bash tools/r03_ab.sh r03ab4 base=langsplatv2_amd/liblsr.so plds=$B/var_plds/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03ab4_5 base=langsplatv2_amd/liblsr.so plds=$B/var_plds/liblsr.so || exit 1
