#!/bin/bash
# scalar-feature forward with RGB staged in LDS (product) vs scalar RGB loads (rgb0): GPU tests, A/B cfg5 and D = 64.
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
OUT=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r03rgb_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/r03rgb_gpu_tests.log; exit 1; }
tail -2 $OUT/r03rgb_gpu_tests.log
LSR_CFG=5 bash tools/r03_ab.sh r03rgb5 rgb0=$B/var_rgb0/liblsr.so rgb=langsplatv2_amd/liblsr.so || exit 1
LSR_D=64 bash tools/r03_ab.sh r03rgb364 rgb0=$B/var_rgb0/liblsr.so rgb=langsplatv2_amd/liblsr.so || exit 1
echo done
