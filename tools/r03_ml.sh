#!/bin/bash
# D = 16 forward with the language channels on MFMA (ML, the product build): GPU tests, A/B vs LSR_FWD_ML=0 (cfg3, 1 Mpix forward).
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
ROOT=$(pwd); OUT=$ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r03ml_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/r03ml_gpu_tests.log; exit 1; }
tail -2 $OUT/r03ml_gpu_tests.log
bash tools/r03_ab.sh r03ml3 noml=$B/var_noml/liblsr.so ml=langsplatv2_amd/liblsr.so || exit 1
LSR_CFG=2 LSR_D=16 bash tools/r03_ab.sh r03ml2 noml=$B/var_noml/liblsr.so ml=langsplatv2_amd/liblsr.so || exit 1
echo done
