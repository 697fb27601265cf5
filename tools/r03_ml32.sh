#!/bin/bash
# D = 32 forward with the language channels on MFMA (var_ml32): GPU tests on it, A/B vs the product build (cfg3, cfg5).
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
ROOT=$(pwd); OUT=$ROOT/gpurun_out
cp $B/var_ml32/liblsr.so /tmp/liblsr_prod_backup.so
cp langsplatv2_amd/liblsr.so $B/prod.so && cp $B/var_ml32/liblsr.so langsplatv2_amd/liblsr.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r03ml32_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/r03ml32_gpu_tests.log; exit 1; }
tail -2 $OUT/r03ml32_gpu_tests.log
bash tools/r03_ab.sh r03ml323 prod=$B/prod.so ml32=$B/var_ml32/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03ml325 prod=$B/prod.so ml32=$B/var_ml32/liblsr.so || exit 1
echo done
