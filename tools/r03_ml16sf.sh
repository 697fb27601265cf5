#!/bin/bash
# D = 16 forward in the ML form with gathered rows (var_ml16sf, LSR_FWD_SFEAT=16): GPU tests on it, A/B vs the product.
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
OUT=gpurun_out
cp langsplatv2_amd/liblsr.so $B/prod.so && cp $B/var_ml16sf/liblsr.so langsplatv2_amd/liblsr.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r03ml16sf_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/r03ml16sf_gpu_tests.log; exit 1; }
tail -2 $OUT/r03ml16sf_gpu_tests.log
bash tools/r03_ab.sh r03ml16sf3 prod=$B/prod.so ml16sf=$B/var_ml16sf/liblsr.so || exit 1
LSR_CFG=2 LSR_D=16 bash tools/r03_ab.sh r03ml16sf2 prod=$B/prod.so ml16sf=$B/var_ml16sf/liblsr.so || exit 1
echo done
