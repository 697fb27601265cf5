#!/bin/bash
# D = 64 forward in the ML form (var_ml64) instead of k_render_fwd_mf: GPU tests on it, A/B vs the product build (cfg3 geometry at D = 64).
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
ROOT=$(pwd); OUT=$ROOT/gpurun_out
cp langsplatv2_amd/liblsr.so $B/prod.so && cp $B/var_ml64/liblsr.so langsplatv2_amd/liblsr.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r03ml64_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/r03ml64_gpu_tests.log; exit 1; }
tail -2 $OUT/r03ml64_gpu_tests.log
LSR_D=64 bash tools/r03_ab.sh r03ml643 prod=$B/prod.so ml64=$B/var_ml64/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03ml645 prod=$B/prod.so ml64=$B/var_ml64/liblsr.so || exit 1
echo done
