#!/bin/bash
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
timeout -k 10 60 ./tools/micro/dpp_xor > gpurun_out/r03ac_dpp.txt 2>&1; rc=$?; cat gpurun_out/r03ac_dpp.txt; [ $rc -eq 0 ] || { echo "dpp check failed rc=$rc"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03ac_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r03ac_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03ac_gpu_tests.log
bash tools/r03_ab.sh r03ac3 prev=$B/var_prev/liblsr.so fused=langsplatv2_amd/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03ac5 prev=$B/var_prev/liblsr.so fused=langsplatv2_amd/liblsr.so || exit 1
echo done
