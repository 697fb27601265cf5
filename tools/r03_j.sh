#!/bin/bash
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03j_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r03j_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03j_gpu_tests.log
bash tools/r03_ab.sh r03j3 prev=$B/var_prev/liblsr.so fused=langsplatv2_amd/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03j5 prev=$B/var_prev/liblsr.so fused=langsplatv2_amd/liblsr.so || exit 1
