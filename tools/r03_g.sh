#!/bin/bash
set -u
export TMPDIR=/tmp
LSR_CFG=5 bash tools/r03_ab.sh r03g5 box=langsplatv2_amd/liblsr.so || exit 1
bash tools/r03_ab.sh r03g3 box=langsplatv2_amd/liblsr.so || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03g_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r03g_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03g_gpu_tests.log
