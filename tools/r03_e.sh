#!/bin/bash
set -u
export TMPDIR=/tmp
bash tools/r03_ab.sh r03e3 lpt=langsplatv2_amd/liblsr.so nolpt=langsplatv2_amd/_build/var_nolpt/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03e5 lpt=langsplatv2_amd/liblsr.so nolpt=langsplatv2_amd/_build/var_nolpt/liblsr.so || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r03e_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03e_gpu_tests.log
