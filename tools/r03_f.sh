#!/bin/bash
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
LSR_CFG=5 bash tools/r03_ab.sh r03f5 base=langsplatv2_amd/liblsr.so scprobe=$B/var_scprobe/liblsr.so cnt1=$B/var_cnt1/liblsr.so cnt2=$B/var_cnt2/liblsr.so aos=$B/var_aos/liblsr.so || exit 1
bash tools/r03_ab.sh r03f3 base=langsplatv2_amd/liblsr.so scprobe=$B/var_scprobe/liblsr.so cnt1=$B/var_cnt1/liblsr.so cnt2=$B/var_cnt2/liblsr.so aos=$B/var_aos/liblsr.so || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r03f_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03f_gpu_tests.log
bash tools/pmc_quick.sh r03 || exit 1
