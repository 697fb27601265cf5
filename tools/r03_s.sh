#!/bin/bash
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03s_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r03s_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03s_gpu_tests.log
bash tools/r03_ab.sh r03s3 prev=$B/var_prev/liblsr.so fused=langsplatv2_amd/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03s5 prev=$B/var_prev/liblsr.so fused=langsplatv2_amd/liblsr.so || exit 1
LSR_CFG=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03s_prof5 -o run -- python -u tools/ab.py fused=langsplatv2_amd/liblsr.so > gpurun_out/r03s_prof5.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r03s_prof5.log; exit 1; }
echo done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03s_prof3 -o run -- python -u tools/ab.py fused=langsplatv2_amd/liblsr.so > gpurun_out/r03s_prof3.log 2>&1 || { echo "prof3 failed"; tail -20 gpurun_out/r03s_prof3.log; exit 1; }
python tools/rocpd_stats.py gpurun_out/r03s_prof5/run_results.db 12 > gpurun_out/r03s_prof5.txt
python tools/rocpd_stats.py gpurun_out/r03s_prof3/run_results.db 20 > gpurun_out/r03s_prof3.txt
