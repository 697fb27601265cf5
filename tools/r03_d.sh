#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/loss_err.py > gpurun_out/r03d_loss_err.json 2>&1 || { echo "loss_err failed"; tail -20 gpurun_out/r03d_loss_err.json; exit 1; }
grep -v amdgpu.ids gpurun_out/r03d_loss_err.json | head -40
bash tools/r03_ab.sh r03d3 base=langsplatv2_amd/_build/base_lib.so binpf=langsplatv2_amd/_build/var_binpf/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03d5 base=langsplatv2_amd/_build/base_lib.so binpf=langsplatv2_amd/_build/var_binpf/liblsr.so || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r03d_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03d_gpu_tests.log
