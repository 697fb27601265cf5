#!/bin/bash
# bwd feature-row prefetch (FPF): GPU tests on the new build, then A/B against FPF=0 and the no-gather probe.
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03fpf_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r03fpf_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03fpf_gpu_tests.log
bash tools/r03_ab.sh r03fpf3 nofpf=$B/var_nofpf/liblsr.so fpf=langsplatv2_amd/liblsr.so nofeat=$B/var_nofeat/liblsr.so nopro=$B/var_nopro/liblsr.so || exit 1
echo done
