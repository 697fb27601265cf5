#!/bin/bash
# ML forward for every D > 16 (old 16-group MFMA forward removed): GPU tests incl. D = 24 / 48, then cfg3 (D = 16, 64) and cfg5 stage times.
set -u
export TMPDIR=/tmp
ROOT=$(pwd); OUT=$ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r03mlx_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/r03mlx_gpu_tests.log; exit 1; }
tail -2 $OUT/r03mlx_gpu_tests.log
bash tools/r03_ab.sh r03mlx3 prod=langsplatv2_amd/liblsr.so || exit 1
LSR_D=64 bash tools/r03_ab.sh r03mlx364 prod=langsplatv2_amd/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03mlx5 prod=langsplatv2_amd/liblsr.so || exit 1
echo done
