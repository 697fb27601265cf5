#!/bin/bash
# Round-5 (session 3): 68-row count bands below 4M Gaussians: the GPU suite, then
# one-process A/B against the previous build at cfg3, cfg2 and the quick path.
set -u
OUT=gpurun_out; mkdir -p $OUT
bash tools/r05_pass.sh r05s3f "tests" || exit 1
for C in 3 2; do
  LSR_CFG=$C timeout -k 10 400 python tools/ab.py prev=langsplatv2_amd/_build/var_prev/liblsr.so new=langsplatv2_amd/liblsr.so > $OUT/r05s3_ab_bands68_cfg$C.txt 2>&1 || { echo "ab cfg$C failed"; tail -20 $OUT/r05s3_ab_bands68_cfg$C.txt; exit 1; }
  cat $OUT/r05s3_ab_bands68_cfg$C.txt
done
LSR_AB_LAYOUT=hwc timeout -k 10 300 python tools/ab_quick.py prev=langsplatv2_amd/_build/var_prev/liblsr.so new=langsplatv2_amd/liblsr.so > $OUT/r05s3_ab_bands68_quick.txt 2>&1 || { echo "ab_quick failed"; tail -20 $OUT/r05s3_ab_bands68_quick.txt; exit 1; }
cat $OUT/r05s3_ab_bands68_quick.txt
echo done
