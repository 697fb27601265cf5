#!/bin/bash
# Round-5 (session 3): 16-tile table-scan groups: the GPU suite, then one-process A/B
# against the previous build at cfg3, cfg5 and the quick path.
set -u
OUT=gpurun_out; mkdir -p $OUT
bash tools/r05_pass.sh r05s3j "tests" || exit 1
grep -q " failed" $OUT/r05s3j_tests.log && { echo "tests failed"; exit 1; }
for C in 3 5; do
  LSR_CFG=$C timeout -k 10 400 python tools/ab.py prev=langsplatv2_amd/_build/var_prev/liblsr.so tbl16=langsplatv2_amd/liblsr.so > $OUT/r05s3_ab_tbl16_cfg$C.txt 2>&1 || { echo "ab cfg$C failed"; tail -20 $OUT/r05s3_ab_tbl16_cfg$C.txt; exit 1; }
  cat $OUT/r05s3_ab_tbl16_cfg$C.txt
done
LSR_AB_LAYOUT=hwc timeout -k 10 300 python tools/ab_quick.py prev=langsplatv2_amd/_build/var_prev/liblsr.so tbl16=langsplatv2_amd/liblsr.so > $OUT/r05s3_ab_tbl16_quick.txt 2>&1 || { echo "ab_quick failed"; tail -20 $OUT/r05s3_ab_tbl16_quick.txt; exit 1; }
cat $OUT/r05s3_ab_tbl16_quick.txt
echo done
