#!/bin/bash
# Round-5 (session 3): split preprocess (SH colour pass on a second stream):
# its tests, then one-process A/B fused vs split at cfg3 / cfg5 / cfg2.
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_split_preprocess.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/r05s3_split_tests.log 2>&1 || { echo "split tests failed"; tail -30 $OUT/r05s3_split_tests.log; exit 1; }
tail -2 $OUT/r05s3_split_tests.log
for C in 3 5 2; do
  LSR_CFG=$C timeout -k 10 400 python tools/ab.py fused=langsplatv2_amd/liblsr.so#split0 split=langsplatv2_amd/liblsr.so > $OUT/r05s3_ab_split_cfg$C.txt 2>&1 || { echo "ab cfg$C failed"; tail -20 $OUT/r05s3_ab_split_cfg$C.txt; exit 1; }
  cat $OUT/r05s3_ab_split_cfg$C.txt
done
echo done
