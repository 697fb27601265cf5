#!/bin/bash
# Round-5 (session 3): speculative scatter: its tests, the GPU suite, then
# one-process step A/B against the previous build at cfg3, cfg2 and cfg5.
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_spec_scatter.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/r05s3_spec_tests.log 2>&1 || { echo "spec tests failed"; tail -30 $OUT/r05s3_spec_tests.log; exit 1; }
tail -2 $OUT/r05s3_spec_tests.log
bash tools/r05_pass.sh r05s3b "tests" || exit 1
for C in 3 2 5; do
  LSR_CFG=$C timeout -k 10 400 python tools/ab.py prev=langsplatv2_amd/_build/var_prev/liblsr.so spec=langsplatv2_amd/liblsr.so > $OUT/r05s3_ab_spec_cfg$C.txt 2>&1 || { echo "ab cfg$C failed"; tail -20 $OUT/r05s3_ab_spec_cfg$C.txt; exit 1; }
  cat $OUT/r05s3_ab_spec_cfg$C.txt
done
echo done
