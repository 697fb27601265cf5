#!/bin/bash
# Round-5 (session 3): quick-path checks and A/Bs on one box: the quick / packed
# code GPU tests of the build, then one-process A/B (tools/ab_quick.py): head,
# the build with and without packed code rows, and the decode reading its
# weights from a few L2-resident tiles (timing probe).
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_quick_packed.py -m gpu -k "quick or hwc or decode or packed or sparse" -x -q --timeout 200 --timeout-method thread > $OUT/r05s3_quick_tests.log 2>&1 || { echo "quick tests failed"; tail -30 $OUT/r05s3_quick_tests.log; exit 1; }
tail -2 $OUT/r05s3_quick_tests.log
LSR_AB_LAYOUT=hwc timeout -k 10 300 python tools/ab_quick.py head:nopack=langsplatv2_amd/_build/var_head/liblsr.so new:nopack=langsplatv2_amd/liblsr.so new=langsplatv2_amd/liblsr.so l2read:nopack=langsplatv2_amd/_build/var_dl2read/liblsr.so > $OUT/r05s3_ab_packed.txt 2>&1 || { echo "ab_quick failed"; tail -20 $OUT/r05s3_ab_packed.txt; exit 1; }
cat $OUT/r05s3_ab_packed.txt
echo done
