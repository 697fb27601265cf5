#!/bin/bash
# Round-5 (session 4): M published by the tile count (the scatter launched while
# the column scan runs): GPU suite, then A/B against the previous build at cfg3 /
# cfg5 / cfg2, both orders.
set -u
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
PREV=langsplatv2_amd/_build/var_prev/liblsr.so
NEW=langsplatv2_amd/liblsr.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r05s4a_tests.log 2>&1
rc=$?; tail -3 $OUT/r05s4a_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/r05s4a_tests.log | head; exit 1; }
for C in 3 5 2; do
  LSR_CFG=$C timeout -k 10 300 python tools/ab.py prev=$PREV early=$NEW > $OUT/r05s4_ab_early_cfg$C.txt 2>&1 || { echo "ab cfg$C failed"; tail -20 $OUT/r05s4_ab_early_cfg$C.txt; exit 1; }
  LSR_CFG=$C timeout -k 10 300 python tools/ab.py early=$NEW prev=$PREV > $OUT/r05s4_ab_early_rev_cfg$C.txt 2>&1 || { echo "ab rev cfg$C failed"; exit 1; }
  echo "== cfg$C"; tail -4 $OUT/r05s4_ab_early_cfg$C.txt; tail -4 $OUT/r05s4_ab_early_rev_cfg$C.txt
done
